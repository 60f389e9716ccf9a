#!/bin/bash
# GPU round: parity tests, then a short bench. Stops at the first crash/timeout.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu -x ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -40 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 3 ${BENCH_ARGS:---no-cpu-baseline} > gpurun_out/bench.log 2>&1
rc2=$?
cat gpurun_out/bench.log
exit $(( rc != 0 ? rc : rc2 ))
