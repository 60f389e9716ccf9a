#!/bin/bash
# Round profile: full bench (with CPU baseline), all configs, rocprofv3 kernel-trace stats and the
# two HBM PMC passes (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).
# Usage (on the GPU box): bash tools/profile_round.sh <tag>      -> gpurun_out/prof_<tag>/...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=${1:-r01}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
B="python3 $ROOT/bench.py"
timeout -k 10 300 $B --steps 50 --warmup 5 > "$OUT/bench_b22.json" 2> "$OUT/bench_b22.err" || exit $?
cat "$OUT/bench_b22.json"
timeout -k 10 200 $B --steps 50 --warmup 5 --config c64 --no-cpu-baseline > "$OUT/bench_c64.json" 2>> "$OUT/bench.err" || exit $?
timeout -k 10 200 $B --steps 50 --warmup 5 --config d22 --no-cpu-baseline > "$OUT/bench_d22.json" 2>> "$OUT/bench.err" || exit $?
cat "$OUT/bench_c64.json" "$OUT/bench_d22.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 20 --warmup 3 --no-cpu-baseline > "$OUT/trace.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/pmc_fetch.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/pmc_write.log" 2>&1 || exit $?
# read requests by size (32/64/128 B): the byte count without FETCH_SIZE's fixed-size assumption
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum \
  -d "$OUT/pmc_rdreq" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/pmc_rdreq.log" 2>&1 || exit $?
find "$OUT" -name "*.csv" | sort
