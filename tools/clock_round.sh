#!/bin/bash
# In-kernel clock of the shipped kernel and its ablations (tools/build_clock.sh builds them):
# random and all-zero input for the shipped build, random input for the others.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
python -c "import sys; sys.path.insert(0,'mi-bminet_amd'); from mibminet.params import ParamSet; open('gpurun_out/p.blob','wb').write(ParamSet.synthetic(1).to_blob())" || exit 1
for b in tools/clkbin_*; do
  [ -x "$b" ] || continue
  echo "=== $b"
  timeout -k 10 60 $b gpurun_out/p.blob 0 ${WARM:-2.5} ${ITERS:-300} || exit $?
  if [ "$(basename $b)" = clkbin_base ]; then timeout -k 10 60 $b gpurun_out/p.blob 1 ${WARM:-2.5} ${ITERS:-300} || exit $?; fi
done
