#!/bin/bash
# runs the phase probes (tools/probebin_* built with -DMIB_STAMPS) on config B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
python -c "import sys; sys.path.insert(0,'mi-bminet_amd'); from mibminet.params import ParamSet; open('gpurun_out/p.blob','wb').write(ParamSet.synthetic(1).to_blob()); open('gpurun_out/pc.blob','wb').write(ParamSet.synthetic(1, C=64, T=1000).to_blob())" || exit 1
for p in tools/probebin_*; do
  [ -x "$p" ] || continue
  echo "=== $p (config B)"
  timeout -k 10 120 $p gpurun_out/p.blob 65536 10 || exit $?
done
