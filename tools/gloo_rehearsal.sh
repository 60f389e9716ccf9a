#!/bin/bash
# Rehearsal of bench.py's multi-rank branch (config E's static split) on a one-GPU box: N ranks
# under torch.distributed.run (bench.py coordinates over gloo only, no RCCL), every rank on device
# 0 with its own 65,536-trial shard.  The ranks share one GPU, so the line shows the branch works
# (per-rank record, world size, backend, max-over-ranks timing), not scaling.
# usage (on the GPU box): bash tools/gloo_rehearsal.sh [N] [tag]   -> gpurun_out/gloo_<tag>_n<N>.json
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
N=${1:-2}
TAG=${2:-r03}
mkdir -p gpurun_out
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus "$N" --steps 20 --warmup 3 \
  > "gpurun_out/gloo_${TAG}_n${N}.json" 2> "gpurun_out/gloo_${TAG}_n${N}.err"
rc=$?
cat "gpurun_out/gloo_${TAG}_n${N}.json"
exit $rc
