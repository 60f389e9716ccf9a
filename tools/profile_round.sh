#!/bin/bash
# Round profile: the bench lines of configs B, C, D (each with its CPU baseline), the PhysioNet
# geometry, the general kernels' geometries (g19, g38, p64l), the exact-division and folded sets, a rocprofv3 kernel-trace/stats run of config B, and the HBM PMC passes of configs B, C
# and D (read requests by size, WRITE_SIZE; FETCH_SIZE for B): every pass is its own rocprofv3 run.
# Usage (on the GPU box): bash tools/profile_round.sh <tag>      -> gpurun_out/prof_<tag>/...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=${1:-r03}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
B="python3 $ROOT/bench.py"
timeout -k 10 300 $B --steps 50 --warmup 5 > "$OUT/bench_b22.json" 2> "$OUT/bench_b22.err" || exit $?
cat "$OUT/bench_b22.json"
for cfg in c64 d22; do
  timeout -k 10 200 $B --steps 50 --warmup 5 --config $cfg --cpu-seconds 8 > "$OUT/bench_$cfg.json" 2>> "$OUT/bench.err" || exit $?
  cat "$OUT/bench_$cfg.json"
done
timeout -k 10 200 $B --steps 50 --warmup 5 --config p64 --no-cpu-baseline > "$OUT/bench_p64.json" 2>> "$OUT/bench.err" || exit $?
# the general (run-time-dimension) kernels: the channel-selected and PhysioNet geometries
for cfg in g19 g38 p64l; do
  timeout -k 10 200 $B --steps 50 --warmup 5 --config $cfg --cpu-seconds 8 > "$OUT/bench_$cfg.json" 2>> "$OUT/bench.err" || exit $?
  cat "$OUT/bench_$cfg.json"
done
# parameter sets off the float envelope: varying filters (exact division) and rails only (folded)
for pr in extreme rails; do
  timeout -k 10 200 $B --steps 50 --warmup 5 --params $pr --no-cpu-baseline > "$OUT/bench_b22_$pr.json" 2>> "$OUT/bench.err" || exit $?
  cat "$OUT/bench_b22_$pr.json"
done
# the other input layouts: channel-major int8 (B, C) and float32 (B)
for cl in b22:ct c64:ct b22:f32; do
  cfg=${cl%%:*}; lay=${cl#*:}
  timeout -k 10 200 $B --steps 50 --warmup 5 --config $cfg --layout $lay --no-cpu-baseline > "$OUT/bench_${cfg}_${lay}.json" 2>> "$OUT/bench.err" || exit $?
  cat "$OUT/bench_${cfg}_${lay}.json"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 20 --warmup 3 --no-cpu-baseline > "$OUT/trace.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_g19" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --config g19 --steps 20 --warmup 3 --no-cpu-baseline > "$OUT/trace_g19.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/pmc_fetch.log" 2>&1 || exit $?
for cl in b22 c64 d22 b22:ct c64:ct b22:f32 g19 g38 p64l; do
  cfg=${cl%%:*}; lay=tc; [ "$cl" != "$cfg" ] && lay=${cl#*:}
  key=$cfg; [ $lay != tc ] && key=${cfg}_$lay
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write_$key" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --config $cfg --layout $lay > "$OUT/pmc_write_$key.log" 2>&1 || exit $?
  # read requests by size (32/64/128 B): the byte count without FETCH_SIZE's fixed-size assumption
  timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum \
    -d "$OUT/pmc_rdreq_$key" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --config $cfg --layout $lay > "$OUT/pmc_rdreq_$key.log" 2>&1 || exit $?
done
find "$OUT" -name "*.csv" | sort
