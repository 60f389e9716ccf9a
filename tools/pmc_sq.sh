#!/bin/bash
# SQ / TCC counter passes of the bench kernel (each pass its own rocprofv3 run, counters only).
# usage: bash tools/pmc_sq.sh <tag> [bench args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=${1:-sq}; shift
OUT=$ROOT/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() {  # name counters...
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" -d "$OUT/$name" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline "${BENCH_EXTRA[@]}" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "pass $name rc=$rc"
  # a bad counter name fails the pass only; a timeout, abort or crash ends the script
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
  return 0
}
BENCH_EXTRA=("$@")
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
run sq2 SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_MISC
run sq3 SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT
run tcc FETCH_SIZE
run tcc2 TCC_HIT_sum TCC_MISS_sum
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
tot = collections.defaultdict(list)
for f in sorted(glob.glob(out + "/*/run_counter_collection.csv")):
    for row in csv.DictReader(open(f)):
        if "k_forward" in row["Kernel_Name"]:
            tot[row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, v in sorted(tot.items()):
    print(f"{k:28s} {sum(v[1:])/max(1,len(v)-1):16.1f}  (per dispatch, {len(v)} dispatches)")
PY
