#!/bin/bash
# GPU box: one SQ counter pass per library (instruction mix A/B of kernel variants).
# Usage: bash tools/pmc_ab.sh <outdir> "<libs>" [bench args]
set -o pipefail
OUT=${1:-gpurun_out/pmc_ab}; LIBS=$2; shift 2
export TMPDIR=/tmp
mkdir -p "$OUT"
CT="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
for lib in $LIBS; do
  t=$(basename $lib .so)
  FFM_LIB_PATH=$PWD/$lib timeout -s KILL 120 rocprofv3 --pmc $CT --output-format csv -d "$OUT/$t" -o run -- python3 bench.py --no-cpu --steps 60 --warmup 10 --repeats 1 --burn-in 300 --multi-step 1 "$@" > "$OUT/$t.log" 2>&1 || { echo "pmc $t failed"; tail -5 "$OUT/$t.log"; exit 1; }
  python3 - "$OUT/$t/run_counter_collection.csv" "$t" <<'PY'
import csv, collections, statistics, sys
agg = collections.defaultdict(dict)
for r in csv.DictReader(open(sys.argv[1])):
    if "core_group_kernel" in r["Kernel_Name"]:
        agg[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
ds = sorted(agg, key=int)[-40:]
m = {c: statistics.median(agg[d][c] for d in ds) for c in agg[ds[0]]}
w = m["SQ_WAVES"]
print(sys.argv[2], "waves", int(w), " ".join(f"{k[3:]}/w={m[k]/w:.0f}" for k in m if k not in ("SQ_WAVES", "SQ_BUSY_CYCLES")),
      "busy/32", int(m["SQ_BUSY_CYCLES"] / 32))
PY
done
