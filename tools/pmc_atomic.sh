#!/bin/bash
# Memory-side atomic requests and wait counters of the learner kernels (one rocprofv3
# run per counter group, kernel trace only).  Usage: bash tools/pmc_atomic.sh <outdir> [bench args]
set -o pipefail
OUT=${1:-gpurun_out/pmcat}; shift || true
export TMPDIR=/tmp
mkdir -p "$OUT"
B="python3 bench.py --no-cpu --steps 60 --warmup 10 --repeats 1 $*"
i=0
for grp in "TCC_EA0_ATOMIC_sum" "GRBM_GUI_ACTIVE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- $B > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
echo pmc done
