#!/bin/bash
# GPU box: C5 learner counter passes (stall breakdown, instruction fetch, LDS) of the
# batch and tile kernels.  Usage: bash tools/c5_pmc.sh <tag> [extra bench args]
set -o pipefail
TAG=${1:-c5pmc}; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/avail.txt" 2>&1 || true
IC=$(grep -o "SQC_ICACHE_[A-Z_]*\|SQ_IFETCH[A-Z_]*\|SQ_WAIT_INST_ANY\b" "$OUT/avail.txt" | sort -u | grep -v "SQ_WAIT_INST_ANY" | head -4 | tr '\n' ' ')
echo "icache counters: $IC"
B="python3 bench.py --config 5 --no-cpu --steps 20 --warmup 5 --repeats 1 $*"
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS" \
           "$IC"; do
  i=$((i+1))
  [ -z "${grp// }" ] && continue
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- $B > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
for k in learn_batch learn_tile_h_kernel learn_tile_v_kernel; do
  echo "== $k"; python3 tools/pmc_summary.py "$OUT" "$k"
done > "$OUT/summary.txt"
cat "$OUT/summary.txt"
