#!/bin/bash
# GPU box: learner counter passes (stall breakdown, instruction mix, LDS, instruction
# fetch) of one bench config's kernels.  Usage: bash tools/learn_pmc.sh <tag> <config 4|5> [bench args]
set -o pipefail
TAG=${1:-lpmc}; CFG=${2:-5}; shift 2 || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/avail.txt" 2>&1 || true
IC=$(grep -o "SQC_ICACHE_[A-Z_]*" "$OUT/avail.txt" | sort -u | head -4 | tr '\n' ' ')
echo "icache counters: $IC"
B="python3 bench.py --config $CFG --no-cpu --steps 20 --warmup 5 --repeats 1 $*"
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS" \
           "$IC"; do
  i=$((i+1))
  [ -z "${grp// }" ] && continue
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- $B > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
for k in learn_batch learn_phase_prep learn_phase_decide learn_phase_resolve learn_phase_learn learn_tile_h_kernel learn_tile_v_kernel; do
  echo "== $k"; python3 tools/pmc_summary.py "$OUT" "$k"
done > "$OUT/summary.txt"
cat "$OUT/summary.txt"
