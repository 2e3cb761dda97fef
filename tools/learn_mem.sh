#!/bin/bash
# GPU box: memory-side counters of one learner config's kernels (HBM bytes, L2 hit rate,
# L1->L2 request latency, TA stalls), one rocprofv3 pass per group.
# Usage: bash tools/learn_mem.sh <tag> <config> [bench args]
set -o pipefail
TAG=${1:-lmem}; CFG=${2:-5}; shift 2 || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
B="python3 bench.py --config $CFG --no-cpu --steps 20 --warmup 5 --repeats 1 $*"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
           "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum" \
           "TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_WAVE_CYCLES SQ_WAVES"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- $B > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
for k in learn_batch learn_phase_prep learn_phase_decide learn_phase_resolve learn_phase_learn learn_tile_h_kernel learn_tile_v_kernel learn_stencil; do
  echo "== $k"; python3 tools/pmc_summary.py "$OUT" "$k"
done > "$OUT/summary.txt"
cat "$OUT/summary.txt"
