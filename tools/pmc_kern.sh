#!/bin/bash
# PMC instruction/wait counters for the default kernel and for extra bench args (e.g. --envs-per-block -1).
# Usage: bash tools/pmc_kern.sh <outdir> "<bench args A>" "<bench args B>" ...
set -o pipefail
OUT=$1; shift
export TMPDIR=/tmp
mkdir -p "$OUT"
k=0
for args in "$@"; do
  k=$((k+1)); i=0; mkdir -p "$OUT/k$k"
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM SQ_BUSY_CYCLES SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_SCA"; do
    i=$((i+1))
    timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d "$OUT/k$k/p$i" -o run -- python3 bench.py --no-cpu --steps 60 --warmup 10 $args > "$OUT/k$k/p$i.log" 2>&1 || { echo "pass failed $k $i"; exit 1; }
  done
done
echo pmc done
