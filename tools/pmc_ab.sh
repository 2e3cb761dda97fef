#!/bin/bash
# PMC A/B: default library vs $1 (FFM_LIB_PATH), same counter groups.
set -o pipefail
ALT=$1; OUT=${2:-gpurun_out/pmc_ab}
export TMPDIR=/tmp
mkdir -p "$OUT"
B="python3 bench.py --no-cpu --steps 60 --warmup 10"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_LDS SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d "$OUT/a/p$i" -o run -- $B > "$OUT/a$i.log" 2>&1 || exit 1
  FFM_LIB_PATH=$ALT timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d "$OUT/b/p$i" -o run -- $B > "$OUT/b$i.log" 2>&1 || exit 1
done
echo ab done
