#!/bin/bash
# GPU box: VALU / wait counters of the C4 batch kernel for two builds (tools/pmc.sh passes 1-3).
set -o pipefail
OUT=gpurun_out/c4pmc
mkdir -p $OUT
export TMPDIR=/tmp
for L in ab/libnopack.so ffm_amd/_lib/libffm_amd.so; do
  t=$(basename $L .so)
  i=0
  mkdir -p "$OUT/$t"
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_INSTS_SMEM" \
             "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32"; do
    i=$((i+1))
    FFM_LIB_PATH=$PWD/$L timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d "$OUT/$t/p$i" -o run -- python3 bench.py --no-cpu --config 4 --steps 60 --warmup 10 --repeats 1 > "$OUT/$t/p$i.log" 2>&1 || { echo "pass $t $i failed"; tail -5 "$OUT/$t/p$i.log"; exit 1; }
  done
done
echo done
