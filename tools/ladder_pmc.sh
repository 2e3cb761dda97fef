#!/bin/bash
# GPU box: one SQ counter pass per skeleton-ladder rung and the product (tools/build_ladder.py),
# for dynamic instruction counts per wave by rung.  Usage: bash tools/ladder_pmc.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/ladder_pmc}
export TMPDIR=/tmp
mkdir -p "$OUT"
CT="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
for lib in lad/libffm_amd_lad0.so lad/libffm_amd_lad1.so lad/libffm_amd_lad2.so lad/libffm_amd_lad3.so ffm_amd/_lib/libffm_amd.so; do
  t=$(basename $lib .so)
  FFM_LIB_PATH=$PWD/$lib timeout -s KILL 120 rocprofv3 --pmc $CT --output-format csv -d "$OUT/$t" -o run -- python3 bench.py --no-cpu --steps 60 --warmup 10 --repeats 1 --burn-in 300 --multi-step 1 > "$OUT/$t.log" 2>&1 || { echo "pmc $t failed"; tail -5 "$OUT/$t.log"; exit 1; }
  echo "pmc $t done"
done
