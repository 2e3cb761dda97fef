#!/bin/bash
# Instruction counts + time per ablation library (one PMC pass each).
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc_abl}
mkdir -p "$OUT"
for f in build_abl/libffm_amd_abl*.so; do
  tag=$(basename $f .so)
  FFM_LIB_PATH=$PWD/$f timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_ANY --output-format csv -d "$OUT/$tag" -o run -- python3 bench.py --no-cpu --steps 40 --warmup 10 > "$OUT/$tag.log" 2>&1 || exit 1
  t=$(FFM_LIB_PATH=$PWD/$f timeout -k 10 120 python3 bench.py --no-cpu --steps 200 --warmup 20 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['kernel_ms_mean']*1000,1))")
  echo "$tag $t us"
done
