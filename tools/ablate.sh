#!/bin/bash
# Diagnostic: time the step kernel for each library in build_abl/ (see tools/build_ablate.py).
set -o pipefail
export TMPDIR=/tmp
for f in build_abl/libffm_amd_*.so; do
  tag=$(basename $f .so)
  v=$(FFM_LIB_PATH=$PWD/$f timeout -k 10 120 python3 bench.py --no-cpu --steps 200 --warmup 20 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['kernel_ms_mean']*1000,1), 'us')") || exit 1
  echo "$tag $v"
done
