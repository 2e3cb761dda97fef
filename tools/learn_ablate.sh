#!/bin/bash
# Diagnostic: time one learning step (HIP events) for each build_abl/libffm_amd_labl*.so.
# Usage (GPU box): bash tools/learn_ablate.sh [bench args...]
set -o pipefail
export TMPDIR=/tmp
for f in build_abl/libffm_amd_labl*.so; do
  tag=$(basename $f .so)
  v=$(FFM_LIB_PATH=$PWD/$f timeout -k 10 120 python3 bench.py --no-cpu "$@" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['step_ms_events']*1000,1), 'us')") || exit 1
  echo "$tag $v"
done
