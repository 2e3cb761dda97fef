#!/bin/bash
# GPU box: per-phase wall-clock stamps of the learner batch kernel (FFM_LSTAMP build at
# ab/libS.so) for configs 4 and 5.  Usage: bash tools/stamps_c45.sh <tag>
set -o pipefail
TAG=${1:-stamps}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for c in ${CONFIGS:-4 5}; do
  FFM_LIB_PATH=$PWD/ab/libS.so timeout -k 10 200 python3 bench.py --no-cpu --config $c --steps 6 --warmup 40 --repeats 1 > "$OUT/stamps_c$c.log" 2>&1 || { echo "stamps c$c failed"; tail -5 "$OUT/stamps_c$c.log"; exit 1; }
  grep LSTAMP "$OUT/stamps_c$c.log" | tail -8
done
