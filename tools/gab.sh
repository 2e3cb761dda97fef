#!/bin/bash
# GPU box: group-kernel parity under a library variant, then interleaved A/B of the C2 bench.
# Usage: bash tools/gab.sh <tag> "<variant libs for parity>" "<libs for ab>"
set -o pipefail
TAG=${1:-gab}; PAR=$2; AB=$3
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for lib in $PAR; do
  FFM_LIB_PATH=$PWD/$lib timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "config2 or param_points or group or sharding or ragged or capture or invariants" > "$OUT/par_$(basename $lib .so).log" 2>&1 || { echo "parity failed $lib"; tail -30 "$OUT/par_$(basename $lib .so).log"; exit 1; }
  echo "$lib: $(tail -1 $OUT/par_$(basename $lib .so).log)"
done
bash tools/ab.sh "$AB" --steps 500 --warmup 20 > "$OUT/ab.log" 2>&1 || { echo "ab failed"; tail -20 "$OUT/ab.log"; exit 1; }
cat "$OUT/ab.log"
