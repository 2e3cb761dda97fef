#!/bin/bash
# GPU box: tiled / owner learner tests, then interleaved A/B of the C5 bench.
# Usage: bash tools/c5ab.sh <tag> "<libs for ab>" [pytest -k]
set -o pipefail
TAG=${1:-c5ab}; AB=$2; K=${3:-"tiled or owner or tile_major or config5"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_learn.py -x -q --timeout 600 --timeout-method thread -k "$K" > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
bash tools/ab.sh "$AB" --config 5 > "$OUT/ab.log" 2>&1 || { echo "ab failed"; tail -20 "$OUT/ab.log"; exit 1; }
cat "$OUT/ab.log"
