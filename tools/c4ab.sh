#!/bin/bash
# GPU box: actor_only (config-4 model) learner parity, then interleaved A/B of the C4 bench.
# Usage: bash tools/c4ab.sh <tag> "<libs for ab>"
set -o pipefail
TAG=${1:-c4ab}; AB=$2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_learn.py -x -q --timeout 600 --timeout-method thread -k "actor_only or config4" > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
bash tools/ab.sh "$AB" --config 4 > "$OUT/ab.log" 2>&1 || { echo "ab failed"; tail -20 "$OUT/ab.log"; exit 1; }
cat "$OUT/ab.log"
