#!/bin/bash
# GPU box: the block-kernel parity tests (C3 shapes, big maps, Moore, MT replays), then an
# interleaved A/B of the C3 bench.  Usage: bash tools/c3ab.sh <tag> "<libs>"
set -o pipefail
TAG=${1:-c3ab}; AB=$2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 600 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
bash tools/ab.sh "$AB" --config 3 --steps 1500 --repeats 3 > "$OUT/ab.log" 2>&1 || { echo "ab failed"; tail -20 "$OUT/ab.log"; exit 1; }
cat "$OUT/ab.log"
