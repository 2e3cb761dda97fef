#!/bin/bash
# GPU box: learner GPU tests, then interleaved A/B (C5 and C4) of library builds.
# Usage: bash tools/ab_learn.sh <tag> "<libs>" ["<pytest files>"]  (words, no -k expression)
set -o pipefail
OUT=gpurun_out/${1:-k}
LIBS=${2:-"build_ab/base.so ffm_amd/_lib/libffm_amd.so"}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest ${3:-tests/test_gpu_learn.py tests/test_gpu_dropin_learn.py} -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 700 bash tools/ab.sh "$LIBS" --config 5 --steps 30 --warmup 5 > "$OUT/ab_c5.log" 2>&1 || { echo "ab c5 failed"; cat "$OUT/ab_c5.log"; exit 1; }
cat "$OUT/ab_c5.log"
timeout -k 10 700 bash tools/ab.sh "$LIBS" --config 4 --steps 100 --warmup 30 > "$OUT/ab_c4.log" 2>&1 || { echo "ab c4 failed"; cat "$OUT/ab_c4.log"; exit 1; }
cat "$OUT/ab_c4.log"
