#!/bin/bash
# GPU box: a selection of GPU tests (pytest -k expression), output under gpurun_out/<tag>.
# Usage: bash tools/gpu_tests.sh <tag> "<-k expression>"
set -o pipefail
TAG=${1:-sel}; K=${2:-}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$K" > "$OUT/pytest.log" 2>&1
rc=$?
tail -25 "$OUT/pytest.log"
exit $rc
