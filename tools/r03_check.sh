#!/bin/bash
# GPU box: a selection of GPU tests, smoke, and the default bench line (driver's flags).
# Usage: bash tools/r03_check.sh <tag> "<-k expression>"
set -o pipefail
TAG=${1:-sel}; K=${2:-}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail -30 "$OUT/smoke.log"; exit 1; }
cat "$OUT/smoke.log" | grep smoke
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 1; }
tail -1 "$OUT/bench.json"
