#!/bin/bash
# GPU box: parity tests, then the bench, then a kernel trace.  Stops at the first failure.
# Usage: bash tools/gpu_check.sh <tag> [extra bench args]
set -o pipefail
TAG=${1:-run}; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 300 python bench.py "$@" > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -30 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 bench.py --no-cpu --steps 200 --warmup 20 "$@" > "$OUT/trace.log" 2>&1 || { echo "trace failed"; exit 1; }
cat "$OUT/trace/run_kernel_stats.csv"
