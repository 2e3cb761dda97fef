#!/bin/bash
# GPU box: tiled / stencil parity, interleaved C5 A/B of library builds, C5 kernel trace.
# Usage: bash tools/r03_j.sh <tag> "<libs>" ["<-k expression>"]
set -o pipefail
OUT=gpurun_out/${1:-j}
LIBS=${2:-"build_ab/head.so ffm_amd/_lib/libffm_amd.so"}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "${3:-tiled or config5 or column_stencil}" > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 700 bash tools/ab.sh "$LIBS" --config 5 --steps 30 --warmup 5 > "$OUT/ab_c5.log" 2>&1 || { echo "ab failed"; cat "$OUT/ab_c5.log"; exit 1; }
cat "$OUT/ab_c5.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_c5" -o run -- python3 bench.py --no-cpu --config 5 --steps 30 --warmup 5 --repeats 1 > "$OUT/trace_c5.log" 2>&1 || { echo "trace failed"; tail -20 "$OUT/trace_c5.log"; exit 1; }
python3 tools/kstats.py "$OUT/trace_c5/run_kernel_trace.csv" 10
