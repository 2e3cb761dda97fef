#!/bin/bash
# GPU box: tiled-step parity, C5 A/B and traces (tiled vs accumulator path), C2 A/B.
set -o pipefail
OUT=gpurun_out/${1:-f}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail 5 -v --timeout 600 --timeout-method thread -k "tiled or config5 or trajectory_capture" > "$OUT/pytest.log" 2>&1
rc=$?
tail -4 "$OUT/pytest.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc: stop"; exit 1; fi
timeout -k 10 900 bash tools/abtree.sh "--config 5 --steps 30 --warmup 5" FFM_TILED=0 > "$OUT/ab_c5.log" 2>&1 || { echo "ab c5 failed"; tail -20 "$OUT/ab_c5.log"; exit 1; }
cat "$OUT/ab_c5.log"
for t in 1 0; do
  FFM_TILED=$t timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_c5_t$t" -o run -- python3 bench.py --no-cpu --config 5 --steps 30 --warmup 5 --repeats 1 > "$OUT/trace_c5_t$t.log" 2>&1 || { echo "trace c5 failed"; exit 1; }
  python3 tools/kstats.py "$OUT/trace_c5_t$t/run_kernel_trace.csv" 10
done
timeout -k 10 900 bash tools/abtree.sh "--steps 300 --warmup 400 --multi-step 0" > "$OUT/ab_c2.log" 2>&1 || { echo "ab c2 failed"; tail -20 "$OUT/ab_c2.log"; exit 1; }
cat "$OUT/ab_c2.log"
