#!/bin/bash
# GPU box: tiled-step parity, C5 A/B (round-start tree, current, FFM_TILED=0), a C5 trace.
set -o pipefail
OUT=gpurun_out/${1:-g}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail 5 -v --timeout 600 --timeout-method thread -k "tiled or config5" > "$OUT/pytest.log" 2>&1
rc=$?
tail -4 "$OUT/pytest.log"
if [ $rc -ne 0 ]; then echo "pytest rc $rc: stop"; exit 1; fi
timeout -k 10 900 bash tools/abtree.sh "--config 5 --steps 30 --warmup 5" FFM_TILED=0 > "$OUT/ab_c5.log" 2>&1 || { echo "ab c5 failed"; tail -20 "$OUT/ab_c5.log"; exit 1; }
cat "$OUT/ab_c5.log"
for sd in 1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_c5_s$sd" -o run -- python3 bench.py --no-cpu --config 5 --steps 30 --warmup 5 --repeats 1 > "$OUT/trace_c5_s$sd.log" 2>&1 || { echo "trace c5 failed"; exit 1; }
  python3 tools/kstats.py "$OUT/trace_c5_s$sd/run_kernel_trace.csv" 10
done
