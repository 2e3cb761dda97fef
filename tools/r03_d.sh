#!/bin/bash
# GPU box: new-feature parity tests, smoke, C2 and C5 A/B (base vs new), C5 kernel trace.
# Test failures are reported but do not stop the measurements; a timeout or crash does.
set -o pipefail
OUT=gpurun_out/${1:-d}; K=${2:-"tiled or config5 or trajectory_capture or async_records or moore or dropin or group or config2 or param_points or multi_step"}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu --maxfail 10 -v --timeout 600 --timeout-method thread -k "$K" > "$OUT/pytest.log" 2>&1
rc=$?
tail -4 "$OUT/pytest.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc: stop"; exit 1; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail -30 "$OUT/smoke.log"; exit 1; }
grep smoke "$OUT/smoke.log"
timeout -k 10 600 bash tools/ab.sh "build_ab/libbase.so build_ab/libnew.so" --steps 300 --warmup 20 --multi-step 0 > "$OUT/ab_c2.log" 2>&1 || { echo "ab failed"; tail -20 "$OUT/ab_c2.log"; exit 1; }
cat "$OUT/ab_c2.log"
timeout -k 10 600 bash tools/ab.sh "build_ab/libbase.so build_ab/libnew.so build_ab/liblabl1.so" --config 5 --steps 30 --warmup 5 > "$OUT/ab_c5.log" 2>&1 || { echo "ab c5 failed"; tail -20 "$OUT/ab_c5.log"; exit 1; }
cat "$OUT/ab_c5.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_c5" -o run -- python3 bench.py --no-cpu --config 5 --steps 30 --warmup 5 --repeats 1 > "$OUT/trace_c5.log" 2>&1 || { echo "trace c5 failed"; exit 1; }
cut -d, -f1-4 "$OUT/trace_c5/run_kernel_stats.csv"
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 1; }
tail -1 "$OUT/bench.json"
