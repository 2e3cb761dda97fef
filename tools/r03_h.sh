#!/bin/bash
# GPU box: tiled-step parity, interleaved C5 A/B of build_ab/head.so against the current
# library, and a steady-state C5 kernel trace.
set -o pipefail
OUT=gpurun_out/${1:-h}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "tiled or config5 or learner_philox_large" > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 600 bash tools/ab.sh "build_ab/head.so ffm_amd/_lib/libffm_amd.so" --config 5 --steps 30 --warmup 5 > "$OUT/ab_c5.log" 2>&1 || { echo "ab failed"; cat "$OUT/ab_c5.log"; exit 1; }
cat "$OUT/ab_c5.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_c5" -o run -- python3 bench.py --no-cpu --config 5 --steps 30 --warmup 5 --repeats 1 --burn-in 0 > "$OUT/trace_c5.log" 2>&1 || { echo "trace failed"; tail -20 "$OUT/trace_c5.log"; exit 1; }
python3 tools/kstats.py "$OUT/trace_c5/run_kernel_trace.csv" 10
