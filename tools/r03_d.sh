#!/bin/bash
# GPU box: C2 / C5 / C4 A/B against the round-start tree, C5 kernel trace, default bench line.
set -o pipefail
OUT=gpurun_out/${1:-d}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 bash tools/abtree.sh "--steps 300 --warmup 400 --multi-step 0" > "$OUT/ab_c2.log" 2>&1 || { echo "ab c2 failed"; tail -20 "$OUT/ab_c2.log"; exit 1; }
cat "$OUT/ab_c2.log"
timeout -k 10 900 bash tools/abtree.sh "--config 5 --steps 30 --warmup 5" FFM_TILED=0 > "$OUT/ab_c5.log" 2>&1 || { echo "ab c5 failed"; tail -20 "$OUT/ab_c5.log"; exit 1; }
cat "$OUT/ab_c5.log"
timeout -k 10 600 bash tools/ab.sh "build_ab/libcur.so build_ab/libvearly.so" --config 4 --steps 100 --warmup 30 > "$OUT/ab_c4.log" 2>&1 || { echo "ab c4 failed"; tail -20 "$OUT/ab_c4.log"; exit 1; }
cat "$OUT/ab_c4.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_c5" -o run -- python3 bench.py --no-cpu --config 5 --steps 30 --warmup 5 --repeats 1 > "$OUT/trace_c5.log" 2>&1 || { echo "trace c5 failed"; exit 1; }
cut -d, -f1-4 "$OUT/trace_c5/run_kernel_stats.csv"
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 1; }
tail -1 "$OUT/bench.json"
