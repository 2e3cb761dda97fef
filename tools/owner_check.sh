#!/bin/bash
# GPU box: the tiled / owner-sharded learner tests, smoke, the C5 bench line and the
# 8-shard coupled C5 step under a kernel trace.  Usage: bash tools/owner_check.sh <tag>
set -o pipefail
TAG=${1:-owner}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_learn.py -x -v --timeout 300 --timeout-method thread -k "tiled or owner or tile_major or config5" > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail -20 "$OUT/smoke.log"; exit 1; }
grep smoke "$OUT/smoke.log"
timeout -k 10 400 python3 bench.py --config 5 > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err" || { echo "bench c5 failed"; tail -20 "$OUT/bench_c5.err"; exit 1; }
tail -1 "$OUT/bench_c5.json" | cut -c1-600
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_c5" -o run -- python3 bench.py --no-cpu --config 5 > "$OUT/trace_c5.log" 2>&1 || { echo "trace c5 failed"; exit 1; }
python3 tools/kstats.py "$OUT/trace_c5/run_kernel_trace.csv" 5 > "$OUT/kstats_c5.txt"; head -20 "$OUT/kstats_c5.txt"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace8" -o run -- python3 tools/c5_replicated_apply.py --shards 8 --steps 20 --warmup 10 --owner > "$OUT/own8.log" 2>&1 || { echo "owner8 failed"; tail -20 "$OUT/own8.log"; exit 1; }
grep ms_per "$OUT/own8.log"
python3 tools/kstats.py "$OUT/trace8/run_kernel_trace.csv" 0 > "$OUT/kstats_own8.txt"; head -30 "$OUT/kstats_own8.txt"
echo all-ok
