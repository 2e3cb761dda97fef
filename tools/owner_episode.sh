#!/bin/bash
# GPU box: the owner-sharded learner tests, then the 8-shard coupled C5 step over a whole
# episode (300-step burn-in, 300 timed steps) under a kernel trace, per-kernel means over the
# timed episode only.  Usage: bash tools/owner_episode.sh <tag> [pytest -k] [ab libs]
set -o pipefail
TAG=${1:-owner}; K=${2:-"owner"}; AB=$3
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "$K" != "-" ]; then
  timeout -k 10 900 python -u -m pytest tests/test_gpu_learn.py -x -v --timeout 900 --timeout-method thread -k "$K" > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
  tail -1 "$OUT/pytest.log"
fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace8" -o run -- python3 tools/c5_replicated_apply.py --shards 8 --steps 300 --warmup 300 --owner > "$OUT/own8.log" 2>&1 || { echo "owner8 failed"; tail -20 "$OUT/own8.log"; exit 1; }
grep ms_per "$OUT/own8.log"
python3 tools/kstats.py "$OUT/trace8/run_kernel_trace.csv" 2400 > "$OUT/kstats_own8.txt"; head -24 "$OUT/kstats_own8.txt"
if [ -n "$AB" ]; then bash tools/ab.sh "$AB" --config 5 > "$OUT/ab.log" 2>&1 || { echo "ab failed"; tail "$OUT/ab.log"; exit 1; }; cat "$OUT/ab.log"; fi
echo all-ok
