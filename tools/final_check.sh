#!/bin/bash
# GPU box, end of a work block: the full GPU suite and smoke, the default bench
# line, every learner / block config's bench line and a kernel trace of each.
# Usage: bash tools/final_check.sh <tag>
set -o pipefail
TAG=${1:-final}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/gpu_check.sh "$TAG" || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
for c in 3 4 5; do
  timeout -k 10 300 python3 bench.py --config $c > "$OUT/bench_c$c.json" 2> "$OUT/bench_c$c.err" || { echo "bench c$c failed"; tail -20 "$OUT/bench_c$c.err"; exit 1; }
  tail -1 "$OUT/bench_c$c.json"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_c$c" -o run -- python3 bench.py --no-cpu --config $c > "$OUT/trace_c$c.log" 2>&1 || { echo "trace c$c failed"; exit 1; }
done
echo all-ok
