#!/bin/bash
# GPU box: smoke, the default bench line
# (the driver's flags), every learner / block config's bench line and a kernel trace of
# each config.  Usage: bash tools/final_check.sh <tag>
set -o pipefail
TAG=${1:-final}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
: # tests run separately (tools/gpu_tests.sh)

timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail -20 "$OUT/smoke.log"; exit 1; }
grep smoke "$OUT/smoke.log"
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err" || { echo "bench c2 failed"; tail -20 "$OUT/bench_c2.err"; exit 1; }
tail -1 "$OUT/bench_c2.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_c2" -o run -- python3 bench.py --no-cpu > "$OUT/trace_c2.log" 2>&1 || { echo "trace c2 failed"; exit 1; }
for c in 3 4 5; do
  timeout -k 10 400 python3 bench.py --config $c > "$OUT/bench_c$c.json" 2> "$OUT/bench_c$c.err" || { echo "bench c$c failed"; tail -20 "$OUT/bench_c$c.err"; exit 1; }
  tail -1 "$OUT/bench_c$c.json"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_c$c" -o run -- python3 bench.py --no-cpu --config $c > "$OUT/trace_c$c.log" 2>&1 || { echo "trace c$c failed"; exit 1; }
done
echo all-ok
