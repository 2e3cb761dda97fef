#!/bin/bash
# GPU box, round-5 measurement pass (after the GPU suite): every config's bench line and
# kernel trace, the PMC traffic of each config's dominant kernel, and the VALU counter
# passes of the C2 / C3 step kernels.  Usage: bash tools/final_r5.sh <tag>
set -o pipefail
TAG=${1:-final5}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for c in 2 3 4 5; do
  timeout -k 10 400 python3 bench.py --config $c > "$OUT/bench_c$c.json" 2> "$OUT/bench_c$c.err" || { echo "bench c$c failed"; tail -20 "$OUT/bench_c$c.err"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_c$c.json'));print('c$c', round(d['value']/1e9,3),'G', round(d['ms_per_step']*1e3,1),'us/step', 'frac', round(d['roofline']['frac'],3))"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_c$c" -o run -- python3 bench.py --no-cpu --config $c --repeats 1 > "$OUT/trace_c$c.log" 2>&1 || { echo "trace c$c failed"; exit 1; }
done
for c in 2 3 4 5; do
  bash tools/traffic.sh "$OUT/traffic_c$c" --config $c > "$OUT/traffic_c$c.log" 2>&1 || { tail "$OUT/traffic_c$c.log"; exit 1; }
  echo "traffic c$c done"
done
bash tools/pmc.sh "$OUT/pmc_c2" --config 2 > "$OUT/pmc_c2.log" 2>&1 || { tail "$OUT/pmc_c2.log"; exit 1; }
bash tools/pmc.sh "$OUT/pmc_c3" --config 3 > "$OUT/pmc_c3.log" 2>&1 || { tail "$OUT/pmc_c3.log"; exit 1; }
echo all-ok
