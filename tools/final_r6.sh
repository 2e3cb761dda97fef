#!/bin/bash
# GPU box, round-6 measurement pass: every config's bench line and kernel trace, the PMC
# traffic of each config's dominant kernel, the SQ counter passes of the C2 / C3 step kernels,
# the C2 E-sweep (8,192-65,536 envs) with a kernel trace at 8,192, and the C4 two-rank
# rehearsal of the table exchange.  Usage: bash tools/final_r6.sh <tag> [parts: bench traffic pmc sweep rehearse]
set -o pipefail
TAG=${1:-final6}; shift
PARTS=${*:-bench traffic pmc sweep rehearse}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
has() { case " $PARTS " in *" $1 "*) return 0;; esac; return 1; }
if has bench; then
  for c in 2 3 4 5; do
    timeout -k 10 400 python3 bench.py --config $c > "$OUT/bench_c$c.json" 2> "$OUT/bench_c$c.err" || { echo "bench c$c failed"; tail -20 "$OUT/bench_c$c.err"; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/bench_c$c.json'));print('c$c', round(d['value']/1e9,3),'G', round(d['ms_per_step']*1e3,1),'us/step', 'frac', round(d['roofline']['frac'],3))"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_c$c" -o run -- python3 bench.py --no-cpu --config $c --repeats 1 > "$OUT/trace_c$c.log" 2>&1 || { echo "trace c$c failed"; exit 1; }
  done
fi
if has traffic; then
  for c in 2 3 4 5; do
    FFM_MEASURED="round 6" bash tools/traffic.sh "$OUT/traffic_c$c" --config $c > "$OUT/traffic_c$c.log" 2>&1 || { tail "$OUT/traffic_c$c.log"; exit 1; }
    echo "traffic c$c done"
  done
fi
if has pmc; then
  bash tools/pmc.sh "$OUT/pmc_c2" --config 2 > "$OUT/pmc_c2.log" 2>&1 || { tail "$OUT/pmc_c2.log"; exit 1; }
  bash tools/pmc.sh "$OUT/pmc_c3" --config 3 > "$OUT/pmc_c3.log" 2>&1 || { tail "$OUT/pmc_c3.log"; exit 1; }
  echo "pmc done"
fi
if has sweep; then
  bash tools/esweep.sh "$OUT/esweep" --multi-step 1 || exit 1
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_e8192" -o run -- python3 bench.py --no-cpu --envs 8192 --steps 500 --warmup 20 --multi-step 1 > "$OUT/trace_e8192.log" 2>&1 || { echo "trace e8192 failed"; exit 1; }
fi
if has rehearse; then
  bash tools/rehearse.sh "$TAG/rehearse_c4" 2 --config 4 --steps 60 --warmup 10 --repeats 2 || exit 1
fi
echo all-ok
