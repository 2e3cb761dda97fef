#!/bin/bash
# GPU box: Philox parity tests (pytest -k expression), then C2 bench of the group
# kernel (auto) beside the lane kernel (-2), then a kernel trace of the default bench.
# Usage: bash tools/group_check.sh <tag> [pytest -k expression]
set -o pipefail
TAG=${1:-grp}; K=${2:-philox}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "$K" > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for r in 1 2; do for epb in 0 -2; do
  timeout -k 10 300 python bench.py --no-cpu --repeats 3 --envs-per-block $epb > "$OUT/bench_epb$epb.json" 2> "$OUT/bench_epb$epb.err" || { echo "bench $epb failed"; tail -20 "$OUT/bench_epb$epb.err"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_epb$epb.json'));print('epb $epb', round(d['value']/1e9,2),'G', round(d['kernel_ms_mean']*1e3,2),'us', d['repeats']['values'])"
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 bench.py --no-cpu --steps 200 --warmup 20 --repeats 1 > "$OUT/trace.log" 2>&1 || { echo "trace failed"; exit 1; }
cat "$OUT/trace/run_kernel_stats.csv"
