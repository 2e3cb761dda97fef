#!/bin/bash
# GPU box: core parity suite (C1-C3 kernels incl. big maps, Moore, MT) with the in-tree
# library, then the C3 bench line and kernel trace.
set -o pipefail
OUT=gpurun_out/c3final
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 600 --timeout-method thread > $OUT/parity.log 2>&1 || { echo "parity failed"; tail -30 $OUT/parity.log; exit 1; }
tail -1 $OUT/parity.log
timeout -k 10 400 python3 bench.py --config 3 > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { echo "bench failed"; tail $OUT/bench_c3.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_c3.json'));print('c3', round(d['value']/1e9,3),'G', round(d['ms_per_step']*1e3,1),'us/step', 'frac', round(d['roofline']['frac'],3))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_c3" -o run -- python3 bench.py --no-cpu --config 3 --repeats 1 > "$OUT/trace_c3.log" 2>&1 || { echo "trace failed"; exit 1; }
echo ok
