#!/bin/bash
# GPU box: the C2 step at the per-GPU env counts of a strong-scaling reading of the headline
# (64k global envs over 8/4/2/1 GPUs), one GPU, product library.  Prints one JSON per E.
set -o pipefail
OUT=${1:-gpurun_out/esweep}; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
for E in 8192 16384 32768 65536; do
  timeout -k 10 180 python3 bench.py --no-cpu --envs $E --steps 500 --warmup 20 "$@" > "$OUT/e$E.json" 2>>"$OUT/err.log" || exit 1
  python3 -c "import json; d=json.load(open('$OUT/e$E.json')); print($E, round(d['kernel_ms_mean']*1000,2), 'us', round(d['value']/1e9,2), 'G')"
done
