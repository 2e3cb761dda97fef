#!/bin/bash
# GPU box: C5 kernel traces (mean per kernel past warmup) under library / env variants.
# Usage: bash tools/c5_trace.sh <tag> "<lib[@VAR=val]> ..." [bench args]
set -o pipefail
TAG=${1:-c5tr}; LIBS=$2; shift 2 || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for f in $LIBS; do
  i=$((i+1))
  lib=${f%%@*}; kv=""; [ "$lib" != "$f" ] && kv=${f#*@}
  env $kv FFM_LIB_PATH=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/t$i" -o run -- python3 bench.py --no-cpu --config 5 --steps 30 --warmup 5 --repeats 1 "$@" > "$OUT/t$i.log" 2>&1 || { echo "trace $f failed"; tail -5 "$OUT/t$i.log"; exit 1; }
  echo "== $f"
  python3 tools/kstats.py "$OUT/t$i/run_kernel_trace.csv" 20 | head -16
done
