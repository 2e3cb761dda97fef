#!/bin/bash
# GPU box: C4 kernel traces (mean per kernel past warmup) under library / env variants.
# Usage: bash tools/c4_trace.sh <tag> "<lib[@VAR=val]> ..."
set -o pipefail
TAG=${1:-c4tr}; LIBS=$2; shift 2 || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for f in $LIBS; do
  i=$((i+1))
  lib=${f%%@*}; kv=""; [ "$lib" != "$f" ] && kv=${f#*@}
  env $kv FFM_LIB_PATH=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/t$i" -o run -- python3 bench.py --no-cpu --config 4 --steps 100 --warmup 30 --repeats 1 "$@" > "$OUT/t$i.log" 2>&1 || { echo "trace $f failed"; tail -5 "$OUT/t$i.log"; exit 1; }
  echo "== $f"
  python3 tools/kstats.py "$OUT/t$i/run_kernel_trace.csv" 40 | head -8
done
