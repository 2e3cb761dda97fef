#!/bin/bash
# HBM traffic of the step kernel: FETCH_SIZE and WRITE_SIZE in separate rocprofv3
# passes (kernel trace only), then <outdir>/traffic.json (copy to profiles/traffic_<H>x<W>_A<A>_E<E>.json).
# Usage: bash tools/traffic.sh <outdir> [bench args]
set -o pipefail
OUT=${1:-gpurun_out/traffic}; shift || true
export TMPDIR=/tmp
mkdir -p "$OUT"
B="python3 bench.py --no-cpu --steps 60 --warmup 10 $*"
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- $B > "$OUT/fetch.log" 2>&1 || { echo "fetch pass failed"; tail -5 "$OUT/fetch.log"; exit 1; }
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- $B > "$OUT/write.log" 2>&1 || { echo "write pass failed"; tail -5 "$OUT/write.log"; exit 1; }
python3 tools/traffic_json.py "$OUT" $*
