#!/bin/bash
# GPU box: C5 learner phase stamps (FFM_LSTAMP build at build_ab/libS.so) and kernel stats.
# Usage: bash tools/c5_profile.sh <tag> [bench args]
set -o pipefail
TAG=${1:-c5prof}; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
FFM_LIB_PATH=$PWD/build_ab/libS.so timeout -k 10 120 python3 bench.py --no-cpu --config 5 --steps 4 --warmup 2 --repeats 1 "$@" > "$OUT/stamps.log" 2>&1 || { echo "stamps failed"; tail -5 "$OUT/stamps.log"; exit 1; }
grep LSTAMP "$OUT/stamps.log" | tail -6
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 bench.py --no-cpu --config 5 --steps 30 --warmup 5 --repeats 1 "$@" > "$OUT/trace.log" 2>&1 || { echo "trace failed"; exit 1; }
cut -d, -f1-4 "$OUT/trace/run_kernel_stats.csv"
