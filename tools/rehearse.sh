#!/bin/bash
# GPU box: the bench's N-rank path rehearsed on one GPU (gloo, FFM_BENCH_REHEARSE=1).
# Usage: bash tools/rehearse.sh <tag> <nproc> [bench args]
set -o pipefail
TAG=${1:-rehearse}; NP=${2:-2}; shift 2 || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp FFM_BENCH_REHEARSE=1
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $NP --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus $NP --no-cpu "$@" > "$OUT/bench.log" 2>&1 || { echo "rehearsal failed"; tail -30 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log"
