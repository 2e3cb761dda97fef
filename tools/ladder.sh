#!/bin/bash
# GPU box: time the C2 group kernel's skeleton ladder (tools/build_ladder.py) and the product,
# interleaved, 3 rounds.  Rungs 0-3 freeze the dynamics (every agent stays), so they run at
# --agents 17 (the product's steady-state live count, 16.9 per env) and at 32; the product runs
# the real workload (32 placed, 16.9 live at steady state).
# Usage: bash tools/ladder.sh <outdir> [bench args]
set -o pipefail
OUT=${1:-gpurun_out/ladder}; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
pick='import json,sys; d=json.loads(sys.stdin.read()); print(round(d.get("step_ms_events", d.get("kernel_ms_mean"))*1000,2), "us", round(d["value"]/1e9,2), "G")'
for r in 1 2 3; do
  for lib in lad/libffm_amd_lad0.so lad/libffm_amd_lad1.so lad/libffm_amd_lad2.so lad/libffm_amd_lad3.so; do
    for n in 17 32; do
      v=$(FFM_LIB_PATH=$PWD/$lib timeout -k 10 120 python3 bench.py --no-cpu --agents $n --burn-in 0 --steps 500 --warmup 20 "$@" 2>>"$OUT/err.log" | python3 -c "$pick") || exit 1
      echo "$(basename $lib .so) agents=$n $v"
    done
  done
  v=$(timeout -k 10 120 python3 bench.py --no-cpu --steps 500 --warmup 20 "$@" 2>>"$OUT/err.log" | python3 -c "$pick") || exit 1
  echo "product agents=32 $v"
done
