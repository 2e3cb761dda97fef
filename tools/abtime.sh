#!/bin/bash
# Diagnostic A/B: kernel time of each library given (FFM_LIB_PATH), interleaved, 3 rounds.
# Usage: bash tools/abtime.sh lib1.so lib2.so[,VAR=value] ...
set -o pipefail
export TMPDIR=/tmp
for round in 1 2 3; do
  for spec in "$@"; do
    f=${spec%%,*}; envs=""
    [ "$spec" != "$f" ] && envs=${spec#*,}
    v=$(env $envs FFM_LIB_PATH=$PWD/$f timeout -k 10 120 python3 bench.py --no-cpu --steps 300 --warmup 30 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['kernel_ms_mean']*1000,2), 'us', round(d['value']/1e9,2), 'G')") || exit 1
    echo "r$round $(basename $f .so) $envs $v"
  done
done
