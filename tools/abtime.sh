#!/bin/bash
# Diagnostic A/B: kernel time of each variant, interleaved, 3 rounds.
# Spec: lib.so[,VAR=value...][@bench_args_with_underscores_for_spaces]
# Usage: bash tools/abtime.sh ffm_amd/_lib/libffm_amd.so lib2.so,FFM_WAVE_BLOCKS=1024 lib.so@--envs-per-block_-1
set -o pipefail
export TMPDIR=/tmp
for round in 1 2 3; do
  for spec in "$@"; do
    bargs=""
    case "$spec" in *@*) bargs=$(echo "${spec#*@}" | tr '_' ' '); spec=${spec%%@*};; esac
    f=${spec%%,*}; envs=""
    [ "$spec" != "$f" ] && envs=$(echo "${spec#*,}" | tr ',' ' ')
    v=$(env $envs FFM_LIB_PATH=$PWD/$f timeout -k 10 120 python3 bench.py --no-cpu --steps 300 --warmup 30 $bargs | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['kernel_ms_mean']*1000,2), 'us', round(d['value']/1e9,2), 'G')") || exit 1
    echo "r$round $(basename $f .so) $envs $bargs $v"
  done
done
