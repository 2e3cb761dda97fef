#!/bin/bash
# A/B timing of one library under different values of an environment variable,
# interleaved (GPU box):  bash tools/ab_env.sh VAR "v1 v2 ..." [bench args...]
set -o pipefail
export TMPDIR=/tmp
VAR=$1; VALS=$2; shift 2
for r in 1 2 3; do
  for v in $VALS; do
    out=$(env "$VAR=$v" timeout -k 10 180 python3 bench.py --no-cpu "$@" 2>/dev/null) || exit 1
    echo "$VAR=$v $(echo "$out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['step_ms_events']*1000,1), 'us', round(d['value']/1e9,3), 'G', 'live', round(d['mean_live_agents_per_env_step'],2))")"
  done
done
