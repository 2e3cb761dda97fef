#!/bin/bash
# Interleaved A/B of the round-start tree (build_ab/base_tree: its own bench.py, Python
# binding and library) against the current tree, plus env-var variants of the current one.
#   bash tools/abtree.sh "<bench args>" ["VAR=val" ...]
set -o pipefail
export TMPDIR=/tmp
ARGS=$1; shift
pick='import json,sys; d=json.loads(sys.stdin.read()); print(round(d.get("step_ms_events", d.get("kernel_ms_mean"))*1000,1), "us", round(d["value"]/1e9,3), "G", round(d.get("mean_live_agents_per_env_step",0),2), "live")'
for r in 1 2 3; do
  v=$( (cd build_ab/base_tree && timeout -k 10 180 python3 bench.py --no-cpu $ARGS 2>/dev/null) | python3 -c "$pick") || exit 1
  echo "base $v"
  v=$(timeout -k 10 180 python3 bench.py --no-cpu --burn-in 0 $ARGS 2>/dev/null | python3 -c "$pick") || exit 1
  echo "cur $v"
  for kv in "$@"; do
    v=$(env $kv timeout -k 10 180 python3 bench.py --no-cpu --burn-in 0 $ARGS 2>/dev/null | python3 -c "$pick") || exit 1
    echo "cur[$kv] $v"
  done
done
