#!/bin/bash
# GPU box: critic_only curriculum (the pretrained critic), then the unified actor_only
# curriculum on it at several env counts, for the comparison with the reference's logged
# actor run (output/logs/unified_actor_training/run_20260119_070834, 100 episodes per
# configuration; tools/actor_pin_compare.py).  E >= 100: one episode per env, envs spread
# over the per-configuration epsilon schedule (--eps-phase, the default); also E = 4096
# with --no-eps-phase (every env at the schedule's first episode) to size that cause.
# Usage: bash tools/actor_pin.sh <tag> [E ...]
set -o pipefail
TAG=${1:-actor_pin}; shift || true
ES=${@:-10 512 4096}
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python3 -m ffm_amd.train --mode critic_only --envs 4096 --episodes 1000 --out $OUT/critic > $OUT/critic.log 2>&1 || { tail $OUT/critic.log; exit 1; }
tail -2 $OUT/critic.log
for e in $ES; do
  timeout -k 10 400 python3 -m ffm_amd.train --mode actor_only --envs $e --episodes 100 --trajectory-every 0 \
      --critic $OUT/critic/V_table.pkl --out $OUT/actor_e$e > $OUT/actor_e$e.log 2>&1 || { tail $OUT/actor_e$e.log; exit 1; }
  tail -2 $OUT/actor_e$e.log
done
timeout -k 10 400 python3 -m ffm_amd.train --mode actor_only --envs 4096 --episodes 100 --trajectory-every 0 --no-eps-phase \
    --critic $OUT/critic/V_table.pkl --out $OUT/actor_e4096_nophase > $OUT/actor_e4096_nophase.log 2>&1 || { tail $OUT/actor_e4096_nophase.log; exit 1; }
tail -2 $OUT/actor_e4096_nophase.log
