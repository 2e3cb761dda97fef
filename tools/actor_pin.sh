#!/bin/bash
# GPU box: critic_only curriculum (the pretrained critic), then the unified actor_only
# curriculum on it, for the comparison with the reference's logged actor run
# (output/logs/unified_actor_training/run_20260119_070834, 100 episodes per configuration).
set -o pipefail
OUT=gpurun_out/actor_pin; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python3 -m ffm_amd.train --mode critic_only --envs 4096 --episodes 1000 --out $OUT/critic > $OUT/critic.log 2>&1 || { tail $OUT/critic.log; exit 1; }
tail -2 $OUT/critic.log
for e in 10 100; do
  timeout -k 10 400 python3 -m ffm_amd.train --mode actor_only --envs $e --episodes 100 --trajectory-every 0 \
      --critic $OUT/critic/V_table.pkl --out $OUT/actor_e$e > $OUT/actor_e$e.log 2>&1 || { tail $OUT/actor_e$e.log; exit 1; }
  tail -3 $OUT/actor_e$e.log
done
