#!/bin/bash
# GPU box: occupancy sweep, skeleton ablation and env-count scaling of the lane kernel.
set -o pipefail
OUT=gpurun_out/lane_diag2; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/ab_core.sh "build_ab/lib_w7.so build_ab/lib_w4.so build_ab/lib_w5.so build_ab/lib_w8.so build_ab/lib_skel.so build_ab/lib_skel2.so" > $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
cat $OUT/ab.log
for e in 16384 32768 131072; do
  bash tools/ab_core.sh "build_ab/lib_w7.so" --envs $e > $OUT/ab_e$e.log 2>&1 || { tail $OUT/ab_e$e.log; exit 1; }
  echo "E=$e"; cat $OUT/ab_e$e.log
done
