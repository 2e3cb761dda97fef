#!/bin/bash
# GPU box: lane kernel time at exactly 1..4 env pairs per wave (7168 waves), full and skeleton.
set -o pipefail
OUT=gpurun_out/lane_diag3; mkdir -p $OUT; export TMPDIR=/tmp
for e in 14336 28672 43008 57344; do
  bash tools/ab_core.sh "build_ab/lib_w7.so build_ab/lib_skel.so" --envs $e > $OUT/ab_e$e.log 2>&1 || { tail $OUT/ab_e$e.log; exit 1; }
  echo "E=$e"; cat $OUT/ab_e$e.log
done
