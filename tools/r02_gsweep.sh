#!/bin/bash
set -o pipefail
OUT=gpurun_out/gsweep; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/ab_core.sh "build_ab/lib_base.so" --envs-per-block -2 > $OUT/lane.log 2>&1 || { tail $OUT/lane.log; exit 1; }
echo lane; cat $OUT/lane.log
bash tools/ab_core.sh "build_ab/lib_g4.so build_ab/lib_g4w7.so build_ab/lib_g6w5.so build_ab/lib_g8.so" --envs-per-block -3 > $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
cat $OUT/ab.log
