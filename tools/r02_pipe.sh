#!/bin/bash
set -o pipefail
OUT=gpurun_out/pipe; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/ab_core.sh "build_ab/lib_base.so build_ab/lib_pipe.so" --envs-per-block -2 > $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
cat $OUT/ab.log
