#!/bin/bash
set -o pipefail
OUT=gpurun_out/fixed_diag; mkdir -p $OUT; export TMPDIR=/tmp
for e in 65536 14336; do
  bash tools/ab_core.sh "build_ab/lib_w7.so build_ab/lib_abl64.so" --envs $e > $OUT/ab_e$e.log 2>&1 || { tail $OUT/ab_e$e.log; exit 1; }
  echo "E=$e"; cat $OUT/ab_e$e.log
done
for b in 896 1280 1792; do
  FFM_WAVE_BLOCKS=$b bash tools/ab_core.sh "build_ab/lib_w7.so" > $OUT/ab_b$b.log 2>&1 || { tail $OUT/ab_b$b.log; exit 1; }
  echo "blocks=$b"; cat $OUT/ab_b$b.log
done
