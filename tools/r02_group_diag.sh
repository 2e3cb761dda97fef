#!/bin/bash
set -o pipefail
OUT=gpurun_out/group_diag; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/ab_core.sh "build_ab/lib_w7.so build_ab/lib_g3.so build_ab/lib_g4.so build_ab/lib_g6.so build_ab/lib_g8.so" > $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
cat $OUT/ab.log
FFM_LIB_PATH=$PWD/build_ab/lib_g8.so bash tools/pmc.sh $OUT/pmc > $OUT/pmc.log 2>&1 || { tail $OUT/pmc.log; exit 1; }
python3 tools/pmc_summary.py $OUT/pmc core_group > $OUT/pmc_summary.txt; cat $OUT/pmc_summary.txt
for e in 24576 49152 73728; do
  bash tools/ab_core.sh "build_ab/lib_g8.so" --envs $e > $OUT/ab_e$e.log 2>&1 || { tail $OUT/ab_e$e.log; exit 1; }
  echo "E=$e"; cat $OUT/ab_e$e.log
done
