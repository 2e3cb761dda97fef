#!/bin/bash
# GPU box: lane-kernel diagnosis -- phase stamps, PMC counter passes, ablation A/B.
set -o pipefail
OUT=gpurun_out/lane_diag; mkdir -p $OUT; export TMPDIR=/tmp
FFM_LIB_PATH=$PWD/build_ab/lib_stamps.so timeout -k 10 120 python3 tools/stamps.py > $OUT/stamps.log 2>&1 || { tail $OUT/stamps.log; exit 1; }
cat $OUT/stamps.log
bash tools/pmc.sh $OUT/pmc > $OUT/pmc.log 2>&1 || { tail $OUT/pmc.log; exit 1; }
python3 tools/pmc_summary.py $OUT/pmc core_lane > $OUT/pmc_summary.txt; cat $OUT/pmc_summary.txt
bash tools/ab_core.sh "build_ab/lib_base.so build_ab/lib_abl1.so build_ab/lib_abl2.so build_ab/lib_abl8.so" > $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
cat $OUT/ab.log
