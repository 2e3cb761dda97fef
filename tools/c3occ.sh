#!/bin/bash
# GPU box: the large-placement learner test, then the C3 A/B of the block kernel's
# occupancy variants (reset keys aliased into the dead arrays; 8 waves per SIMD).
set -o pipefail
OUT=gpurun_out/c3occ
mkdir -p $OUT
export TMPDIR=/tmp
bash tools/place_gpu.sh || exit 1
bash tools/ab.sh "ab/libhead.so ab/libbw1.so ab/libbw8.so" --config 3 --steps 1500 --repeats 3 > $OUT/ab.log 2>&1 || { echo "ab failed"; tail $OUT/ab.log; exit 1; }
cat $OUT/ab.log
