#!/bin/bash
# GPU box: learner Philox tests (small-map reset kernel), then C4 kernel times of two builds.
set -o pipefail
OUT=gpurun_out/lreset; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_learn.py -m gpu -x -v --timeout 300 --timeout-method thread -k "philox_12x12" > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for f in build_ab/lib_g_rank2.so build_ab/lib_l_rank.so; do
  n=$(basename $f .so)
  FFM_LIB_PATH=$PWD/$f timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$n -o run -- python3 bench.py --no-cpu --config 4 --repeats 1 > $OUT/$n.log 2>&1 || { tail $OUT/$n.log; exit 1; }
  echo "== $n"; python3 -c "
import csv
for r in csv.DictReader(open('$OUT/$n/run_kernel_stats.csv')):
    print('  %-60s %8.1f us' % (r['Name'][:60], float(r['AverageNs'])/1e3))" | head -4
done
