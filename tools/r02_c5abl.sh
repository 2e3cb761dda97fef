#!/bin/bash
# GPU box: C5 kernel times of library builds (rocprof kernel stats per build).
set -o pipefail
OUT=gpurun_out/c5abl; mkdir -p $OUT; export TMPDIR=/tmp
for f in $1; do
  n=$(basename $f .so)
  FFM_LIB_PATH=$PWD/$f timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$n -o run -- python3 bench.py --no-cpu --config 5 --steps 30 --warmup 3 --repeats 1 > $OUT/$n.log 2>&1 || { tail $OUT/$n.log; exit 1; }
  echo "== $n"; python3 -c "
import csv
for r in csv.DictReader(open('$OUT/$n/run_kernel_stats.csv')):
    print('  %-60s %8.1f us' % (r['Name'][:60], float(r['AverageNs'])/1e3))" | head -7
done
