#!/bin/bash
# A/B timing of library builds, interleaved (GPU box):
#   bash tools/ab.sh "libA.so libB.so ..." [bench args...]
set -o pipefail
export TMPDIR=/tmp
LIBS=$1; shift
for r in 1 2 3; do
  for f in $LIBS; do
    v=$(FFM_LIB_PATH=$PWD/$f timeout -k 10 120 python3 bench.py --no-cpu "$@" 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['step_ms_events']*1000,1), 'us')") || exit 1
    echo "$(basename $f .so) $v"
  done
done
