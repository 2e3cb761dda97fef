#!/bin/bash
# A/B timing of library builds, interleaved (GPU box):
#   bash tools/ab.sh "libA.so libB.so@VAR=val ..." [bench args...]
# an entry lib@VAR=val runs that library with the environment variable set.  Prints the
# event-timed step, the median window rate, and the mean step over all timed windows.
set -o pipefail
export TMPDIR=/tmp
LIBS=$1; shift
pick='import json,sys; d=json.loads(sys.stdin.read()); r=d["repeats"]; print(round(d.get("step_ms_events", d.get("kernel_ms_mean"))*1000,1), "us", round(d["value"]/1e9,2), "G", round(sum(r["elapsed_s"])/(len(r["elapsed_s"])*d["steps"])*1e6,1), "us/step over the windows")'
for r in 1 2 3; do
  for f in $LIBS; do
    lib=${f%%@*}; kv=""; [ "$lib" != "$f" ] && kv=${f#*@}
    v=$(env $kv FFM_LIB_PATH=$PWD/$lib timeout -k 10 120 python3 bench.py --no-cpu "$@" 2>/dev/null | python3 -c "$pick") || exit 1
    echo "$(basename $lib .so)${kv:+[$kv]} $v"
  done
done
