#!/bin/bash
# GPU box: PMC counters of the C3 block kernel and the C4 learner batch kernel at HEAD,
# the multi-step K sweep for C2 and C3.
set -o pipefail
OUT=gpurun_out/pmc34; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/pmc.sh $OUT/c3 --config 3 --multi-step 0 > $OUT/c3.log 2>&1 || { tail $OUT/c3.log; exit 1; }
python3 tools/pmc_summary.py $OUT/c3 core_block > $OUT/pmc_c3_summary.txt; cat $OUT/pmc_c3_summary.txt
bash tools/pmc.sh $OUT/c4 --config 4 > $OUT/c4.log 2>&1 || { tail $OUT/c4.log; exit 1; }
python3 tools/pmc_summary.py $OUT/c4 learn_batch > $OUT/pmc_c4_summary.txt; cat $OUT/pmc_c4_summary.txt
for k in 10 25 50; do
  timeout -k 10 300 python3 bench.py --no-cpu --repeats 3 --multi-step $k > $OUT/c2_k$k.json 2> $OUT/c2_k$k.err || { tail $OUT/c2_k$k.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/c2_k$k.json'));m=d['multi_step'];print('C2 K=$k', round(m['value']/1e9,2),'G', round(m['ms_per_step']*1e3,2),'us/step; single', round(d['value']/1e9,2))"
done
timeout -k 10 300 python3 bench.py --no-cpu --repeats 3 --config 3 --multi-step 10 > $OUT/c3_k10.json 2> $OUT/c3_k10.err || { tail $OUT/c3_k10.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/c3_k10.json'));m=d['multi_step'];print('C3 K=10', round(m['value']/1e9,2),'G; single', round(d['value']/1e9,2))"
