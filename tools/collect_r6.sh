#!/bin/bash
# Host side: copy a tools/final_r6.sh pass (gpurun_out/<tag>) into profiles/r06/final and the
# profile JSONs bench.py reads (traffic_*.json, valu_*.json), stamped with the pass.
set -e
O=gpurun_out/${1:-final6b}; D=profiles/r06/final; STAMP="round 6 (${1:-final6b} pass)"
mkdir -p $D/pmc $D/esweep
for c in 2 3 4 5; do
  [ -f $O/bench_c$c.json ] && cp $O/bench_c$c.json $D/bench_c$c.json
  [ -f $O/trace_c$c/run_kernel_stats.csv ] && cp $O/trace_c$c/run_kernel_stats.csv $D/kernel_stats_c$c.csv
  if [ -f $O/traffic_c$c/traffic.json ]; then
    python3 -c "
import json; d=json.load(open('$O/traffic_c$c/traffic.json')); d['measured']='$STAMP'
p='profiles/traffic_'+d['config']+'.json'; json.dump(d, open(p,'w'), indent=1); print(p, round(d['traffic_over_algorithmic'],3))"
  fi
done
[ -f $O/trace_e8192/run_kernel_stats.csv ] && cp $O/trace_e8192/run_kernel_stats.csv $D/kernel_stats_c2_e8192.csv
[ -d $O/esweep ] && cp $O/esweep/e*.json $D/esweep/
[ -f $O/rehearse_c4/bench.log ] && tail -1 $O/rehearse_c4/bench.log > profiles/r06/rehearse_c4_n2.json
if [ -d $O/pmc_c2 ]; then
  FFM_MEASURED="$STAMP" python3 tools/valu_json.py $O/pmc_c2 12 12 32 65536
  FFM_MEASURED="$STAMP" python3 tools/valu_json.py $O/pmc_c3 64 64 512 8192 core_block_kernel
  python3 tools/pmc_summary.py $O/pmc_c2 core_group_kernel > $D/pmc/pmc_c2_summary.txt
  python3 tools/pmc_summary.py $O/pmc_c3 core_block_kernel > $D/pmc/pmc_c3_summary.txt
fi
echo collected $O
