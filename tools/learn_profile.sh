#!/bin/bash
# GPU box: the C3 bench line at its defaults, PMC HBM traffic of the learner batch
# kernels (C4, C5; regenerates the profiles/traffic_*_learn{4,5}.json the bench reads),
# and the SQ instruction / wait counters of the C4 and C5 batch kernels.
# Usage: bash tools/learn_profile.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-lp}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py --config 3 > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err" || { echo "bench c3 failed"; tail -20 "$OUT/bench_c3.err"; exit 1; }
tail -1 "$OUT/bench_c3.json" | cut -c1-600
for c in 4 5; do
  timeout -k 10 600 bash tools/traffic.sh "$OUT/traffic_c$c" --config $c || { echo "traffic c$c failed"; exit 1; }
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM SQ_BUSY_CYCLES SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_SCA"; do
    i=$((i+1))
    timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pmc_c$c/p$i" -o run -- python3 bench.py --no-cpu --config $c --steps 20 --warmup 5 --repeats 1 > "$OUT/pmc_c${c}_p$i.log" 2>&1 || { echo "pmc c$c pass $i failed"; exit 1; }
  done
  python3 tools/pmc_summary.py "$OUT/pmc_c$c" learn_batch > "$OUT/pmc_c${c}_batch_summary.txt"
  cat "$OUT/pmc_c${c}_batch_summary.txt"
done
echo all-ok
