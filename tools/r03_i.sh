#!/bin/bash
# GPU box: tiled / stencil parity, interleaved C5 A/B (build_ab/head.so vs current),
# C5 kernel trace, PMC instruction/wait counters of the C5 tile and stencil kernels.
set -o pipefail
OUT=gpurun_out/${1:-i}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "${2:-tiled or config5 or column_stencil}" > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 600 bash tools/ab.sh "build_ab/head.so ffm_amd/_lib/libffm_amd.so" --config 5 --steps 30 --warmup 5 > "$OUT/ab_c5.log" 2>&1 || { echo "ab failed"; cat "$OUT/ab_c5.log"; exit 1; }
cat "$OUT/ab_c5.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_c5" -o run -- python3 bench.py --no-cpu --config 5 --steps 30 --warmup 5 --repeats 1 > "$OUT/trace_c5.log" 2>&1 || { echo "trace failed"; tail -20 "$OUT/trace_c5.log"; exit 1; }
python3 tools/kstats.py "$OUT/trace_c5/run_kernel_trace.csv" 10
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM SQ_BUSY_CYCLES SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_SCA"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pmc/p$i" -o run -- python3 bench.py --no-cpu --config 5 --steps 10 --warmup 2 --repeats 1 > "$OUT/pmc_p$i.log" 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done
for k in learn_tile_v learn_tile_h_kernel learn_stencil_col learn_batch; do echo "== $k"; python3 tools/pmc_summary.py "$OUT/pmc" $k; done > "$OUT/pmc_summary.txt"
cat "$OUT/pmc_summary.txt"
