#!/bin/bash
# Profile the bench kernel with rocprofv3 (run on the GPU box via gpurun).
# Usage: bash tools_profile.sh <outdir> [bench args...]
set -eo pipefail
OUT=${1:-gpurun_out/prof}; shift || true
export TMPDIR=/tmp
mkdir -p "$OUT"
B="python3 bench.py --no-cpu --steps 200 --warmup 20 $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- $B > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- $B > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- $B > "$OUT/write.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d "$OUT/sq" -o run -- $B > "$OUT/sq.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d "$OUT/sq2" -o run -- $B > "$OUT/sq2.log" 2>&1
echo done
