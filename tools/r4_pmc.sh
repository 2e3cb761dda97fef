#!/bin/bash
# GPU box: PMC passes of the C2 group kernel and the C3 block kernel, their summaries and the
# C2 VALU-issue JSON.  Usage: bash tools/r4_pmc.sh <tag>
set -o pipefail
TAG=${1:-pmc}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
bash tools/pmc.sh "$OUT/c2" || exit 1
python3 tools/pmc_summary.py "$OUT/c2" core_group > "$OUT/pmc_c2_summary.txt" && cat "$OUT/pmc_c2_summary.txt"
python3 tools/valu_json.py "$OUT/c2" 12 12 32 65536 core_group_kernel || exit 1
bash tools/pmc.sh "$OUT/c3" --config 3 || exit 1
python3 tools/pmc_summary.py "$OUT/c3" core_block > "$OUT/pmc_c3_summary.txt" && cat "$OUT/pmc_c3_summary.txt"
python3 tools/valu_json.py "$OUT/c3" 64 64 512 8192 core_block_kernel || exit 1
cp profiles/valu_*.json "$OUT/"
echo all-ok
