#!/bin/bash
# GPU box: issue rates of the integer multiplies and the calibration of valu_issue_frac
# (tools/alubench.hip: kernels of a known VALU count per wave, 8 waves per SIMD).
set -o pipefail
OUT=${1:-gpurun_out/alu}
export TMPDIR=/tmp
mkdir -p "$OUT"
hipcc --offload-arch=gfx950 -O3 -o "$OUT/alubench" tools/alubench.hip || exit 1
timeout -k 10 60 "$OUT/alubench" | tee "$OUT/rates.txt" || exit 1
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc" -o run -- "$OUT/alubench" > "$OUT/pmc.log" 2>&1 || { echo "alu pmc failed"; tail -5 "$OUT/pmc.log"; exit 1; }
echo alu done
