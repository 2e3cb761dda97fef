#!/bin/bash
# Resource usage of the C2 wave kernel (VGPR/SGPR/spills/occupancy) for a source tree.
# Usage: bash tools/regs.sh [csrc_dir] [extra hipcc flags]
SRC=${1:-$(dirname $0)/../ffm_amd/csrc}; shift || true
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-gpu-flush-denormals-to-zero \
  -fhip-fp32-correctly-rounded-divide-sqrt --cuda-device-only -c -Rpass-analysis=kernel-resource-usage "$@" \
  $SRC/core_step.hip -o /tmp/regs_$$.o 2>&1 | grep -A16 "core_wave_kernelILi4ELb0ELi2ELi12ELi12" | \
  grep -E "VGPRs:|SGPRs:|Spill|Occupancy|Scratch" | sed 's/.*remark: *//; s/ \[-Rpass.*//' | head -7 | paste -sd' '
rm -f /tmp/regs_$$.o
