#!/bin/bash
# Resource usage and instruction counts of learner batch / tile kernels (device asm).
# Usage: bash tools/lregs.sh <out.s> [extra hipcc flags]; prints one line per kernel.
OUT=${1:-/tmp/lregs.s}; shift || true
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-gpu-flush-denormals-to-zero \
  -fhip-fp32-correctly-rounded-divide-sqrt --cuda-device-only -S "$@" -o "$OUT" \
  $(dirname $0)/../ffm_amd/csrc/learn_step.hip 2>&1 | grep -E "error" 
grep -n "^_ZN3ffm12_GLOBAL__N_1[0-9]*learn_\(batch\|tile\)[^ ]*:" "$OUT" | while IFS=: read L name rest; do
  t=$(echo $name | sed 's/_ZN3ffm12_GLOBAL__N_1[0-9]*//;s/EEEv.*//;s/EvNS.*//')
  E=$(awk -v s=$L 'NR>s && /^\.Lfunc_end/ {print NR; exit}' "$OUT")
  n=$(awk -v s=$L -v e=$E 'NR>s && NR<e && /^[ \t]+[sv]_/' "$OUT" | wc -l)
  v=$(awk -v s=$L -v e=$E 'NR>s && NR<e && /^[ \t]+v_/' "$OUT" | wc -l)
  echo -n "$t insts=$n valu=$v "
  awk -v s=$L 'NR>=s' "$OUT" | grep -m4 -E "; (NumVgprs|TotalNumSgprs|ScratchSize|Occupancy):" | sed 's/; //' | tr '\n' ' '; echo
done
