#!/bin/bash
# Register / scratch usage of the LJ13-shape kernels (M=128, L=3, D=3) from the compiler's resource remarks.
# Usage: tools/resusage.sh [extra hipcc flags]
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -fno-slp-vectorize -mllvm -amdgpu-mfma-vgpr-form \
  -Wno-pass-failed -Wno-unused-value -Wno-unused-result -I "$ROOT/include" -DECNF_PART_M=${M:-128} -DECNF_PART_L=${L:-3} \
  -DECNF_PART_D=${D:-3} -DECNF_PART_TAN=${TAN:-0} -DECNF_PART_PREC=${PREC:-0} --offload-device-only -Rpass-analysis=kernel-resource-usage "$@" \
  -c "$ROOT/ecnf-baseline-neurips-2023_amd/csrc/ecnf_part.hip" -o /tmp/resusage.o 2>&1 |
  grep -E "Function Name|VGPRs:|Scratch|Spill|Occupancy" | sed -e 's/.*remark: *//' -e 's/ \[-Rpass.*//'
