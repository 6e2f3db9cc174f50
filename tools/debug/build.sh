#!/bin/bash
# Device-checked diagnostic build ("a HIP debug build with bounds asserts"): the LJ13-shape
# kernels with ECNF_DCHECK bounds checks compiled in (egnn_eval.hpp), plus ecnf_debug_checks() to read the failed-check
# bits.  Output: tools/debug/libecnf_hip_checked.so (git-ignored; never the product library).
set -e
ROOT="$(cd "$(dirname "$0")/../.." && pwd)"
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -shared -fno-slp-vectorize -mllvm -amdgpu-mfma-vgpr-form \
  -Wno-pass-failed -Wno-unused-value -Wno-unused-result -DECNF_DEVICE_CHECKS -DECNF_DEV_LJ13_ONLY -I "$ROOT/include" \
  -o "$ROOT/tools/debug/libecnf_hip_checked.so" "$ROOT/ecnf-baseline-neurips-2023_amd/csrc/ecnf_hip.hip" \
  "$ROOT/ecnf-baseline-neurips-2023_amd/csrc/ecnf_train.hip"
echo "built $ROOT/tools/debug/libecnf_hip_checked.so"
