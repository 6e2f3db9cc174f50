#!/bin/bash
# Diagnostic build with in-kernel phase stamps (never the product library).
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -shared -fno-slp-vectorize -mllvm -amdgpu-mfma-vgpr-form -Wno-pass-failed -Wno-unused-value \
  -Wno-unused-result -DECNF_STAMPS ${DEVFLAGS:--DECNF_DEV_LJ13_ONLY} -I "$ROOT/include" -o "$ROOT/tools/libecnf_hip_stamps${STAMPS_TAG}.so" \
  "$ROOT/ecnf-baseline-neurips-2023_amd/csrc/ecnf_hip.hip" "$ROOT/ecnf-baseline-neurips-2023_amd/csrc/ecnf_train.hip"
