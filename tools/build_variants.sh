#!/bin/bash
# Timing-only experiment builds of the stamps library (never the product).  Usage: tools/build_variants.sh NAME:FLAGS ...
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
for spec in "$@"; do
  name="${spec%%:*}"; flags="${spec#*:}"
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -shared -fno-slp-vectorize -mllvm -amdgpu-mfma-vgpr-form -Wno-pass-failed -Wno-unused-value \
    -Wno-unused-result -DECNF_STAMPS -DECNF_DEV_LJ13_ONLY $flags -I "$ROOT/include" -o "$ROOT/tools/libvar_${name}.so" \
    "$ROOT/ecnf-baseline-neurips-2023_amd/csrc/ecnf_hip.hip" &
done
wait
