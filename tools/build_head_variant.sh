#!/bin/bash
# Timing baseline: the stamps library built from git HEAD (or $1), as tools/libvar_head.so, for A/B runs next to
# tools/build_variants.sh variants of the working tree.
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
REV=${1:-HEAD}
TMP=$(mktemp -d)
git -C "$ROOT" archive "$REV" ecnf-baseline-neurips-2023_amd/csrc include | tar -x -C "$TMP"
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -shared -fno-slp-vectorize -mllvm -amdgpu-mfma-vgpr-form \
  -Wno-pass-failed -Wno-unused-value -Wno-unused-result -DECNF_STAMPS -DECNF_DEV_LJ13_ONLY -I "$TMP/include" \
  -o "$ROOT/tools/libvar_head.so" "$TMP/ecnf-baseline-neurips-2023_amd/csrc/ecnf_hip.hip"
rm -rf "$TMP"
