#!/bin/bash
# Timing-only experiment builds WITHOUT stamps (LJ13 shape only), as tools/libt_<name>.so; "head" builds git HEAD.
# Usage: [DEVFLAGS='-DECNF_DEV_M=64 -DECNF_DEV_L=2 -DECNF_DEV_D=3'] tools/build_timing.sh NAME:FLAGS ...   (a NAME of "head"
# takes the sources of git HEAD, "rev_<sha>" those of that commit)
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
for spec in "$@"; do
  name="${spec%%:*}"; flags="${spec#*:}"
  SRC="$ROOT"
  if [ "$name" = "head" ] || [ "${name#rev_}" != "$name" ]; then
    rev=HEAD; [ "$name" != "head" ] && rev="${name#rev_}"
    SRC=$(mktemp -d)
    git -C "$ROOT" archive "$rev" ecnf-baseline-neurips-2023_amd/csrc include | tar -x -C "$SRC"
  fi
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -shared -fno-slp-vectorize -mllvm -amdgpu-mfma-vgpr-form \
    -Wno-pass-failed -Wno-unused-value -Wno-unused-result ${DEVFLAGS:--DECNF_DEV_LJ13_ONLY} $flags -I "$SRC/include" \
    -o "$ROOT/tools/libt_${name}.so" "$SRC/ecnf-baseline-neurips-2023_amd/csrc/ecnf_hip.hip" "$SRC/ecnf-baseline-neurips-2023_amd/csrc/ecnf_train.hip" &
done
wait
