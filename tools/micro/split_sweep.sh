#!/bin/bash
# Build (no arg) or run (arg "run") the split-chain microbenchmark variants tools/micro/sb_<name>.
# Variants: waves per CU (1 or 2 per SIMD) x {production, cheap activation, no weight loads, no transcendentals}.
D="$(cd "$(dirname "$0")" && pwd)"
V="w4:-DWAVES=4 w8:-DWAVES=8 w4two:-DWAVES=4|-DTWO_TILES w4twonowl:-DWAVES=4|-DTWO_TILES|-DECNF_SPLIT_NO_WLOAD w8nowl:-DWAVES=8|-DECNF_SPLIT_NO_WLOAD"
if [ "$1" = "run" ]; then
  for v in $V; do n=${v%%:*}; echo -n "$n: "; timeout -k 5 60 "$D/sb_$n" || exit 1; done
  exit 0
fi
for v in $V; do
  n=${v%%:*}; f=${v#*:}; f=${f//|/ }
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fno-slp-vectorize -mllvm -amdgpu-mfma-vgpr-form \
    -Wno-pass-failed -Wno-unused-value -Wno-unused-result $f -o "$D/sb_$n" "$D/split_bench.hip" &
done
wait
ls "$D"/sb_*
