#!/bin/bash
# Build (no arg) or run (arg "run") the split-chain microbenchmark variants tools/micro/sb_<name>.
# Variants: waves per CU (1 or 2 per SIMD) x {production, cheap activation, no weight loads, no transcendentals}.
D="$(cd "$(dirname "$0")" && pwd)"
V="w8:-DWAVES=8 w8ring:-DWAVES=8|-DECNF_SPLIT_RING w8ring8:-DWAVES=8|-DECNF_SPLIT_RING|-DECNF_RING_IV=8 w8ring2:-DWAVES=8|-DECNF_SPLIT_RING|-DECNF_RING_IV=2 w8wlds:-DWAVES=8|-DECNF_SPLIT_WLDS"
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
