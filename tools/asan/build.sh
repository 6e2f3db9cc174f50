#!/bin/bash
# AddressSanitizer build of the host side of libecnf_hip.so and of its driver abi_asan.cpp.
# The host translation units (ecnf_hip.hip host code, ecnf_train.hip) are instrumented on the HOST pass only
# (-Xarch_host); device code is not.  The per-shape kernel objects are the product build's (run
# __graft_entry__.build() first; it passes the exact object list as arguments, else every ecnf_part_*.o of the build
# directory is linked).  Outputs: tools/asan/libecnf_hip_asan.so and tools/asan/abi_asan (git-ignored).
set -e
ROOT="$(cd "$(dirname "$0")/../.." && pwd)"
OUT="$ROOT/tools/asan"
OBJ="$ROOT/ecnf-baseline-neurips-2023_amd/build"
CSRC="$ROOT/ecnf-baseline-neurips-2023_amd/csrc"
HIPCC=/opt/rocm/bin/hipcc
SAN="-Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer -Xarch_host -fsanitize-address-use-after-scope"
FLAGS="-O1 -g --offload-arch=gfx950 -std=c++17 -fPIC -fno-slp-vectorize -mllvm -amdgpu-mfma-vgpr-form -Wno-pass-failed -Wno-unused-value -Wno-unused-result -I $ROOT/include"
if [ $# -gt 0 ]; then PARTS=("$@"); else PARTS=("$OBJ"/ecnf_part_*.o); fi
ls "${PARTS[@]}" > /dev/null
$HIPCC $FLAGS $SAN -DECNF_SPLIT_TU -c "$CSRC/ecnf_hip.hip" -o "$OUT/ecnf_host_asan.o" &
$HIPCC $FLAGS $SAN -c "$CSRC/ecnf_train.hip" -o "$OUT/ecnf_train_asan.o" &
wait
$HIPCC --offload-arch=gfx950 -shared -fPIC $SAN -o "$OUT/libecnf_hip_asan.so" "$OUT/ecnf_host_asan.o" \
  "$OUT/ecnf_train_asan.o" "${PARTS[@]}"
$HIPCC -O1 -g -std=c++17 $SAN -I "$ROOT/include" "$OUT/abi_asan.cpp" -o "$OUT/abi_asan" -L "$OUT" -lecnf_hip_asan \
  -Wl,-rpath,'$ORIGIN'
rm -f "$OUT"/*.o
echo "built $OUT/abi_asan"
