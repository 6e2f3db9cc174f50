"""Per-kernel register / scratch usage of a built library, read from the AMDGPU metadata notes of its gfx950 code
objects (the clang offload bundles in the .hip_fatbin section; llvm-objcopy + llvm-readelf, no GPU needed).

Usage: python tools/kernel_resources.py [lib.so]    (default: the product library)
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "ecnf-baseline-neurips-2023_amd", "ecnf_amd", "libecnf_hip.so")
LLVM = "/opt/rocm/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
FIELDS = ("private_segment_fixed_size", "vgpr_count", "vgpr_spill_count", "sgpr_spill_count")


def code_objects(lib):
    """the gfx950 code objects (ELF bytes) embedded in lib"""
    with tempfile.TemporaryDirectory() as td:
        fat = os.path.join(td, "fat.bin")
        subprocess.run([f"{LLVM}/llvm-objcopy", "-O", "binary", "--only-section=.hip_fatbin", lib, fat], check=True)
        data = open(fat, "rb").read()
    out, pos = [], 0
    while (i := data.find(MAGIC, pos)) >= 0:
        n = struct.unpack_from("<Q", data, i + 24)[0]
        p = i + 32
        for _ in range(n):
            off, size, idlen = struct.unpack_from("<QQQ", data, p)
            p += 24
            ident = data[p:p + idlen].decode()
            p += idlen
            if "gfx950" in ident:
                out.append(data[i + off:i + off + size])
        pos = i + 1
    return out


def kernels(lib=LIB):
    """{mangled kernel name: {field: int}} over every code object of lib"""
    res = {}
    with tempfile.TemporaryDirectory() as td:
        for k, co in enumerate(code_objects(lib)):
            path = os.path.join(td, f"co{k}.elf")
            open(path, "wb").write(co)
            notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", path], check=True, capture_output=True,
                                   text=True).stdout
            for block in re.split(r"\n(?=\s+- \.)", notes):   # one block per metadata list entry
                m = re.search(r"\.?name:\s+(\S+)", block)
                if not m or not m.group(1).startswith("_Z"):
                    continue
                rec = {}
                for f in FIELDS:
                    v = re.search(rf"\.?{f}:\s+(\d+)", block)
                    if v:
                        rec[f] = int(v.group(1))
                res[m.group(1)] = rec
    return res


def demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
    return dict(zip(names, out))


if __name__ == "__main__":
    ks = kernels(sys.argv[1] if len(sys.argv) > 1 else LIB)
    dm = demangle(sorted(ks))
    for name in sorted(ks):
        r = ks[name]
        short = re.sub(r"\(.*", "", dm[name]).replace("ecnf::", "")
        print(f"{short:48s} scratch {r.get('private_segment_fixed_size', -1):5d}  vgpr {r.get('vgpr_count', -1):3d}  "
              f"vgpr_spill {r.get('vgpr_spill_count', -1):4d}")
