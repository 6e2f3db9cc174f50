"""Static instruction mix of one kernel of a built library (gfx950 disassembly, no GPU).

Counts every instruction of the kernel's code by class, and the same restricted to the MFMA-dense regions (runs of
code where consecutive v_mfma are at most GAP instructions apart: the split chains), per MFMA.  Static counts: the
edge tile is straight-line code, so within a region they are also the dynamic counts per tile execution.

Usage: python tools/isa_mix.py KERNEL_REGEX [lib.so] [GAP]
  e.g. python tools/isa_mix.py 'integrate_kernelILi4ELi0ELi3ELi3ELi0ELb0ELb0ELb0E'
"""
import collections
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import kernel_resources as KR  # noqa: E402

CLASSES = (
    ("mfma", lambda op: op.startswith("v_mfma")),
    ("trans", lambda op: re.match(r"v_(exp|rcp|rsq|sqrt|log|sin|cos)_", op) is not None),
    ("dpp", lambda op: op.endswith("_dpp")),
    ("pk_f32", lambda op: re.match(r"v_pk_\w+_f32", op) is not None),
    ("mix_cvt", lambda op: re.match(r"v_(fma_mix|cvt_pk)", op) is not None),
    ("vmov", lambda op: re.match(r"v_(mov|accvgpr)", op) is not None),
    ("valu", lambda op: op.startswith("v_")),
    ("ds", lambda op: op.startswith("ds_")),
    ("vmem", lambda op: re.match(r"(buffer|global|flat|scratch)_", op) is not None),
    ("waitcnt", lambda op: op.startswith("s_waitcnt")),
    ("nop", lambda op: op.startswith("s_nop")),
    ("salu", lambda op: op.startswith("s_")),
)


def classify(op):
    for name, f in CLASSES:
        if f(op):
            return name
    return "other"


def kernel_ops(lib, pattern):
    """[(mnemonic, text)] of the first kernel whose mangled name matches pattern, and that name"""
    with tempfile.TemporaryDirectory() as td:
        for k, co in enumerate(KR.code_objects(lib)):
            p = os.path.join(td, f"co{k}")
            open(p, "wb").write(co)
            out = subprocess.run([f"{KR.LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", p], capture_output=True,
                                 text=True, check=True).stdout
            fn, ops = None, []
            for line in out.splitlines():
                m = re.match(r"^[0-9a-f]+ <(.*)>:", line)
                if m:
                    if fn and ops:
                        return fn, ops
                    fn = m.group(1) if re.search(pattern, m.group(1)) else None
                    ops = []
                    continue
                if fn and line.startswith("\t"):
                    t = line.strip().split("//")[0].strip()
                    if t:
                        ops.append((t.split()[0], t))
            if fn and ops:
                return fn, ops
    return None, []


def mix(ops):
    c = collections.Counter(classify(op) for op, _ in ops)
    return c


def dense_regions(ops, gap):
    idx = [i for i, (op, _) in enumerate(ops) if op.startswith("v_mfma")]
    regions, start, prev = [], None, None
    for i in idx:
        if start is None:
            start = prev = i
        elif i - prev > gap:
            regions.append((start, prev))
            start = i
        prev = i
    if start is not None:
        regions.append((start, prev))
    return [(a, b) for a, b in regions if sum(1 for op, _ in ops[a:b + 1] if op.startswith("v_mfma")) >= 24]


def main():
    pattern = sys.argv[1]
    lib = sys.argv[2] if len(sys.argv) > 2 else KR.LIB
    gap = int(sys.argv[3]) if len(sys.argv) > 3 else 24
    fn, ops = kernel_ops(lib, pattern)
    if not fn:
        sys.exit(f"no kernel matches {pattern}")
    print(fn, len(ops), "instructions")
    tot = mix(ops)
    print("whole kernel:", dict(tot.most_common()))
    regs = dense_regions(ops, gap)
    inside = collections.Counter()
    for a, b in regs:
        inside += mix(ops[a:b + 1])
    n = inside["mfma"]
    print(f"{len(regs)} MFMA-dense regions, {n} MFMAs, {sum(inside.values()) - n} other instructions "
          f"({(sum(inside.values()) - n) / max(n, 1):.2f} per MFMA)")
    print("  per MFMA:", {k: round(v / max(n, 1), 3) for k, v in inside.most_common() if k != "mfma"})
    outside = tot - inside
    print(f"outside the regions: {sum(outside.values())} instructions:", dict(outside.most_common()))
    top = collections.Counter(op for a, b in regs for op, _ in ops[a:b + 1])
    print("  top mnemonics inside:", top.most_common(16))
    top_out = collections.Counter(op for op, _ in ops) - top
    print("  top mnemonics outside:", top_out.most_common(24))


if __name__ == "__main__":
    main()
