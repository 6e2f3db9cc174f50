"""Find vector writes that the compiler placed where EXEC is zero: at the head of a block that `s_cbranch_execz`
jumps to, before that block's `s_or_b64 exec, exec, s[..]` restores EXEC (the join of a divergent region).  Reached
through the branch, such a block runs with EXEC = 0, so a vector write there (typically a register-allocation copy
such as `v_accvgpr_write_b32 aN, vM` of a value live in every lane) writes no lane, and a later read of the copy
returns whatever the previous wave left in the register.

This is the instruction-level cause of the round-4/5 aggregation fault: in the (128, 2, 3) tangent
vf_kernel of the ds_add_f32 build, `v_accvgpr_write_b32 a26, v23` (a live-range split copy of a per-lane value
computed at kernel entry) sits before the EXEC restore of a loop-exit block reached only through s_cbranch_execz, and
the block loop reads a26 back.  A block that is also entered by fall-through (a partial EXEC) is reported too.

Usage: python tools/isa_exec_copies.py [LIB.so] [KERNEL_REGEX]    (exit status 1 if any is found)
tests/test_isa_hazards.py runs it on every kernel of the shipped library.
"""
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import kernel_resources as KR  # noqa: E402

VEC_WRITE = re.compile(r"^(v_|ds_read|ds_bpermute|buffer_load|global_load|flat_load|scratch_load)")
NO_VEC_DST = ("v_cmp", "v_cmpx", "v_readlane", "v_readfirstlane", "v_writelane")   # (lane ops ignore EXEC)


def functions(lib):
    """{kernel name: [(address, text)]} of every code object of lib"""
    out = {}
    with tempfile.TemporaryDirectory() as td:
        for k, co in enumerate(KR.code_objects(lib)):
            p = os.path.join(td, f"co{k}")
            open(p, "wb").write(co)
            dis = subprocess.run([f"{KR.LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", p], capture_output=True, text=True,
                                 check=True).stdout
            fn = None
            for line in dis.splitlines():
                m = re.match(r"^[0-9a-f]+ <(.*)>:", line)
                if m:
                    fn = m.group(1)
                    out[fn] = []
                    continue
                if fn and line.startswith("\t"):
                    code, _, com = line.partition("//")
                    a = re.match(r"\s*([0-9A-Fa-f]+):", com)
                    if code.strip() and a:
                        out[fn].append((int(a.group(1), 16), code.strip()))
    return out


def check(insts):
    idx = {a: i for i, (a, _) in enumerate(insts)}
    targets = set()
    for a, t in insts:
        if t.startswith("s_cbranch_execz"):
            off = int(t.split()[1])
            off -= 65536 if off >= 32768 else 0
            if a + 4 + 4 * off in idx:
                targets.add(idx[a + 4 + 4 * off])
    found = []
    for i in sorted(targets):
        writes = []
        for j in range(i, min(len(insts), i + 64)):
            t = insts[j][1]
            op = t.split()[0]
            if "exec" in t.split(",")[0] or op.startswith(("s_branch", "s_cbranch", "s_setpc", "s_endpgm")):
                if re.match(r"s_or_b64 exec, exec, s\[\d+:\d+\]", t) and writes:
                    found.append((insts[i][0], writes, t))
                break
            if VEC_WRITE.match(op) and not op.startswith(NO_VEC_DST):
                writes.append(t)
    return found


def main(argv):
    lib = argv[1] if len(argv) > 1 else KR.LIB
    pat = argv[2] if len(argv) > 2 else ""
    n = 0
    for fn, insts in functions(lib).items():
        if pat and not re.search(pat, fn):
            continue
        for a, writes, restore in check(insts):
            n += 1
            print(f"{fn}: block {a:#x} (entered by s_cbranch_execz) writes {writes} before `{restore}`")
    print(f"{n} vector writes under a zero EXEC")
    return 1 if n else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
