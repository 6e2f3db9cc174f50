"""Find vector writes that the compiler placed where EXEC is zero: at the head of a basic block that is entered only
with EXEC = 0 -- through `s_cbranch_execz`, or by falling through an `s_cbranch_execnz` that was not taken (the exit
of a divergent loop) -- before the block's first EXEC write (any form: `s_or_b64 exec` with exec as either source,
`s_mov_b64 exec`, the saveexec family, `v_cmpx`).  Such a write (typically a register-allocation copy such as
`v_accvgpr_write_b32 aN, vM` of a value live in every lane) writes no lane, and a later read of the copy returns
whatever the previous wave left in the register.  The whole block is scanned.

This is the instruction-level cause of the round-4/5 aggregation fault: in the (128, 2, 3) tangent
vf_kernel of the ds_add_f32 build, `v_accvgpr_write_b32 a26, v23` (a live-range split copy of a per-lane value
computed at kernel entry) sits before the EXEC restore of a loop-exit block reached only through s_cbranch_execz, and
the block loop reads a26 back.  Blocks also entered with live lanes (a plain fall-through or another branch) are
not reported: their writes reach the lanes of that entry.

Usage: python tools/isa_exec_copies.py [LIB.so] [KERNEL_REGEX]    (exit status 1 if any is found)
tests/test_isa_hazards.py runs it on every kernel of the shipped library and on known-answer blocks of every idiom.
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


# any instruction that writes EXEC: a scalar op with exec as its destination, the saveexec family, v_cmpx
EXEC_WRITE = re.compile(r"^(s_\w+ exec\b|s_\w*saveexec\w*|v_cmpx_)")
BRANCH = ("s_branch", "s_cbranch", "s_setpc", "s_swappc", "s_endpgm")


def _target(a, t):
    off = int(t.split()[1])
    off -= 65536 if off >= 32768 else 0
    return a + 4 + 4 * off


def check(insts):
    """[(block start address, [vector writes], the instruction that ends them, entry)] for every basic block that is
    entered ONLY with EXEC = 0 and issues vector writes before its first EXEC write (such writes reach no lane).  A
    zero-EXEC entry edge is an `s_cbranch_execz` to the block ('execz') or the fall-through of an `s_cbranch_execnz`
    that was not taken ('execnz-fallthrough': e.g. the exit of a divergent loop whose last iteration cleared EXEC).
    Blocks start at branch targets and after branches; the whole block is scanned up to its first EXEC write of any
    form (s_or / s_mov / s_and / s_xor ... exec with either operand order, the saveexec family, v_cmpx) or its
    terminator.  A block also entered by another branch or a plain fall-through is not reported: its writes reach the
    lanes of that entry."""
    idx = {a: i for i, (a, _) in enumerate(insts)}
    starts, zero, live = {0}, {}, {0}
    for i, (a, t) in enumerate(insts):
        f = t.split()
        op = f[0]
        if op.startswith(("s_branch", "s_cbranch")) and len(f) > 1 and re.match(r"-?\d+$", f[1]):
            tgt = _target(a, t)
            if tgt in idx:
                starts.add(idx[tgt])
                if op == "s_cbranch_execz":
                    zero.setdefault(idx[tgt], "execz")
                else:
                    live.add(idx[tgt])
        if i + 1 < len(insts):
            if op == "s_cbranch_execnz":
                zero.setdefault(i + 1, "execnz-fallthrough")
            elif not op.startswith(("s_branch", "s_setpc", "s_endpgm")):
                live.add(i + 1)   # plain fall-through (or a conditional branch not on EXEC)
        if op.startswith(BRANCH):
            starts.add(i + 1)
    starts = sorted(s for s in starts if s < len(insts))
    found = []
    for k, i in enumerate(starts):
        if i not in zero or i in live:
            continue
        stop = starts[k + 1] if k + 1 < len(starts) else len(insts)
        writes, end = [], "end of block"
        for j in range(i, stop):
            t = insts[j][1]
            op = t.split()[0]
            if EXEC_WRITE.match(t) or op.startswith(BRANCH):
                end = t
                break
            if VEC_WRITE.match(op) and not op.startswith(NO_VEC_DST):
                writes.append(t)
        if writes:
            found.append((insts[i][0], writes, end, zero[i]))
    return found


def main(argv):
    lib = argv[1] if len(argv) > 1 else KR.LIB
    pat = argv[2] if len(argv) > 2 else ""
    n = 0
    for fn, insts in functions(lib).items():
        if pat and not re.search(pat, fn):
            continue
        for a, writes, restore, entry in check(insts):
            n += 1
            print(f"{fn}: block {a:#x} ({entry} EXEC on entry) writes {writes} before `{restore}`")
    print(f"{n} blocks with vector writes ahead of an EXEC restore")
    return 1 if n else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
