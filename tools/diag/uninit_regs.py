"""Round-5 fault study, step 16: "maybe-uninitialised register" dataflow over one kernel's gfx950
disassembly.  Builds the control-flow graph from the branch offsets, then a forward must-analysis: a VGPR / AGPR is
defined after an instruction writes it on EVERY path from the kernel entry (v0 = the work-item id is defined at entry;
SGPRs are not tracked).  Every read of a register that is not defined on all paths is reported.  Known benign reads:
the high dword of v_mad_u64_u32's 64-bit addend when only the low dword of the result is used is still reported
(the caller compares two builds; report lines unique to one build are the suspects).

Usage: python tools/diag/uninit_regs.py LIB.so KERNEL_REGEX
"""
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import kernel_resources as KR  # noqa: E402

REG = re.compile(r"\b([va])(?:(\d+)|\[(\d+):(\d+)\])")
# instructions whose first operand is not a vector destination
NO_DST = ("ds_write", "ds_add_f32", "ds_add_u32", "buffer_store", "global_store", "flat_store", "scratch_store", "s_",
          "v_cmp", "v_cmpx", "v_readlane", "v_readfirstlane", "global_atomic", "flat_atomic", "buffer_atomic")
READS_DST = ("v_fmac", "v_mac", "v_fma_mixlo", "v_fma_mixhi", "v_writelane", "v_cvt_pk", "v_pk_fmac",
             "v_dot2c", "v_mov_b32_dpp", "v_mfma")   # (partial / accumulating writes; MFMA: src C is read explicitly)


DIVERGENT_FALLTHROUGH = False   # (True breaks loops lowered through s_cbranch_execz; kept for reference)


def regs(text):
    out = set()
    for kind, single, lo, hi in REG.findall(text):
        if single:
            out.add(f"{kind}{single}")
        else:
            out.update(f"{kind}{r}" for r in range(int(lo), int(hi) + 1))
    return out


def disasm(lib, pattern):
    with tempfile.TemporaryDirectory() as td:
        for k, co in enumerate(KR.code_objects(lib)):
            p = os.path.join(td, f"co{k}")
            open(p, "wb").write(co)
            out = subprocess.run([f"{KR.LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", p], capture_output=True,
                                 text=True, check=True).stdout
            fn, insts = None, []
            for line in out.splitlines():
                m = re.match(r"^[0-9a-f]+ <(.*)>:", line)
                if m:
                    if fn and insts:
                        return fn, insts
                    fn = m.group(1) if re.search(pattern, m.group(1)) else None
                    insts = []
                    continue
                if fn and line.startswith("\t"):
                    code, _, com = line.partition("//")
                    a = re.match(r"\s*([0-9A-Fa-f]+):", com)
                    t = code.strip()
                    if t and a:
                        insts.append((int(a.group(1), 16), t))
            if fn and insts:
                return fn, insts
    return None, []


def operands(t):
    op, _, rest = t.partition(" ")
    parts = [p.strip() for p in rest.split(",")] if rest.strip() else []
    if op.startswith(("ds_bpermute", "ds_permute", "ds_swizzle", "ds_read", "ds_add_rtn")):
        dst, src = regs(parts[0]), parts[1:]
    elif op.startswith(NO_DST):
        dst, src = set(), parts
    else:   # (a scalar second destination, e.g. v_mad_u64_u32's carry, holds no vector register)
        dst, src = (regs(parts[0]) if parts else set()), parts[1:]
    rd = set()
    for p in src:
        rd |= regs(p.split(" ")[0])
    if op.startswith(READS_DST) and not op.startswith("v_mfma"):
        rd |= dst
    return op, dst, rd


def analyse(insts):
    n = len(insts)
    addr_idx = {a: i for i, (a, _) in enumerate(insts)}
    succ = [[] for _ in range(n)]
    pc = add = None   # long branches: s_getpc_b64 s[x:y]; s_add_u32 sx, sx, IMM; s_addc_u32 ...; s_setpc_b64 s[x:y]
    for i, (a, t) in enumerate(insts):
        op = t.split()[0]
        if op == "s_getpc_b64":
            pc, add = a + 4, None
        elif op == "s_add_u32" and pc is not None and add is None:
            add = int(t.split(",")[2].strip(), 0)
            add = add - (1 << 32) if add >= (1 << 31) else add
        if op == "s_setpc_b64":
            if pc is not None and add is not None and (pc + add) in addr_idx:
                succ[i].append(addr_idx[pc + add])
            else:
                raise SystemExit(f"unresolved s_setpc at {a:#x}")
            pc = add = None
            continue
        if op.startswith(("s_branch", "s_cbranch")):
            off = int(t.split()[1])
            if off >= 32768:
                off -= 65536
            tgt = a + 4 + 4 * off
            # a divergent if / else (EXEC-masked arms) runs both arms in program order for some lanes:
            # s_cbranch_execz only skips an arm with no lane, so it is followed by its fall-through only
            if tgt in addr_idx and not (DIVERGENT_FALLTHROUGH and op == "s_cbranch_execz"):
                succ[i].append(addr_idx[tgt])
            if op.startswith("s_cbranch") and i + 1 < n:
                succ[i].append(i + 1)
        elif op.startswith("s_endpgm"):
            pass
        elif i + 1 < n:
            succ[i].append(i + 1)
    parsed = [operands(t) for _, t in insts]
    ALL = None   # "top" (unvisited)
    IN = [ALL] * n
    IN[0] = frozenset({"v0"})
    work = [0]
    while work:
        i = work.pop()
        cur = IN[i] | parsed[i][1]
        for j in succ[i]:
            new = cur if IN[j] is ALL else (IN[j] & cur)
            if IN[j] is ALL or new != IN[j]:
                IN[j] = frozenset(new)
                work.append(j)
    out = []
    for i, (a, t) in enumerate(insts):
        if IN[i] is ALL:
            continue
        miss = sorted(parsed[i][2] - IN[i], key=lambda r: (r[0], int(r[1:])))
        if miss:
            out.append((i, a, t, miss))
    return out


def main():
    lib, pat = sys.argv[1], sys.argv[2]
    fn, insts = disasm(lib, pat)
    print(fn, len(insts), "instructions")
    for i, a, t, miss in analyse(insts):
        print(f"{i:6d} {a:#x}: {t[:90]:90s} uninit {miss}")


if __name__ == "__main__":
    main()
