"""Scan a gfx950 disassembly for the data hazards that the compiler's hazard recognizer does not see because one side of
the dependency is an inline-asm instruction (the DPP segment scans `v_fmac_f32_dpp` of SegScan::sum_fused, the fp16
residual `v_fma_mix{lo,hi}_f16` of split_pair).  LLVM's GCNHazardRecognizer only inspects inline asm for the 12-dword
store and dst-sel forwarding hazards; every other wait-state requirement around an asm statement is the source's job.

Checked (wait states = instructions between producer and consumer, s_nop N counting N + 1; straight-line only, a
branch or label ends the window):
  raw_xdl   an XDL MFMA writes a VGPR that an asm instruction reads            need >= 12 (8-pass 32x32x16 on gfx950)
  raw_dpp   a VALU writes a VGPR that an asm DPP instruction reads as src0     need >= 2
  raw_exec  an EXEC write before an asm DPP instruction                        need >= 5
  raw_trans a transcendental writes a VGPR that an asm instruction reads       need >= 1
  asm_mfma  an asm instruction writes a VGPR that an MFMA reads                need >= 2
  asm_dpp   an asm instruction writes a VGPR that a (compiler) DPP reads       need >= 2
  asm_rdln  an asm instruction writes a VGPR that v_readlane / v_readfirstlane reads   need >= 1
  war_xdl   an asm instruction overwrites a VGPR an in-flight XDL MFMA reads as SrcC   need >= 11
            (SrcA / SrcB are read in the MFMA's first pass: no WAR requirement)

Usage: python tools/isa_hazards.py FILE.s [FUNCTION_SUBSTRING]   (llvm-objdump -d --mcpu=gfx950 output)
Exit status 1 if any hazard is found.  tests/test_isa_hazards.py runs it on the built library's kernels.
"""
from __future__ import annotations

import re
import sys

REG = re.compile(r"\b([va])(?:(\d+)|\[(\d+):(\d+)\])")
NEED = {"raw_xdl": 12, "raw_dpp": 2, "raw_exec": 5, "raw_trans": 1, "asm_mfma": 2, "asm_dpp": 2, "asm_rdln": 1,
        "war_xdl": 11}
TRANS = ("v_exp_", "v_log_", "v_rcp_", "v_rsq_", "v_sqrt_", "v_sin_", "v_cos_")
THROUGH_CBRANCH = False   # --through-cbranch: conditional branches do not end a window (their fall-through path)
ASM_OPS = ("v_fmac_f32_dpp", "v_fma_mixlo_f16", "v_fma_mixhi_f16")


def regs(text):
    out = set()
    for kind, single, lo, hi in REG.findall(text):
        if single:
            out.add((kind, int(single)))
        else:
            out.update((kind, r) for r in range(int(lo), int(hi) + 1))
    return out


class Inst:
    __slots__ = ("op", "dst", "src", "srcc", "text", "line", "ws", "is_asm", "xdl", "dpp", "barrier")

    def __init__(self, op, operands, text, line):
        self.op, self.text, self.line = op, text, line
        parts = [p.strip() for p in operands.split(",")] if operands else []
        no_dst = op.startswith(("ds_write", "ds_add", "buffer_store", "global_store", "flat_store", "flat_atomic",
                                "global_atomic", "buffer_atomic", "s_", "v_cmp"))
        if op.startswith("v_mad_u64_u32") or op.startswith("v_div_scale"):
            self.dst, src = regs(parts[0]), parts[2:]
        elif no_dst:
            self.dst, src = set(), parts
        else:
            self.dst, src = (regs(parts[0]) if parts else set()), parts[1:]
        self.src = set()
        for p in src:
            self.src |= regs(p.split(" ")[0])
        self.ws = 1
        m = re.match(r"s_nop (\d+)", text)
        if m:
            self.ws = int(m.group(1)) + 1
        self.xdl = op.startswith("v_mfma")
        self.srcc = regs(parts[3].split(" ")[0]) if self.xdl and len(parts) > 3 else set()
        self.dpp = "_dpp" in op or " row_" in text or "quad_perm" in text
        self.is_asm = op in ASM_OPS
        self.barrier = op.startswith(("s_cbranch", "s_branch", "s_setpc", "s_swappc", "s_endpgm"))
        if THROUGH_CBRANCH and op.startswith("s_cbranch"):
            self.barrier = False   # the fall-through path continues the window


def parse(path, func=None):
    insts, cur, keep = [], None, func is None
    for n, raw in enumerate(open(path), 1):
        line = raw.split("//")[0].rstrip()
        if re.match(r"^[0-9a-f]+ <", line):
            keep = func is None or func in line
            insts.append(None)   # function boundary
            continue
        if not keep or not line.startswith("\t"):
            if line.strip().endswith(":"):
                insts.append(None)
            continue
        t = line.strip()
        op, _, rest = t.partition(" ")
        insts.append(Inst(op, rest.strip(), t, n))
    return insts


def check(insts):
    found = []

    def window_back(i):
        d = 0
        for j in range(i - 1, max(-1, i - 40), -1):
            x = insts[j]
            if x is None or x.barrier:
                return
            yield x, d
            d += x.ws

    def window_fwd(i):
        d = 0
        for j in range(i + 1, min(len(insts), i + 40)):
            x = insts[j]
            if x is None or x.barrier:
                return
            yield x, d
            d += x.ws

    for i, x in enumerate(insts):
        if x is None or not x.is_asm:
            continue
        # producers of what the asm reads
        reads = set(x.src) | (x.dst if x.op.startswith("v_fmac") else set())
        dpp_src0 = set()
        if x.op == "v_fmac_f32_dpp":
            ops = x.text.split(None, 1)[1].split(",")
            dpp_src0 = regs(ops[1].split(" ")[0])
        for y, d in window_back(i):
            if y.is_asm:
                continue
            if y.xdl and y.dst & reads and d < NEED["raw_xdl"]:
                found.append(("raw_xdl", y, x, d))
            if x.dpp and not y.xdl and y.dst & dpp_src0 and d < NEED["raw_dpp"]:
                found.append(("raw_dpp", y, x, d))
            if x.dpp and "exec" in y.text.split(",")[0] and d < NEED["raw_exec"]:
                found.append(("raw_exec", y, x, d))
            if y.op.startswith(TRANS) and y.dst & reads and d < NEED["raw_trans"]:
                found.append(("raw_trans", y, x, d))
            if y.xdl and y.srcc & x.dst and d < NEED["war_xdl"]:
                found.append(("war_xdl", y, x, d))
        # consumers of what the asm writes
        for y, d in window_fwd(i):
            if y.is_asm:
                continue
            if y.xdl and y.src & x.dst and d < NEED["asm_mfma"]:
                found.append(("asm_mfma", x, y, d))
            if y.dpp and y.src & x.dst and d < NEED["asm_dpp"]:
                found.append(("asm_dpp", x, y, d))
            if y.op.startswith(("v_readlane", "v_readfirstlane")) and y.src & x.dst and d < NEED["asm_rdln"]:
                found.append(("asm_rdln", x, y, d))
    return found


def main(argv):
    global THROUGH_CBRANCH
    if "--through-cbranch" in argv:
        THROUGH_CBRANCH = True
        argv = [a for a in argv if a != "--through-cbranch"]
    path = argv[1]
    func = argv[2] if len(argv) > 2 else None
    found = check(parse(path, func))
    for kind, a, b, d in found:
        print(f"{kind}: {d} wait states (need {NEED[kind]})\n   line {a.line}: {a.text}\n   line {b.line}: {b.text}")
    print(f"{len(found)} hazards")
    return 1 if found else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
