"""ISA checks of the shipped kernels (CPU; disassembles libecnf_hip.so's gfx950 code objects with llvm-objdump).

1. No data hazard around an inline-asm instruction (tools/isa_hazards.py: the fused DPP segment scans of
   SegScan::sum_fused and the fp16 residual split of split_pair; LLVM's hazard recognizer does not look inside inline
   asm, so these wait states are the source's responsibility).
2. No vector write where EXEC is zero (tools/isa_exec_copies.py): the cause of the round-4/5 aggregation fault
   (DESIGN 5.4).  In the failing (128, 2, 3) tangent vf_kernel builds the compiler placed five register-allocation
   copies (`v_accvgpr_write_b32 a26, v23`, ...) at the head of a loop-exit block that only s_cbranch_execz enters,
   BEFORE the block's `s_or_b64 exec, exec, s[..]`: with EXEC = 0 they write no lane, and the block loop later reads
   a26 back (a per-lane value computed at kernel entry), i.e. whatever the previous wave left in the register.
   Proven on the GPU: the build's results follow the register contents at launch (registers poisoned with 0 / NaN /
   1.0 give 0.1497849 / NaN / NaN, tools/diag/poison.hip); zeroing register subsets at the kernel entry spells a26
   (index 282); moving the EXEC restore above the five copies in that build's assembly, nothing else changed, makes
   every case correct (tools/diag/asm_swap.py asm_ds_fix); and the same ds_add_f32 atomics swapped into the passing
   build's schedule are correct (asm_p2ds).  The atomic form was never the cause, only the register allocation it led
   to.  This check flags the pattern in any kernel of the shipped library.
3. The message aggregation's LDS atomics are ds_add_f32 with the row offsets in the instruction at M = 64 and 256
   (round 5: the form is correct, item 2 was the fault, and it is faster there than the flat_atomic_add_f32 form the
   product used in rounds 4-5; M = 128 stays flat, equally fast, since the ds form hits item 2's miscompile in one of
   its kernels).  A run of 16 consecutive ds_add_f32 is that aggregation; the shift sums (dxacc) issue at most 2 D
   per site.
"""
import os
import re
import shutil
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import isa_exec_copies as XC  # noqa: E402
import isa_hazards as IH  # noqa: E402
import kernel_resources as KR  # noqa: E402

pytestmark = pytest.mark.skipif(not (os.path.exists(KR.LIB) and os.path.exists(f"{KR.LLVM}/llvm-objdump")),
                                reason="needs the built library and the ROCm LLVM tools")


@pytest.fixture(scope="module")
def disassembly():
    cos = KR.code_objects(KR.LIB)
    assert cos, "no gfx950 code objects in the library"
    td = tempfile.mkdtemp()

    def dis(k_co):
        k, co = k_co
        p = os.path.join(td, f"co{k}")
        open(p, "wb").write(co)
        out = subprocess.run([f"{KR.LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", p], capture_output=True, text=True,
                             check=True).stdout
        open(p + ".s", "w").write(out)
        return p + ".s"

    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 4)) as ex:
        paths = list(ex.map(dis, enumerate(cos)))
    yield paths
    shutil.rmtree(td, ignore_errors=True)


def test_no_inline_asm_hazards(disassembly):
    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 4)) as ex:
        found = sum(ex.map(lambda p: IH.check(IH.parse(p)), disassembly), [])
    n_asm = sum(open(p).read().count("v_fmac_f32_dpp") for p in disassembly)
    assert n_asm > 1000, "expected the fused DPP scans in the kernels"
    msg = [f"{k}: {d} wait states (need {IH.NEED[k]}): line {a.line} {a.text} -> line {b.line} {b.text}"
           for k, a, b, d in found[:10]]
    assert not found, "\n".join(msg)


def test_no_vector_writes_under_zero_exec():
    found = []
    fns = XC.functions(KR.LIB)
    assert len(fns) > 20, "expected the library's kernels"
    for fn, insts in fns.items():
        found += [(fn, hex(a), w, r) for a, w, r in XC.check(insts)]
    assert not found, found[:5]


def test_aggregation_atomics_are_ds_add(disassembly):
    """the batch kernels' aggregation is 16 consecutive ds_add_f32 per block row (item 3)"""
    runs = {}
    for p in disassembly:
        fn, run = None, 0
        for line in open(p):
            m = re.match(r"^[0-9a-f]+ <(.*)>:", line)
            if m:
                fn, run = m.group(1), 0
                continue
            if "ds_add_f32" in line:
                run += 1
                runs[fn] = max(runs.get(fn, 0), run)
            elif line.startswith("\t"):
                run = 0
    agg = [f for f, r in runs.items() if r >= 16]
    assert any("vf_kernel" in f for f in agg) and any("integrate_kernel" in f for f in agg), sorted(runs.items())[:5]


def test_integrate_kernels_never_touch_scratch(disassembly):
    """No spill or private-memory access in any split-precision (P = 0) integrate kernel's ISA (the solve loop keeps
    everything in registers and LDS; test_kernel_resources.py reads the reserved private-segment sizes, which can be
    non-zero and unreferenced): no scratch_* instruction and, outside the team kernels (whose exchange stores are
    buffer stores), no buffer store (the batch kernels' only buffer instructions are the weight-fragment loads, so a
    buffer store would be a spill through the scratch descriptor).  The strict-fp32
    comparator kernels (P = 1) keep their bounded spills."""
    bad = {}
    for p in disassembly:
        fn = None
        for line in open(p):
            m = re.match(r"^[0-9a-f]+ <(.*)>:", line)
            if m:
                fn = m.group(1)
                continue
            split = fn and re.search(r"integrate_kernelILi\d+ELi\d+ELi\d+ELi\d+ELi0E", fn)
            team = fn and re.search(r"ELi0ELb1E", fn)   # the team exchange's write-through stores are buffer stores
            if split and re.search(r"\bscratch_(load|store)" if team else r"\b(scratch_(load|store)|buffer_store)", line):
                bad[fn] = bad.get(fn, 0) + 1
    assert not bad, bad


def test_exec_copy_checker_known_answers():
    """tools/isa_exec_copies.check on hand-written blocks.  Flagged: vector writes ahead of the first EXEC write of a
    block entered only with EXEC = 0, for every EXEC-write idiom (s_or_b64 with exec as either source, s_mov_b64 exec,
    the saveexec family, v_cmpx), however far down the block it sits, and for both zero-EXEC entries (s_cbranch_execz,
    and the not-taken fall-through of s_cbranch_execnz that exits a divergent loop).  Not flagged: lane writes,
    writes after the EXEC write, and blocks also entered with live lanes (a plain fall-through or another branch)."""
    def prog(block, guard="s_cbranch_execz 1"):
        # 0x0: s_and_saveexec; 0x4: the guard branch -> 0xc; 0x8: s_endpgm (so 0xc has no fall-through)
        head = [(0x0, "s_and_saveexec_b64 s[4:5], vcc"), (0x4, guard), (0x8, "s_endpgm")]
        return head + [(0xc + 4 * k, t) for k, t in enumerate(block)]

    copy = "v_accvgpr_write_b32 a26, v23"
    restores = ["s_or_b64 exec, exec, s[4:5]", "s_or_b64 exec, s[4:5], exec", "s_mov_b64 exec, s[4:5]",
                "s_or_saveexec_b64 s[6:7], s[4:5]", "s_xor_b64 exec, exec, s[4:5]", "s_and_saveexec_b64 s[6:7], vcc",
                "v_cmpx_gt_f32_e32 vcc, 0, v1"]
    for r in restores:
        found = XC.check(prog([copy, r, "v_accvgpr_read_b32 v23, a26"]))
        assert len(found) == 1 and found[0][1] == [copy] and found[0][2] == r and found[0][3] == "execz", (r, found)
    # the whole block is scanned (the round-5 checker stopped after 64 instructions)
    long_block = [copy] + ["s_nop 0"] * 200 + ["v_mov_b32_e32 v1, v2", restores[2]]
    found = XC.check(prog(long_block))
    assert len(found) == 1 and found[0][1] == [copy, "v_mov_b32_e32 v1, v2"]
    # a block with no EXEC write before its end is scanned to its terminator
    assert XC.check(prog([copy, "s_endpgm"]))[0][2] == "s_endpgm"
    # loop exit: the fall-through of a not-taken s_cbranch_execnz (the last iteration cleared EXEC)
    loop = [(0x0, "v_add_f32_e32 v1, v2, v3"), (0x4, "s_andn2_b64 exec, exec, vcc"), (0x8, "s_cbranch_execnz 65533"),
            (0xc, copy), (0x10, "s_or_b64 exec, exec, s[4:5]")]
    found = XC.check(loop)
    assert len(found) == 1 and found[0][0] == 0xc and found[0][3] == "execnz-fallthrough"
    # not flagged
    assert not XC.check(prog(["s_or_b64 exec, exec, s[4:5]", copy]))
    assert not XC.check(prog(["v_writelane_b32 v253, s3, 0", "s_or_b64 exec, exec, s[4:5]"]))
    assert not XC.check(prog(["s_nop 0", "s_or_b64 exec, exec, s[4:5]"]))
    live_ft = [(0x0, "s_and_saveexec_b64 s[4:5], vcc"), (0x4, "s_cbranch_execz 0"), (0x8, copy),
               (0xc, "s_or_b64 exec, exec, s[4:5]")]
    assert not XC.check(live_ft)   # also entered by the fall-through of the execz guard (live lanes)
    both = prog([copy, "s_or_b64 exec, exec, s[4:5]"]) + [(0x14, "s_cbranch_vccnz 65533")]
    assert not XC.check(both)      # also the target of a branch on VCC (live lanes)
