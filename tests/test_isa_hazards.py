"""ISA checks of the shipped kernels (CPU; disassembles libecnf_hip.so's gfx950 code objects with llvm-objdump).

1. No data hazard around an inline-asm instruction (tools/isa_hazards.py: the fused DPP segment scans of
   SegScan::sum_fused and the fp16 residual split of split_pair; LLVM's hazard recognizer does not look inside inline
   asm, so these wait states are the source's responsibility).
2. The message aggregation's LDS atomics stay in the validated flat form.  Rounds 4 and 5 saw NaN fields
   and faults in single-shape builds of the (128, 2, 3) tangent vf_kernel, first attributed to the ds_add_f32 form of
   this aggregation; round 5 found that failing build's kernel byte-identical to the passing one (flat atomics in
   both), but also a current-source reproducer: both aggregation sites of that kernel in ds_add_f32 form return wrong
   fields (a different value in every process) while either site alone, or both flat, is correct
   (tools/diag/ds_agg_variants.py).  Not root-caused; the validated flat form is kept.
   A run of 8 or more consecutive ds_add_f32 is that aggregation; the shift sums (dxacc) issue at most 2 D per site.
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


def test_aggregation_atomics_are_flat(disassembly):
    bad, flat_kernels = [], 0
    for p in disassembly:
        fn, run, best = None, 0, {}
        for line in open(p):
            m = re.match(r"^[0-9a-f]+ <(.*)>:", line)
            if m:
                fn, run = m.group(1), 0
                continue
            if "ds_add_f32" in line:
                run += 1
                best[fn] = max(best.get(fn, 0), run)
            elif line.startswith("\t"):
                run = 0
            if "flat_atomic_add_f32" in line and fn is not None:
                best.setdefault(fn, 0)
        for f, r in best.items():
            if r >= 8:
                bad.append(f"{f}: a run of {r} ds_add_f32")
        flat_kernels += sum(1 for f in best)
    assert flat_kernels > 0
    assert not bad, "\n".join(bad[:10])


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
