"""Register budget of the shipped kernels (CPU; reads the AMDGPU metadata of libecnf_hip.so's gfx950 code objects via
tools/kernel_resources.py).  A kernel that spills to scratch in the solve loop loses most of its throughput: the M = 256
split primal kernel compiled at 2 waves per SIMD spilled 968 B per lane and QM9 B = 2048 Euler-100 ran 2162 -> 3423 ms
with every parity test still green, so the budget is pinned here."""
import os
import re
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import kernel_resources as KR  # noqa: E402

pytestmark = pytest.mark.skipif(not (os.path.exists(KR.LIB) and os.path.exists(f"{KR.LLVM}/llvm-readelf")
                                     and shutil.which("c++filt")),
                                reason="needs the built library and the ROCm LLVM tools")

# template arguments <NF, NT, L, D, P, ...> of integrate_kernel (TEAM, COLS, BN follow) / vf_kernel (BN follows).
# (Up to round 4 this pattern ended at the fifth argument with '>', which the integrate kernels' extra flags never
# matched: their scratch limits were not checked.)
SIG = re.compile(r"(integrate_kernel|vf_kernel)<(\d+), (\d+), (\d+), (\d+), (\d+)[,>]")


def _kernels():
    ks = KR.kernels()
    dm = KR.demangle(sorted(ks))
    out = []
    for name, rec in ks.items():
        m = SIG.search(dm[name])
        if m:
            out.append((m.group(1), *map(int, m.groups()[1:]), rec.get("private_segment_fixed_size", -1)))
    return out


def test_split_kernels_do_not_spill():
    ks = _kernels()
    assert len(ks) >= 80, "expected the integrate / vf kernels of every compiled shape"
    assert sum(k[0] == "integrate_kernel" for k in ks) >= 40
    bad = []
    for kind, nf, nt, l, d, p, scratch in ks:
        if p != 0:
            continue   # the strict-fp32 comparator kernels (8 waves of fp32 MFMA chains) are not budgeted here
        # Round 4: every split-precision integrate kernel (batch and team modes, primal and tangent, every M)
        # runs without scratch; the loop-invariant values that used to spill (division constants of runtime sizes,
        # the solver's sizes and control flags, the aggregation's lane addresses) are re-derived at their use sites
        # (opaque_u / solver_size / an opaque row offset).  vf_kernel (one evaluation, not the solve loop): the M = 64
        # tangent form keeps 28 B per lane outside its edge tiles (2 waves per SIMD at 256 registers); the split
        # primal forms report a 20 B private segment that no instruction of theirs addresses (no scratch_* in their
        # ISA, round 4)
        # The M = 256 tangent integrate kernels, and since round 5 (the re-dealt solves' state copies) the split primal
        # ones, report a 20 B private segment that, like the split primal vf_kernel's, no instruction addresses
        # (tests/test_isa_hazards.py: no scratch or buffer-store instruction in any split integrate kernel).
        limit = ((20 if (nt == 0 or nf == 8) else 0) if kind == "integrate_kernel" else 28 if (nf == 2 and nt == 1)
                 else 96 if (nf == 8 and nt == 1) else 20 if nt == 0 else 0)
        if scratch > limit:
            bad.append(f"{kind}<{nf},{nt},{l},{d},{p}> scratch {scratch} B/lane (limit {limit})")
    assert not bad, "\n".join(bad)


def test_strict_fp32_tangent_kernels_exist_for_every_shape():
    """Every compiled shape has tangent kernels at both precisions, M = 256 included (Geo::kWideT32, round 3: the
    strict-fp32 route for QM9 divergence solves and >= 2^15 weights).  Their sequential fp32 chain passes keep a
    bounded spill (364 B/lane at build time; the weight loads of the two passes must not be merged, which once
    spilled 4.3 KB/lane)."""
    ks = _kernels()
    shapes = {(nf, l, d) for kind, nf, nt, l, d, p, s in ks if kind == "integrate_kernel"}
    have = {(nf, nt, l, d, p) for kind, nf, nt, l, d, p, s in ks if kind == "integrate_kernel"}
    missing = [(nf, nt, l, d, p) for nf, l, d in shapes for nt in (0, 1) for p in (0, 1)
               if (nf, nt, l, d, p) not in have]
    assert not missing, missing
    wide32 = [(l, d, s) for kind, nf, nt, l, d, p, s in ks if nf == 8 and nt == 1 and p == 1]
    assert wide32 and all(s <= 512 for _, _, s in wide32), wide32
