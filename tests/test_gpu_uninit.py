"""No shipped kernel reads a register or LDS word it never wrote.  The round-4/5 aggregation fault was a
compiler miscompile of exactly that kind: register copies placed where EXEC is 0, read back later as whatever the
previous wave left in the register (tests/test_isa_hazards.py checks the ISA for that pattern).  Here every SIMD's
VGPRs / AGPRs and the LDS are filled with a NaN pattern right before each launch (tools/diag/poison.hip, built by
__graft_entry__.build()), and the results must be BITWISE those of a launch after a zero pattern: the vector field, the
JVP and a short Hutchinson solve of every BASELINE network (DW4, LJ13, ALDP, QM9), split and strict-fp32 kernels.
(Bitwise: a node's aggregate has at most two atomic contributions, 0 + a + b = 0 + b + a.)"""
import ctypes
import os

import pytest
import torch

from ecnf_amd import CONFIGS, init_params, _lib
from ecnf_amd.engine import EcnfHandle, SolveOptions

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs a ROCm GPU", allow_module_level=True)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PLIB = os.path.join(ROOT, "tools", "diag", "libpoison.so")


@pytest.fixture(scope="module")
def poison():
    assert os.path.exists(PLIB), "tools/diag/libpoison.so is built by __graft_entry__.build()"
    lib = ctypes.CDLL(PLIB)

    def fill(bits):
        torch.cuda.synchronize()
        assert lib.poison_launch(ctypes.c_uint(bits), 4096, 3) == 0

    return fill


def _run(h, cfg, B, fill, bits):
    g = torch.Generator("cuda").manual_seed(5)
    z = torch.randn((B, cfg.event_dim), device="cuda", generator=g)
    x = h.base_sample(z)
    t = torch.rand(B, device="cuda", generator=g)
    feat = (torch.arange(cfg.n_nodes, device="cuda", dtype=torch.int32) % cfg.n_features).expand(B, -1).contiguous()
    u = torch.randn((B, 2, cfg.event_dim), device="cuda", generator=g)
    out = []
    fill(bits)
    out.append(h.vector_field(x, t, feat))
    fill(bits)
    out += list(h.jvp(x, t, feat, u))
    fill(bits)
    y, dl, nfe, st = h.integrate(x, feat, 1.0, 0.0, SolveOptions("euler", 0.25), _lib.DIV_HUTCHINSON, z,
                                 check_status=False)
    out += [y, dl, st]
    torch.cuda.synchronize()
    return out


@pytest.mark.timeout(240)
@pytest.mark.parametrize("name,B", [("dw4", 64), ("lj13", 64), ("aldp", 16), ("qm9", 8)])
@pytest.mark.parametrize("precision", ["split_f16", "fp32"])
def test_results_do_not_depend_on_stale_registers(poison, name, B, precision):
    cfg = CONFIGS[name]
    h = EcnfHandle(cfg, init_params(cfg, 0), 0)
    h.set_precision(precision)
    a = _run(h, cfg, B, poison, 0x00000000)
    b = _run(h, cfg, B, poison, 0x7FC00000)   # quiet NaN in every register and LDS word
    for k, (p, q) in enumerate(zip(a, b)):
        assert torch.equal(p, q), f"output {k} differs with poisoned registers / LDS"
    assert all(bool(torch.isfinite(p.float()).all()) for p in a[:5])
    h.close()
