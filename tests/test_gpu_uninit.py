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


@pytest.mark.timeout(240)
def test_redealt_adaptive_solve_does_not_depend_on_stale_state(poison):
    """The re-dealt adaptive solve (two launches, tests/test_gpu_redeal.py): the second launch loads the stored state of
    its occupied slots only, so the padding slots of its last workgroup (slots past the unfinished count) must start
    from the kernel's zero fill of the eval AND solver LDS, not from whatever the previous launch or a poison pattern
    left there.  ALDP B = 1101 PID sample_cnf (several molecules per workgroup; the engine passes a workspace, so the
    solve is re-dealt, asserted through ecnf_integrate_plan), bitwise equal under a zero and a NaN fill."""
    cfg = CONFIGS["aldp"]
    h = EcnfHandle(cfg, init_params(cfg, 0), 0)
    B = 1101
    opts = SolveOptions("dopri5", None)
    wg, launches = h.integrate_plan(B, 0.0, 1.0, opts, _lib.DIV_NONE)
    assert launches == 2 and wg < B, (wg, launches)   # re-dealt, more than one molecule per workgroup
    g = torch.Generator("cuda").manual_seed(9)
    z = torch.randn((B, cfg.event_dim), device="cuda", generator=g)
    x = h.base_sample(z)
    feat = (torch.arange(cfg.n_nodes, device="cuda", dtype=torch.int32) % cfg.n_features).expand(B, -1).contiguous()
    outs = []
    for bits in (0x00000000, 0x7FC00000):
        poison(bits)
        y, _, nfe, st = h.integrate(x, feat, 0.0, 1.0, opts, _lib.DIV_NONE, None, check_status=False)
        torch.cuda.synchronize()
        outs.append((y, nfe, st))
    for p, q in zip(*outs):
        assert torch.equal(p, q)
    assert int(outs[0][2].abs().sum()) == 0 and bool(torch.isfinite(outs[0][0]).all())
    h.close()


@pytest.mark.timeout(240)
def test_stop_and_team_solve_does_not_depend_on_stale_state(poison):
    """The three-launch Hutchinson log_prob: the tail-team second launch stops early and the third launch
    resumes every survivor as a team of four, each member zero-filling its eval and solver LDS before it loads the stored
    state and tangent rows.  ALDP B = 512 PID Hutchinson, asserted three launches, bitwise equal under a zero and a NaN
    fill."""
    cfg = CONFIGS["aldp"]
    h = EcnfHandle(cfg, init_params(cfg, 0), 0)
    B = 512
    opts = SolveOptions("dopri5", None)
    wg, launches = h.integrate_plan(B, 1.0, 0.0, opts, _lib.DIV_HUTCHINSON)
    assert launches == 3, (wg, launches)
    g = torch.Generator("cuda").manual_seed(11)
    z = torch.randn((B, cfg.event_dim), device="cuda", generator=g)
    x = h.base_sample(z)
    feat = (torch.arange(cfg.n_nodes, device="cuda", dtype=torch.int32) % cfg.n_features).expand(B, -1).contiguous()
    eps = torch.randn((B, cfg.event_dim), device="cuda", generator=g)
    outs = []
    for bits in (0x00000000, 0x7FC00000):
        poison(bits)
        y, dl, nfe, st = h.integrate(x, feat, 1.0, 0.0, opts, _lib.DIV_HUTCHINSON, eps, check_status=False)
        torch.cuda.synchronize()
        outs.append((y, dl, nfe, st))
    for p, q in zip(*outs):
        assert torch.equal(p, q)
    assert int(outs[0][3].abs().sum()) == 0 and bool(torch.isfinite(outs[0][1]).all())
    h.close()
