"""Chunked, re-dealt adaptive solves (csrc/ecnf_hip.hip redeal_kernel, SolveP::resume / chunk_steps): when an
adaptive Dopri5 solve has more workgroups than the device has CUs and the workspace holds the scratch, the first launch
runs every molecule for kChunkSteps step controls and stores its solver state, one workgroup sorts the unfinished
molecules by their estimated remaining steps, and a second launch resumes them longest first.  A molecule's arithmetic
does not depend on its slot and its state crosses the launches exactly, so the results must be BITWISE those of the
one-launch solve (the same C call without a workspace), outputs in batch order.  Reference: the per-molecule adaptive
solves of diffrax under vmap (sample_and_log_prob.py:81-94), which the batch path restates."""
import ctypes

import pytest
import torch

from ecnf_amd import CONFIGS, init_params, _lib
from ecnf_amd.engine import EcnfHandle, SolveOptions, _ptr, _stream

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs a ROCm GPU", allow_module_level=True)


def _solve(h, x0, feat, eps, t0, t1, div, workspace, max_steps=4096):
    B = x0.shape[0]
    o = SolveOptions("dopri5", None, max_steps=max_steps).to_c(t0, t1, div)
    nbytes = ctypes.c_size_t(0)
    _lib.check(h.lib.ecnf_integrate_workspace_size(h._h, ctypes.byref(o), B, ctypes.byref(nbytes)))
    ws = torch.empty(nbytes.value, device="cuda", dtype=torch.uint8) if (workspace and nbytes.value) else None
    y1 = torch.empty_like(x0)
    dl = torch.empty(B, device="cuda") if div != _lib.DIV_NONE else None
    nfe = torch.empty(B, device="cuda", dtype=torch.int32)
    st = torch.empty(B, device="cuda", dtype=torch.int32)
    _lib.check(h.lib.ecnf_integrate_ws(h._h, ctypes.byref(o), _ptr(x0), _ptr(feat), _ptr(eps), _ptr(y1), _ptr(dl),
                                       _ptr(nfe), _ptr(st), B, _ptr(ws), nbytes.value if ws is not None else 0,
                                       _stream(h.device)))
    torch.cuda.synchronize()
    return y1, dl, nfe, st, nbytes.value


@pytest.mark.timeout(240)
@pytest.mark.parametrize("name,B,div", [("aldp", 512, _lib.DIV_HUTCHINSON), ("aldp", 1100, _lib.DIV_NONE),
                                        ("lj13", 1024, _lib.DIV_HUTCHINSON),
                                        ("aldp", 5000, _lib.DIV_NONE)])   # > 4096: the sort in the workspace
def test_redealt_solve_is_bitwise_the_one_launch_solve(name, B, div):
    cfg = CONFIGS[name]
    h = EcnfHandle(cfg, init_params(cfg, 0), 0)
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    mpw = h.molecules_per_workgroup(div != _lib.DIV_NONE)
    g = torch.Generator("cuda").manual_seed(7)
    z = torch.randn((B, cfg.event_dim), device="cuda", generator=g)
    x0 = h.base_sample(z)
    feat = (torch.arange(cfg.n_nodes, device="cuda", dtype=torch.int32) % cfg.n_features).expand(B, -1).contiguous()
    eps = torch.randn((B, cfg.event_dim), device="cuda", generator=g) if div == _lib.DIV_HUTCHINSON else None
    t0, t1 = (1.0, 0.0) if div != _lib.DIV_NONE else (0.0, 1.0)
    one = _solve(h, x0, feat, eps, t0, t1, div, workspace=False)
    red = _solve(h, x0, feat, eps, t0, t1, div, workspace=True)
    assert red[4] > 0, "an adaptive solve asks for the re-deal scratch"
    wg, launches = h.integrate_plan(B, t0, t1, SolveOptions("dopri5", None), div)
    print(f"{name} B={B}: handle MPW {mpw}, {wg} workgroups, {launches} launches, {ncu} CUs, NFE max {int(one[2].max())}")
    # the case really is the re-dealt form (the grid net_for_batch picks exceeds the CU count), not one vs one; ALDP's
    # Hutchinson solves add the tail teams and the stop-and-team launch (3 launches)
    assert wg > ncu and launches == (3 if (name, div) == ("aldp", _lib.DIV_HUTCHINSON) else 2), (wg, launches, ncu)
    assert int(one[3].abs().sum()) == 0
    assert torch.equal(red[0], one[0])
    assert torch.equal(red[2], one[2])
    assert torch.equal(red[3], one[3])
    if div != _lib.DIV_NONE:
        assert torch.equal(red[1], one[1])
    # the engine's call (workspace from the caching allocator) is the re-dealt form
    y, dl, nfe, st = h.integrate(x0, feat, t0, t1, SolveOptions("dopri5", None), div, eps)
    assert torch.equal(y, one[0]) and torch.equal(nfe, one[2])
    h.close()


@pytest.mark.timeout(240)
def test_redealt_solve_statuses():
    """Per-molecule statuses through the two launches: molecules that exceed max_steps inside the first launch (4 steps)
    or the second (12), and molecules with embedding ids out of range (ECNF_E_INVALID, solved with id 0), end
    bitwise as in one launch."""
    cfg = CONFIGS["aldp"]
    h = EcnfHandle(cfg, init_params(cfg, 0), 0)
    B = 512
    g = torch.Generator("cuda").manual_seed(11)
    z = torch.randn((B, cfg.event_dim), device="cuda", generator=g)
    x0 = h.base_sample(z)
    feat = (torch.arange(cfg.n_nodes, device="cuda", dtype=torch.int32) % cfg.n_features).expand(B, -1).contiguous()
    feat[5, 3] = cfg.n_features + 4
    feat[300, 0] = -1
    eps = torch.randn((B, cfg.event_dim), device="cuda", generator=g)
    for max_steps in (4, 12):
        one = _solve(h, x0, feat, eps, 1.0, 0.0, _lib.DIV_HUTCHINSON, False, max_steps)
        red = _solve(h, x0, feat, eps, 1.0, 0.0, _lib.DIV_HUTCHINSON, True, max_steps)
        st = one[3].cpu()
        # (a molecule that also runs out of steps reports ECNF_E_MAX_STEPS, the later of the two)
        assert int(st[5]) in (_lib.ECNF_E_INVALID, _lib.ECNF_E_MAX_STEPS) and int(st[300]) != _lib.ECNF_OK
        assert int((st == _lib.ECNF_E_MAX_STEPS).sum()) > 0
        for a, b in zip(one[:4], red[:4]):
            assert torch.equal(a, b)
    h.close()


@pytest.mark.timeout(120)
def test_fixed_step_solves_need_no_redeal_scratch():
    cfg = CONFIGS["aldp"]
    h = EcnfHandle(cfg, init_params(cfg, 0), 0)
    for opts, div in ((SolveOptions("euler", 0.05), _lib.DIV_HUTCHINSON), (SolveOptions("dopri5", 0.1), _lib.DIV_NONE)):
        o = opts.to_c(1.0, 0.0, div)
        nbytes = ctypes.c_size_t(1)
        _lib.check(h.lib.ecnf_integrate_workspace_size(h._h, ctypes.byref(o), 512, ctypes.byref(nbytes)))
        assert nbytes.value == 0
    h.close()
