"""The precision contract of the split-fp16 GEMM path, its failure detection and the strict-fp32 kernels.

Contract (include/ecnf.h ecnf_precision): ECNF_PREC_SPLIT_F16 computes every GEMM as three fp16 cross terms with fp32
accumulation and must be fp32-CLASS: its error against the fp64 oracle may be at most C = 4 times the error of a plain
fp32 evaluation of the same math (the numpy oracle with dtype=float32, the reference's x64-off arithmetic,
loop.py:62-63), plus 2e-7 x max|ref| for cases where the fp32 oracle happens to be nearly exact.  The strict-fp32
kernels (ECNF_PREC_FP32) are held to the same bound.  Activations beyond the fp16 range (|a| >= 65504) cannot be
split: such molecules must report ECNF_E_NONFINITE, never a silent ECNF_OK, and the host falls back to the fp32
kernels for them.
"""
import numpy as np
import pytest
import torch

from oracle import ecnf_oracle as O

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs a ROCm GPU", allow_module_level=True)

from ecnf_amd import CONFIGS  # noqa: E402
from ecnf_amd import _lib  # noqa: E402
from ecnf_amd.engine import EcnfHandle, SolveOptions  # noqa: E402

DEV = torch.device("cuda", 0)
C = 4.0
FLOOR = 2e-7


def g(a, dtype=torch.float32):
    return torch.as_tensor(np.asarray(a), device=DEV, dtype=dtype)


def _inputs(name, B, seed=0, stress=True):
    cfg = CONFIGS[name]
    oc = O.CONFIGS[name]
    p = O.init_params(oc, seed)
    if stress:
        p = O.stress_params(p, oc)
    rng = np.random.default_rng(seed + 11)
    z = rng.standard_normal((B, cfg.event_dim)).astype(np.float32)
    x0 = O.base_sample(z, oc)
    feat = rng.integers(0, cfg.n_features, (B, cfg.n_nodes)).astype(np.int32)
    return cfg, oc, p, x0, feat


def _check(name, got, ref64, ref32):
    scale = max(1.0, float(np.abs(ref64).max()))
    e_hip = float(np.abs(got - ref64).max())
    e_32 = float(np.abs(ref32 - ref64).max())
    print(f"{name}: |hip - fp64| = {e_hip:.3e}, |fp32 oracle - fp64| = {e_32:.3e}, ratio {e_hip / max(e_32, 1e-30):.2f}")
    assert e_hip <= C * e_32 + FLOOR * scale, (e_hip, e_32)


@pytest.mark.parametrize("name", ["dw4", "lj13", "aldp", "qm9"])
@pytest.mark.parametrize("precision", ["split_f16", "fp32"])
def test_eval_is_fp32_class(name, precision):
    cfg, oc, p, x0, feat = _inputs(name, 12)
    t = np.linspace(0.0, 1.0, 12).astype(np.float32)
    h = EcnfHandle(cfg, p, 0, precision=precision)
    assert h.chain_arithmetic() == ("split_f16" if precision == "split_f16" else "fp32_mfma")
    v = h.vector_field(g(x0), g(t), g(feat, torch.int32)).cpu().numpy()
    ref64 = O.egnn_vector_field(p, oc, x0, t, feat, dtype=np.float64)
    ref32 = O.egnn_vector_field(p, oc, x0, t, feat, dtype=np.float32)
    _check(f"{name}/{precision} eval", v, ref64, ref32)


@pytest.mark.parametrize("name,B,steps", [("lj13", 8, 100), ("dw4", 8, 100), ("aldp", 4, 25), ("qm9", 2, 5)])
def test_trajectory_is_fp32_class(name, B, steps):
    """Euler trajectories (the headline solver): the split kernel's end-point error vs fp64 within C x the fp32
    oracle's."""
    cfg, oc, p, x0, feat = _inputs(name, B)
    h = EcnfHandle(cfg, p, 0)
    y1, _, nfe, status = h.integrate(g(x0), g(feat, torch.int32), 0.0, 1.0, SolveOptions("euler", 1.0 / steps))
    assert (status.cpu().numpy() == 0).all() and (nfe.cpu().numpy() == steps).all()
    ref64, _ = O.sample_cnf(p, oc, x0, feat, solver="euler", dt0=1.0 / steps, dtype=np.float64)
    ref32, _ = O.sample_cnf(p, oc, x0, feat, solver="euler", dt0=1.0 / steps, dtype=np.float32)
    _check(f"{name} Euler-{steps}", y1.cpu().numpy(), ref64, ref32)


def test_jvp_is_fp32_class():
    cfg, oc, p, x0, feat = _inputs("lj13", 5)
    t = np.full(5, 0.4, np.float32)
    u = np.random.default_rng(5).standard_normal((5, 2, cfg.event_dim)).astype(np.float32)
    h = EcnfHandle(cfg, p, 0)
    _, ju = h.jvp(g(x0), g(t), g(feat, torch.int32), g(u))
    _, j64 = O.egnn_vector_field(p, oc, x0, t, feat, tangents=u, dtype=np.float64)
    _, j32 = O.egnn_vector_field(p, oc, x0, t, feat, tangents=u, dtype=np.float32)
    _check("lj13 jvp", ju.cpu().numpy(), j64, j32)


def _overflow_case():
    """LJ13 at the default init with molecule 1 scaled x1000 (edge pre-activations ~1e8, |r|^2 ~ 1e6 into phi_e.0:
    beyond fp16 for certain) and molecule 3 x100 (~1e5: near the fp16 limit, either outcome allowed), while plain
    fp32 stays accurate (the oracle's fp32 / fp64 agree to ~1e-6 of the displacement)."""
    cfg, oc, p, x0, feat = _inputs("lj13", 4, stress=False)
    x0 = x0.copy()
    x0[1] *= 1000.0
    x0[3] *= 100.0
    return cfg, oc, p, x0, feat


def _check_flags(st):
    assert st[0] == 0 and st[2] == 0 and st[1] == _lib.ECNF_E_NONFINITE, st
    assert st[3] in (0, _lib.ECNF_E_NONFINITE), st


def test_nonfinite_status_and_fp32_fallback():
    cfg, oc, p, x0, feat = _overflow_case()
    h = EcnfHandle(cfg, p, 0)
    opts = SolveOptions("euler", 0.5)
    y_raw, _, _, st = h.integrate(g(x0), g(feat, torch.int32), 0.0, 1.0, opts, check_status=False)
    st = st.cpu().numpy()
    _check_flags(st)
    ok = st == 0
    assert torch.isfinite(y_raw[torch.from_numpy(ok).cuda()]).all()
    # the host re-solves the flagged molecules on the strict-fp32 kernels (no CPU path)
    y, _, nfe, st2 = h.integrate(g(x0), g(feat, torch.int32), 0.0, 1.0, opts)
    assert (st2.cpu().numpy() == 0).all() and torch.isfinite(y).all()
    assert torch.equal(y[torch.from_numpy(ok).cuda()], y_raw[torch.from_numpy(ok).cuda()])
    ref64, _ = O.sample_cnf(p, oc, x0, feat, solver="euler", dt0=0.5, dtype=np.float64)
    ref32, _ = O.sample_cnf(p, oc, x0, feat, solver="euler", dt0=0.5, dtype=np.float32)
    # molecule 1 sits at |x| ~ 1e8 after the first step, where summation order alone moves fp32 results by ~1e-5
    # relative (the fp32 kernels: 1.8e-5, the numpy fp32 oracle: 1.7e-6): the bound is relative to |x| there
    e = np.abs(y.cpu().numpy() - ref64).max(axis=1)
    e32 = np.abs(ref32 - ref64).max(axis=1)
    scale = np.abs(ref64).max(axis=1)
    assert (e <= C * e32 + 3e-5 * scale).all(), (e, e32, scale)
    # fp32 handles directly: the same numbers, ECNF_OK
    h32 = EcnfHandle(cfg, p, 0, precision="fp32")
    y32, _, _, st3 = h32.integrate(g(x0[[1]]), g(feat[[1]], torch.int32), 0.0, 1.0, opts)
    assert torch.equal(y32, y[[1]]) and (st3.cpu().numpy() == 0).all()


def test_nonfinite_in_divergence_solve():
    cfg, oc, p, x0, feat = _overflow_case()
    h = EcnfHandle(cfg, p, 0)
    eps = np.random.default_rng(2).standard_normal(x0.shape).astype(np.float32)
    _, dl, _, st = h.integrate(g(x0), g(feat, torch.int32), 0.0, 1.0, SolveOptions("euler", 0.5),
                               divergence=_lib.DIV_HUTCHINSON, eps=g(eps), check_status=False)
    _check_flags(st.cpu().numpy())
    x1, dl2, _, st2 = h.integrate(g(x0), g(feat, torch.int32), 0.0, 1.0, SolveOptions("euler", 0.5),
                                  divergence=_lib.DIV_HUTCHINSON, eps=g(eps))
    assert (st2.cpu().numpy() == 0).all() and torch.isfinite(dl2).all()
    _, lq64, _ = O.sample_and_log_prob(p, oc, x0, feat, eps=eps, approx=True, solver="euler", dt0=0.5,
                                       dtype=np.float64)
    _, lq32, _ = O.sample_and_log_prob(p, oc, x0, feat, eps=eps, approx=True, solver="euler", dt0=0.5,
                                       dtype=np.float32)
    lq = (h.base_log_prob(g(x0)) - dl2).cpu().numpy()
    assert np.abs(lq - lq64).max() <= C * np.abs(lq32 - lq64).max() + 1e-5 * max(1.0, np.abs(lq64).max())


def test_device_feature_ids_checked_in_kernel():
    """Device-resident features are validated by the kernels (no host sync): an out-of-range id gives
    ECNF_E_INVALID from integrate (ValueError on the host) and NaN rows from the vector field; valid rows are
    unaffected (bitwise)."""
    cfg, oc, p, x0, feat = _inputs("aldp", 3)
    h = EcnfHandle(cfg, p, 0)
    t = g([0.2, 0.5, 0.7])
    fd = g(feat, torch.int32)
    v_ok = h.vector_field(g(x0), t, fd)
    bad = fd.clone()
    bad[1, 4] = cfg.n_features          # out of range, on the device
    v = h.vector_field(g(x0), t, bad)
    assert torch.isnan(v[1]).all() and torch.equal(v[[0, 2]], v_ok[[0, 2]])
    _, _, _, st = h.integrate(g(x0), bad, 0.0, 1.0, SolveOptions("euler", 0.25), check_status=False)
    assert list(st.cpu().numpy()) == [0, _lib.ECNF_E_INVALID, 0]
    with pytest.raises(ValueError):
        h.integrate(g(x0), bad, 0.0, 1.0, SolveOptions("euler", 0.25))
    with pytest.raises(ValueError):     # host features: checked before the upload
        h.vector_field(g(x0), t, np.full((3, cfg.n_nodes), -1, np.int32))


def test_huge_chain_weight_runs_strict_fp32():
    """An edge-MLP weight >= 2^15 cannot be split into unscaled fp16 pieces: ecnf_create makes the handle strict
    fp32 (instead of refusing it), the results are fp32-class, and asking for the split arithmetic is refused."""
    cfg, oc, p, x0, feat = _inputs("lj13", 6, stress=False)
    p = dict(p)
    w = p["EGNN_0/1/phi_x_torso/Dense_1/kernel"].copy()
    w[3, 5] = 40000.0
    p["EGNN_0/1/phi_x_torso/Dense_1/kernel"] = w
    h = EcnfHandle(cfg, p, 0)
    assert h.precision == "fp32" and h.chain_arithmetic() == "fp32_mfma"
    with pytest.raises(ValueError):
        h.set_precision("split_f16")
    t = np.linspace(0.1, 0.9, 6).astype(np.float32)
    v = h.vector_field(g(x0), g(t), g(feat, torch.int32)).cpu().numpy()
    ref64 = O.egnn_vector_field(p, oc, x0, t, feat, dtype=np.float64)
    ref32 = O.egnn_vector_field(p, oc, x0, t, feat, dtype=np.float32)
    _check("lj13 huge weight eval", v, ref64, ref32)
    # back to ordinary weights: the split arithmetic is available again
    h.update_params(O.init_params(oc, 0))
    h.set_precision("split_f16")
    assert h.chain_arithmetic() == "split_f16"
