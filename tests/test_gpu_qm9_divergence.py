"""GPU parity of the M = 256 tangent kernels (QM9, Geo::kWideT: per-edge phi_e.0, sequential primal / tangent split
chains, in-place phi_h; Geo::kWideT32: the same structure in strict fp32) against the CPU oracle: the JVP, the
Hutchinson log-density of get_log_prob / sample_and_log_prob_cnf on the qm9.yaml network (N = 29), and the exact trace
on a small-N M = 256 network, at both GEMM precisions; a checkpoint with an edge weight >= 2^15 runs its divergence on
the strict-fp32 kernels.

Reference: setup_training.py:190-203 (get_log_prob on the test set for every config), sample_and_log_prob.py:41-149,
examples/config/qm9.yaml:5-13.  Tolerances as tests/test_gpu_parity.py: JVP max |err| <= 2e-5 * max(1, |ref|);
short fixed-step trajectories and log-densities fp32-class (tests/tolerance.py)."""
import numpy as np
import pytest
import torch

from oracle import ecnf_oracle as O
from tolerance import fp32_class

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # collected on CPU-only hosts, skipped there
    pytest.skip("needs a ROCm GPU", allow_module_level=True)

from ecnf_amd import CONFIGS, CNFConfig  # noqa: E402
from ecnf_amd import _lib  # noqa: E402
from ecnf_amd.engine import EcnfHandle, SolveOptions  # noqa: E402

from test_gpu_parity import g, rel_err, setup  # noqa: E402

# small-N network of the QM9 widths (M = 256, L = 4) for the exact trace (N * D = 15 tangents per evaluation)
WIDE_TINY = CNFConfig(n_nodes=5, dim=3, n_features=2, hidden=32, mlp_width=256, mlp_depth=4, n_blocks=2,
                      base_scale=1.0)


_FP32 = {}


def setup_prec(cfg, B, precision):
    """setup() of test_gpu_parity, with a strict-fp32 handle of the same weights for precision == "fp32"."""
    oc, params, h, z, x0, feat = setup(cfg, B)
    if precision == "fp32":
        if cfg not in _FP32:
            _FP32[cfg] = EcnfHandle(cfg, params, 0, precision="fp32")
        h = _FP32[cfg]
    return oc, params, h, z, x0, feat


@pytest.mark.parametrize("precision", ["split_f16", "fp32"])
def test_qm9_tangent_kernel_exists(precision):
    cfg = CONFIGS["qm9"]
    _, _, h, _, _, _ = setup_prec(cfg, 1, precision)
    assert h.molecules_per_workgroup(with_tangent=True) == 1
    assert h.chain_arithmetic(with_tangent=True) == ("split_f16" if precision == "split_f16" else "fp32_mfma")


@pytest.mark.parametrize("precision", ["split_f16", "fp32"])
def test_jvp_wide(precision):
    cfg = CONFIGS["qm9"]
    oc, params, h, z, x0, feat = setup_prec(cfg, 3, precision)
    t = np.array([0.1, 0.5, 0.9], np.float32)
    u = np.random.default_rng(3).standard_normal((3, 2, cfg.event_dim)).astype(np.float32)
    v, ju = h.jvp(g(x0), g(t), g(feat, torch.int32), g(u))
    vr, jr = O.egnn_vector_field(params, oc, x0, t, feat, tangents=u, dtype=np.float64)
    assert rel_err(v, vr) <= 2e-5, rel_err(v, vr)
    assert rel_err(ju, jr) <= 2e-5, rel_err(ju, jr)


@pytest.mark.parametrize("precision", ["split_f16", "fp32"])
def test_qm9_log_prob_hutchinson_fixed(precision):
    """get_log_prob(approx=True, fixed steps) on qm9.yaml: 1 -> 0, 8 Euler steps."""
    cfg = CONFIGS["qm9"]
    oc, params, h, z, x0, feat = setup_prec(cfg, 2, precision)
    eps = np.random.default_rng(77).standard_normal(x0.shape).astype(np.float32)
    x, dl, nfe, st = h.integrate(g(x0), g(feat, torch.int32), 1.0, 0.0, SolveOptions("euler", 0.125),
                                 divergence=_lib.DIV_HUTCHINSON, eps=g(eps))
    r64 = O.get_log_prob(params, oc, x0, feat, eps=eps, approx=True, solver="euler", dt0=0.125, dtype=np.float64)
    r32 = O.get_log_prob(params, oc, x0, feat, eps=eps, approx=True, solver="euler", dt0=0.125, dtype=np.float32)
    assert int(nfe.min()) == 8 and int(st.abs().sum()) == 0
    fp32_class("qm9 hutch x", x, r64[4], r32[4])
    fp32_class("qm9 hutch dl", dl, r64[2], r32[2])
    lp = (h.base_log_prob(x) + dl).cpu().numpy()
    fp32_class("qm9 hutch log_p", lp, r64[0], r32[0])


def test_qm9_sample_and_log_prob_hutchinson():
    """sample_and_log_prob_cnf(approx=True, fixed steps) on qm9.yaml: 0 -> 1, Dopri5 dt = 0.25, eps = z."""
    cfg = CONFIGS["qm9"]
    oc, params, h, z, x0, feat = setup(cfg, B=2)
    x1, dl, nfe, _ = h.integrate(g(x0), g(feat, torch.int32), 0.0, 1.0, SolveOptions("dopri5", 0.25),
                                 divergence=_lib.DIV_HUTCHINSON, eps=g(z))
    x1r, lq_ref, _ = O.sample_and_log_prob(params, oc, x0, feat, eps=z, approx=True, solver="dopri5", dt0=0.25,
                                           dtype=np.float64)
    x1r32, lq_32, _ = O.sample_and_log_prob(params, oc, x0, feat, eps=z, approx=True, solver="dopri5", dt0=0.25,
                                            dtype=np.float32)
    fp32_class("qm9 s+lp x1", x1, x1r, x1r32)
    lq = (h.base_log_prob(g(x0)) - dl).cpu().numpy()
    fp32_class("qm9 s+lp log_q", lq, lq_ref, lq_32)


@pytest.mark.parametrize("precision", ["split_f16", "fp32"])
def test_wide_log_prob_exact_fixed(precision):
    """get_log_prob(approx=False): the full N*D trace through the M = 256 tangent kernels (small N)."""
    cfg = WIDE_TINY
    oc, params, h, z, x0, feat = setup_prec(cfg, 3, precision)
    x, dl, nfe, _ = h.integrate(g(x0), g(feat, torch.int32), 1.0, 0.0, SolveOptions("euler", 0.125),
                                divergence=_lib.DIV_EXACT)
    r64 = O.get_log_prob(params, oc, x0, feat, approx=False, solver="euler", dt0=0.125, dtype=np.float64)
    r32 = O.get_log_prob(params, oc, x0, feat, approx=False, solver="euler", dt0=0.125, dtype=np.float32)
    fp32_class("wide exact x", x, r64[4], r32[4])
    fp32_class("wide exact dl", dl, r64[2], r32[2])
    lp = (h.base_log_prob(x) + dl).cpu().numpy()
    fp32_class("wide exact log_p", lp, r64[0], r32[0])


def test_wide_huge_weight_divergence_runs_strict_fp32():
    """An edge-MLP weight >= 2^15 on the M = 256 network: ecnf_create makes the handle strict fp32 and its divergence
    solves run on the fp32 M = 256 tangent kernels (round 2 refused them with ECNF_E_UNSUPPORTED)."""
    cfg = WIDE_TINY
    oc, _, _, z, x0, feat = setup(cfg, B=3)
    p = dict(O.init_params(oc, 0))
    w = p["EGNN_0/1/phi_x_torso/Dense_1/kernel"].copy()
    w[3, 5] = 40000.0
    p["EGNN_0/1/phi_x_torso/Dense_1/kernel"] = w
    h = EcnfHandle(cfg, p, 0)
    assert h.precision == "fp32" and h.chain_arithmetic(with_tangent=True) == "fp32_mfma"
    t = np.array([0.2, 0.5, 0.8], np.float32)
    u = np.random.default_rng(4).standard_normal((3, 2, cfg.event_dim)).astype(np.float32)
    v, ju = h.jvp(g(x0), g(t), g(feat, torch.int32), g(u))
    vr, jr = O.egnn_vector_field(p, oc, x0, t, feat, tangents=u, dtype=np.float64)
    vr32, jr32 = O.egnn_vector_field(p, oc, x0, t, feat, tangents=u, dtype=np.float32)
    fp32_class("wide huge-weight v", v, vr, vr32)
    fp32_class("wide huge-weight jvp", ju, jr, jr32)
    eps = np.random.default_rng(5).standard_normal(x0.shape).astype(np.float32)
    x, dl, nfe, st = h.integrate(g(x0), g(feat, torch.int32), 1.0, 0.0, SolveOptions("euler", 0.5),
                                 divergence=_lib.DIV_HUTCHINSON, eps=g(eps))
    r64 = O.get_log_prob(p, oc, x0, feat, eps=eps, approx=True, solver="euler", dt0=0.5, dtype=np.float64)
    r32 = O.get_log_prob(p, oc, x0, feat, eps=eps, approx=True, solver="euler", dt0=0.5, dtype=np.float32)
    assert int(st.abs().sum()) == 0
    fp32_class("wide huge-weight x", x, r64[4], r32[4])
    fp32_class("wide huge-weight dl", dl, r64[2], r32[2])


def test_wide_nonfinite_divergence_reruns_on_strict_fp32():
    """A molecule whose activations leave the fp16 range in the split M = 256 tangent kernels reports
    ECNF_E_NONFINITE; with the host fallback it is solved again on the strict-fp32 M = 256 tangent kernels (round 2
    had none: the molecule stayed flagged) and its log-density is fp32-class; the other molecules are unchanged."""
    cfg = WIDE_TINY
    oc, _, _, z, x0, feat = setup(cfg, B=3)
    p = O.init_params(oc, 0)
    h = EcnfHandle(cfg, p, 0)
    x0 = x0.copy()
    x0[1] *= 1000.0            # |r|^2 ~ 1e6 into phi_e.0: pre-activations beyond fp16
    eps = np.random.default_rng(6).standard_normal(x0.shape).astype(np.float32)
    opts = SolveOptions("euler", 0.5)
    _, dl_raw, _, st = h.integrate(g(x0), g(feat, torch.int32), 0.0, 1.0, opts, divergence=_lib.DIV_HUTCHINSON,
                                   eps=g(eps), check_status=False)
    st = st.cpu().numpy()
    assert st[0] == 0 and st[2] == 0 and st[1] == _lib.ECNF_E_NONFINITE, st
    x1, dl, _, st2 = h.integrate(g(x0), g(feat, torch.int32), 0.0, 1.0, opts, divergence=_lib.DIV_HUTCHINSON,
                                 eps=g(eps))
    assert (st2.cpu().numpy() == 0).all() and torch.isfinite(dl).all()
    assert torch.equal(dl[[0, 2]], dl_raw[[0, 2]])
    _, lq64, _ = O.sample_and_log_prob(p, oc, x0, feat, eps=eps, approx=True, solver="euler", dt0=0.5,
                                       dtype=np.float64)
    _, lq32, _ = O.sample_and_log_prob(p, oc, x0, feat, eps=eps, approx=True, solver="euler", dt0=0.5,
                                       dtype=np.float32)
    lq = (h.base_log_prob(g(x0)) - dl).cpu().numpy()
    C = 4.0
    assert np.abs(lq - lq64).max() <= C * np.abs(lq32 - lq64).max() + 1e-5 * max(1.0, np.abs(lq64).max())


def test_wide_fp32_adaptive_sample_and_log_prob():
    """sample_and_log_prob_cnf with the reference's default adaptive solve (Dopri5 + PID, rtol = atol = 1e-5) through
    the strict-fp32 M = 256 tangent kernels, held to the envelope of test_gpu_eval_modes.py: the fp32 oracle's adaptive
    solves of x0 and of 5 copies perturbed by 1e-7 relative against an fp64 truth (Dopri5, fixed dt = 0.005).

    Round 3 compared the kernel's NFE (63 / 159) with the fp64 ADAPTIVE oracle's (57 / 111) and widened the bound to
    50 %.  The fp32 oracle's own NFE for these molecules is 57 ... 69 and 117 ... 267 over x0 and the perturbed copies
    (x0 alone: 63 / 267): the second molecule's step sequence is chaotic in fp32, the controller is not different.  So
    the bound is the 30 % one against that fp32 envelope: each molecule's NFE within [0.7 min, 1.3 max]."""
    from test_gpu_eval_modes import envelope, nfe_envelope
    from test_gpu_parity import _perturbed
    cfg = WIDE_TINY
    oc, params, h, z, x0, feat = setup_prec(cfg, 2, "fp32")
    xd = h.base_sample(g(z))
    x1, dl, nfe, st = h.integrate(xd, g(feat, torch.int32), 0.0, 1.0, SolveOptions("dopri5", None),
                                  divergence=_lib.DIV_HUTCHINSON, eps=g(z))
    assert int(st.abs().sum()) == 0
    xf, lqf, _ = O.sample_and_log_prob(params, oc, x0, feat, eps=z, approx=True, solver="dopri5", dt0=0.005,
                                       dtype=np.float64)
    xs, lqs, nfes = [], [], []
    for k in range(6):
        x32, lq32, n32 = O.sample_and_log_prob(params, oc, _perturbed(x0, k), feat, eps=z, approx=True,
                                               solver="dopri5", dt0=None, dtype=np.float32)
        xs.append(x32), lqs.append(lq32), nfes.append(n32)
    nfe_envelope("wide fp32 adaptive", nfe, np.stack(nfes))
    envelope("wide fp32 adaptive x1", x1, xf, np.stack(xs), 2e-4)
    lq = h.base_log_prob(xd) - dl
    envelope("wide fp32 adaptive log_q", lq, lqf, np.stack(lqs), 1e-4 * max(1.0, float(np.abs(lqf).max())))
