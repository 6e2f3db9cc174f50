"""The reference's CONFIGURED eval modes on the HIP path, through the reference-named surface (ecnf_amd.cnf).

Every example yaml sets `use_fixed_step_size: false`, so the reference's evaluation runs Dopri5 + PIDController
(rtol = atol = 1e-5, dtmin = 1e-5, Hairer's initial step):

  * LJ13 / DW4 test-set log-likelihood: get_log_prob(approx=False), exact N*D trace, 1 -> 0 (lj13.yaml:33-34,
    dw4.yaml:32-33, setup_training.py:196-200);
  * LJ13 reverse ESS: sample_and_log_prob_cnf(approx=True), Hutchinson with eps = the base draw, 0 -> 1, ONE molecule
    per call (setup_training.py:166-182) -- here at B = 1 and at B = 4;
  * QM9 test-set log-likelihood: get_log_prob(approx=True), Hutchinson, 1 -> 0 (qm9.yaml:32-33,
    setup_training.py:202-203);
  * sample_and_log_prob_cnf(approx=False): the reference CNF test's own call (ecnf/cnf/core_test.py:42) with the
    default adaptive solve (DW4 network), and with fixed steps (sample_and_log_prob.py:111-121), fp32-class.

Adaptive tolerances (the envelope of test_gpu_parity.py's adaptive cases, against committed fixtures
tests/golden/eval_modes_v1.npz made by tests/golden/make_eval_modes.py): the fixture holds an fp64 truth (Dopri5,
fixed dt = 0.005) and the fp32 oracle's adaptive solves of the input and of 1e-7-perturbed copies.  A PID solve forks
in fp32, so the kernel's distance to the truth may be at most 2x the largest distance among those fp32 solves plus
a floor (2e-4 for positions; 1e-4 x max(1, |truth|) for log-densities), and every molecule's NFE must lie within
30 % of the range the fp32 solves span ([0.7 min, 1.3 max]).  Fixed-step cases are fp32-class (tests/tolerance.py).
"""
import os

import numpy as np
import pytest
import torch

from oracle import ecnf_oracle as O
from tolerance import fp32_class

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # collected on CPU-only hosts, skipped there
    pytest.skip("needs a ROCm GPU", allow_module_level=True)

from ecnf_amd import CONFIGS  # noqa: E402
from ecnf_amd import _lib  # noqa: E402
from ecnf_amd import cnf as C  # noqa: E402
from ecnf_amd.engine import SolveOptions  # noqa: E402

from test_gpu_parity import g, setup  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
E = np.load(os.path.join(HERE, "golden", "eval_modes_v1.npz"))
PID = SolveOptions("dopri5", None)          # PIDController(rtol = atol = 1e-5, dtmin = 1e-5), dt0 = None


def _fixture(case):
    pre = case + "/"
    return {k[len(pre):]: E[k] for k in E.files if k.startswith(pre)}


def _build(name):
    c = CONFIGS[name]
    return C.build_cnf(n_frames=c.n_nodes, dim=c.dim, sigma_min=c.sigma_min, base_scale=c.base_scale,
                       n_blocks_egnn=c.n_blocks, mlp_units=(c.mlp_width,) * c.mlp_depth,
                       n_invariant_feat_hidden=c.hidden, time_embedding_dim=c.time_embedding_dim,
                       n_features=c.n_features, device=0)


def _np(a):
    return a.detach().cpu().numpy() if torch.is_tensor(a) else np.asarray(a)


def envelope(name, got, fine, o32, floor):
    """max |got - fine| <= 2 max_k |o32[k] - fine| + floor (o32: [n_solves, ...])."""
    got, fine = _np(got).astype(np.float64), np.asarray(fine, np.float64)
    spread = float(np.abs(np.asarray(o32, np.float64) - fine[None]).max())
    err = float(np.abs(got - fine).max())
    print(f"{name}: |hip - truth| {err:.3e}, fp32-oracle spread {spread:.3e}, bound {2 * spread + floor:.3e}")
    assert err <= 2 * spread + floor, (name, err, spread)


def nfe_envelope(name, nfe, o32_nfe):
    """Each molecule's NFE within [0.7 min, 1.3 max] of the fp32 oracle's solves of it (o32_nfe: [n_solves, B])."""
    nfe = _np(nfe).astype(np.int64)
    lo, hi = 0.7 * o32_nfe.min(axis=0), 1.3 * o32_nfe.max(axis=0)
    print(f"{name}: NFE {nfe.tolist()}, fp32 oracle {o32_nfe.T.tolist()}")
    assert np.all((nfe >= lo) & (nfe <= hi)), (name, nfe, o32_nfe)


def _check_case(case, name, B):
    """Setup of the fixture case (the inputs are test_gpu_parity.setup()'s: checked against the fixture)."""
    oc, params, h, z, x0, feat = setup(CONFIGS[name], B=B)
    F = _fixture(case)
    assert abs(float(O.flatten_params(params, oc).astype(np.float64).sum()) - float(F["param_checksum"])) < 1e-6
    assert np.array_equal(F["x"], x0) and np.array_equal(F["feat"], feat)
    return oc, params, h, z, x0, feat, F


# ------------------------------------------------------------------------------------------------------------------
@pytest.mark.timeout(300)
@pytest.mark.parametrize("name,B", [("lj13", 2), ("dw4", 3)])
def test_get_log_prob_exact_pid(name, B):
    """get_log_prob(approx=False, use_fixed_step_size=False): the LJ13 / DW4 test-set log-likelihood as the example
    configs run it (exact trace, PID)."""
    oc, params, h, z, x0, feat, F = _check_case(f"{name}_logp_exact_pid", name, B)
    x, dl, nfe, st = h.integrate(g(x0), g(feat, torch.int32), 1.0, 0.0, PID, divergence=_lib.DIV_EXACT)
    assert int(st.abs().sum()) == 0
    nfe_envelope(f"{name} exact pid", nfe, F["o32_nfe"])
    envelope(f"{name} exact pid x(0)", x, F["fine_x"], F["o32_x"], 2e-4)
    envelope(f"{name} exact pid delta", dl, F["fine_dl"], F["o32_dl"], 1e-4 * max(1.0, np.abs(F["fine_dl"]).max()))
    # the reference-named call (defaults: approx=False, use_fixed_step_size=False) is the same launch
    cnf = _build(name)
    log_p, lpb, dl2 = C.get_log_prob(cnf, h, g(x0), None, features=feat)
    assert torch.equal(dl2, dl)
    assert torch.equal(lpb, h.base_log_prob(x))
    envelope(f"{name} exact pid log_p", log_p, F["fine_lp"], F["o32_lp"], 1e-4 * max(1.0, np.abs(F["fine_lp"]).max()))


@pytest.mark.timeout(300)
def test_sample_and_log_prob_hutchinson_pid_one_molecule_per_call():
    """LJ13 reverse-ESS sampling: sample_and_log_prob_cnf(approx=True) with PID (eps = the raw draw z behind x0),
    at B = 4 in one launch and at B = 1 per call as setup_training.py:166-182 scans it: every single-molecule call
    is bitwise its row of the batch (no cross-molecule coupling under per-molecule adaptive steps)."""
    oc, params, h, z, x0, feat, F = _check_case("lj13_slp_hutch_pid", "lj13", 4)
    xd = h.base_sample(g(z))       # x0 as sample_and_log_prob_cnf draws it (the device base sample of z)
    x1, dl, nfe, st = h.integrate(xd, g(feat, torch.int32), 0.0, 1.0, PID, divergence=_lib.DIV_HUTCHINSON, eps=g(z))
    assert int(st.abs().sum()) == 0
    nfe_envelope("lj13 hutch pid", nfe, F["o32_nfe"])
    envelope("lj13 hutch pid x1", x1, F["fine_x"], F["o32_x"], 2e-4)
    lq = h.base_log_prob(xd) - dl
    envelope("lj13 hutch pid log_q", lq, F["fine_lp"], F["o32_lp"], 1e-4 * max(1.0, np.abs(F["fine_lp"]).max()))
    cnf = _build("lj13")
    xs, lqs = C.sample_and_log_prob_cnf(cnf, h, None, features=feat, approx=True, z=z)
    assert torch.equal(xs, x1) and torch.equal(lqs, lq)
    for i in (0, 2):
        x1i, lqi = C.sample_and_log_prob_cnf(cnf, h, None, features=feat[i], approx=True, z=z[i])
        assert x1i.shape == (cnf.cfg.event_dim,) and lqi.shape == ()
        assert torch.equal(x1i, x1[i]) and torch.equal(lqi, lq[i]), i


@pytest.mark.timeout(300)
def test_qm9_get_log_prob_hutchinson_pid():
    """QM9 test-set log-likelihood: get_log_prob(approx=True) with PID on the qm9.yaml network (N = 29, M = 256 split
    tangent kernels)."""
    oc, params, h, z, x0, feat, F = _check_case("qm9_logp_hutch_pid", "qm9", 2)
    eps = F["eps"]
    x, dl, nfe, st = h.integrate(g(x0), g(feat, torch.int32), 1.0, 0.0, PID, divergence=_lib.DIV_HUTCHINSON,
                                 eps=g(eps))
    assert int(st.abs().sum()) == 0
    nfe_envelope("qm9 hutch pid", nfe, F["o32_nfe"])
    envelope("qm9 hutch pid x(0)", x, F["fine_x"], F["o32_x"], 2e-4)
    envelope("qm9 hutch pid delta", dl, F["fine_dl"], F["o32_dl"], 1e-4 * max(1.0, np.abs(F["fine_dl"]).max()))
    cnf = _build("qm9")
    log_p, _, dl2 = C.get_log_prob(cnf, h, g(x0), None, features=feat, approx=True, eps=g(eps))
    assert torch.equal(dl2, dl)
    envelope("qm9 hutch pid log_p", log_p, F["fine_lp"], F["o32_lp"], 1e-4 * max(1.0, np.abs(F["fine_lp"]).max()))


@pytest.mark.timeout(300)
def test_sample_and_log_prob_exact_pid_core_test_call():
    """sample_and_log_prob_cnf(cnf, params, key, features, approx=False) with its defaults (adaptive PID): the call of
    ecnf/cnf/core_test.py:42, on the DW4 network (exact trace, 0 -> 1)."""
    oc, params, h, z, x0, feat, F = _check_case("dw4_slp_exact_pid", "dw4", 3)
    x1, dl, nfe, st = h.integrate(h.base_sample(g(z)), g(feat, torch.int32), 0.0, 1.0, PID, divergence=_lib.DIV_EXACT)
    assert int(st.abs().sum()) == 0
    nfe_envelope("dw4 exact pid sample", nfe, F["o32_nfe"])
    envelope("dw4 exact pid x1", x1, F["fine_x"], F["o32_x"], 2e-4)
    cnf = _build("dw4")
    xs, lq = C.sample_and_log_prob_cnf(cnf, h, None, features=feat, approx=False, z=z)
    assert torch.equal(xs, x1)
    envelope("dw4 exact pid log_q", lq, F["fine_lp"], F["o32_lp"], 1e-4 * max(1.0, np.abs(F["fine_lp"]).max()))


@pytest.mark.timeout(300)
@pytest.mark.parametrize("name,B,dt", [("lj13", 2, 0.25), ("dw4", 3, 0.1)])
def test_sample_and_log_prob_exact_fixed(name, B, dt):
    """sample_and_log_prob_cnf(approx=False, use_fixed_step_size=True) (sample_and_log_prob.py:111-121; the fixed-step
    branch repaired to y0 = (x0, 0)): exact trace 0 -> 1, fp32-class against the oracle."""
    oc, params, h, z, x0, feat = setup(CONFIGS[name], B=B)
    cnf = _build(name)
    x1, lq = C.sample_and_log_prob_cnf(cnf, h, None, features=feat, approx=False, use_fixed_step_size=True,
                                       step_size=dt, z=z)
    x64, lq64, nfe64 = O.sample_and_log_prob(params, oc, x0, feat, approx=False, solver="dopri5", dt0=dt,
                                             dtype=np.float64)
    x32, lq32, _ = O.sample_and_log_prob(params, oc, x0, feat, approx=False, solver="dopri5", dt0=dt,
                                         dtype=np.float32)
    assert int(nfe64.min()) == 6 * round(1 / dt) + 1
    fp32_class(f"{name} exact fixed x1", x1, x64, x32)
    fp32_class(f"{name} exact fixed log_q", lq, lq64, lq32)
