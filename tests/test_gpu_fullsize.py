"""Parity at the BASELINE.json batch sizes (configs[1..3]): the full batch runs in one launch, and strided molecules
of it are checked against the fp64 oracle and bitwise against a small-batch run of the same molecules.

  * LJ13, B = 1024, Euler NFE = 100 (the headline workload): 6 strided molecules vs the fp64 oracle, |err| <= 1e-4
  * ALDP, B = 512 real frames of the reference's aldp_500K_train_mini.h5 (zero-CoM centred, setup_training.py:91-94),
    get_log_prob with PIDController(rtol = atol = 1e-5) and Hutchinson: 4 strided molecules held to the adaptive
    envelope of test_gpu_parity.py (within 2x (+2e-4 / +2e-3) the largest distance of the fp32 oracle's own solves
    of x and 3 perturbed copies to an accurate fp64 fixed-step solution)
  * LJ13, B = 1024, get_log_prob(approx=False) with Euler NFE = 100: the shipped exact trace (sparse blocks 1 and K,
    primal aggregates cached in a caller workspace of 1024 + MPW slots) for the whole batch in one launch; 3 strided
    molecules fp32-class (tests/tolerance.py) in x and the log-density against the fp64 / fp32 oracle's full N*D trace,
    and bitwise against a small-batch run of the same molecules (other workgroup sizes, other cache slots)
  * ALDP, B = 512 real frames, get_log_prob(approx=False) with Euler NFE = 20: the same checks on 2 strided molecules
    (ALDP: 15 primal + 2 dual tiles per molecule in the sparse blocks)
  * QM9 shape (N = 29, M = 256, L = 4, K = 5), B = 2048, Euler NFE = 10 (the full NFE-100 batch is timed by
    tools/bench_paths.py; 10 steps bound the oracle's CPU time): 2 strided molecules vs fp64, |err| <= 1e-4
"""
import os

import numpy as np
import pytest
import torch

from oracle import ecnf_oracle as O
from tolerance import fp32_class

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs a ROCm GPU", allow_module_level=True)

from ecnf_amd import CONFIGS  # noqa: E402
from ecnf_amd import _lib  # noqa: E402
from ecnf_amd.engine import EcnfHandle, SolveOptions  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
DEV = torch.device("cuda", 0)


def g(a, dtype=torch.float32):
    return torch.as_tensor(np.asarray(a), device=DEV, dtype=dtype)


def _setup(name, B, stress=True):
    cfg, oc = CONFIGS[name], O.CONFIGS[name]
    p = O.init_params(oc, 0)
    if stress:
        p = O.stress_params(p, oc)
    rng = np.random.default_rng(2024)
    z = rng.standard_normal((B, cfg.event_dim)).astype(np.float32)
    return cfg, oc, p, z, EcnfHandle(cfg, p, 0)


def test_lj13_b1024_euler100():
    cfg, oc, p, z, h = _setup("lj13", 1024)
    x0 = O.base_sample(z, oc)
    feat = np.zeros((1024, cfg.n_nodes), np.int32)
    y, _, nfe, st = h.integrate(g(x0), g(feat, torch.int32), 0.0, 1.0, SolveOptions("euler", 0.01))
    assert (st.cpu().numpy() == 0).all() and (nfe.cpu().numpy() == 100).all()
    idx = np.array([0, 205, 411, 617, 822, 1023])
    ref, _ = O.sample_cnf(p, oc, x0[idx], feat[idx], solver="euler", dt0=0.01, dtype=np.float64)
    assert np.abs(y.cpu().numpy()[idx] - ref).max() <= 1e-4
    y_small, _, _, _ = h.integrate(g(x0[idx]), g(feat[idx], torch.int32), 0.0, 1.0, SolveOptions("euler", 0.01))
    assert torch.equal(y[idx], y_small)


def _aldp_frames(B):
    frames = np.load(os.path.join(HERE, "golden", "aldp_frames.npy")).astype(np.float32)
    assert frames.shape[0] >= B and frames.shape[1:] == (22, 3)
    frames = frames[:B]
    return (frames - frames.mean(axis=1, keepdims=True)).reshape(B, -1)   # setup_training.py:91-94


def _exact_fullsize(name, x, feat, p, oc, h, dt, idx):
    xb, dl, nfe, st = h.integrate(g(x), g(feat, torch.int32), 1.0, 0.0, SolveOptions("euler", dt),
                                  divergence=_lib.DIV_EXACT)
    assert (st.cpu().numpy() == 0).all() and torch.isfinite(dl).all()
    assert (nfe.cpu().numpy() == round(1 / dt)).all()
    lp = h.base_log_prob(xb) + dl
    r64 = O.get_log_prob(p, oc, x[idx], feat[idx], approx=False, solver="euler", dt0=dt, dtype=np.float64)
    r32 = O.get_log_prob(p, oc, x[idx], feat[idx], approx=False, solver="euler", dt0=dt, dtype=np.float32)
    fp32_class(f"{name} exact x", xb[idx], r64[4], r32[4])
    fp32_class(f"{name} exact dl", dl[idx], r64[2], r32[2])
    fp32_class(f"{name} exact log_p", lp[idx], r64[0], r32[0])
    xs, dls, _, _ = h.integrate(g(x[idx]), g(feat[idx], torch.int32), 1.0, 0.0, SolveOptions("euler", dt),
                                divergence=_lib.DIV_EXACT)
    assert torch.equal(xb[idx], xs) and torch.equal(dl[idx], dls)


@pytest.mark.timeout(400)
def test_lj13_b1024_exact_log_prob_euler100():
    """get_log_prob(approx=False) (sample_and_log_prob.py:57-67) at the headline batch and NFE."""
    cfg, oc, p, z, h = _setup("lj13", 1024)
    x = O.base_sample(z, oc)
    feat = np.zeros((1024, cfg.n_nodes), np.int32)
    _exact_fullsize("lj13 B=1024", x, feat, p, oc, h, 0.01, np.array([0, 511, 1023]))


@pytest.mark.timeout(300)
def test_aldp_b512_exact_log_prob_real_frames():
    cfg, oc, p, _, h = _setup("aldp", 512)
    x = _aldp_frames(512)
    feat = np.tile(np.arange(22, dtype=np.int32), (512, 1))          # data.py:146
    _exact_fullsize("aldp B=512", x, feat, p, oc, h, 0.05, np.array([0, 511]))


@pytest.mark.timeout(400)
def test_aldp_b512_adaptive_hutchinson_log_prob():
    cfg, oc, p, _, h = _setup("aldp", 512)
    x = _aldp_frames(512)
    feat = np.tile(np.arange(22, dtype=np.int32), (512, 1))          # data.py:146
    eps = np.random.default_rng(4321).standard_normal(x.shape).astype(np.float32)
    xb, dl, nfe, st = h.integrate(g(x), g(feat, torch.int32), 1.0, 0.0, SolveOptions("dopri5", None),
                                  divergence=_lib.DIV_HUTCHINSON, eps=g(eps))
    assert (st.cpu().numpy() == 0).all() and torch.isfinite(dl).all()
    lp = (h.base_log_prob(xb) + dl).cpu().numpy()
    idx = np.array([0, 170, 341, 511])
    lp_f, _, dl_f, _, x_f = O.get_log_prob(p, oc, x[idx], feat[idx], eps=eps[idx], approx=True, solver="dopri5",
                                           dt0=0.005, dtype=np.float64)
    # the envelope: the oracle's own fp32 adaptive solves of x and of 3 copies perturbed by 1e-7 (relative) -- these
    # ~900-step solves fork: the perturbations alone move one molecule's log-prob by 0.05 .. 0.34
    eo_x = eo_lp = 0.0
    for k in range(4):
        xk = x[idx] if k == 0 else \
            (x[idx] * (1 + 1e-7 * np.random.default_rng(100 + k).standard_normal(x[idx].shape))).astype(np.float32)
        lp_32, _, _, nfe_k, x_32 = O.get_log_prob(p, oc, xk, feat[idx], eps=eps[idx], approx=True, solver="dopri5",
                                                  dt0=None, dtype=np.float32)
        eo_x = max(eo_x, float(np.abs(x_32 - x_f).max()))
        eo_lp = max(eo_lp, float(np.abs(lp_32 - lp_f).max()))
        if k == 0:
            nfe_32 = nfe_k
    ek = np.abs(xb.cpu().numpy()[idx] - x_f).max()
    print(f"aldp adaptive x: kernel {ek:.3e}, oracle envelope {eo_x:.3e}")
    assert ek <= 2 * eo_x + 2e-4, (ek, eo_x)
    ek = np.abs(lp[idx] - lp_f).max()
    print(f"aldp adaptive log_p: kernel {ek:.3e}, oracle envelope {eo_lp:.3e}")
    assert ek <= 2 * eo_lp + 2e-3, (ek, eo_lp)
    nfe = nfe.cpu().numpy()
    assert abs(nfe[idx].mean() - nfe_32.mean()) <= 0.3 * nfe_32.mean(), (nfe[idx], nfe_32)
    xb_s, dl_s, _, _ = h.integrate(g(x[idx]), g(feat[idx], torch.int32), 1.0, 0.0, SolveOptions("dopri5", None),
                                   divergence=_lib.DIV_HUTCHINSON, eps=g(eps[idx]))
    assert torch.equal(xb[idx], xb_s) and torch.equal(dl[idx], dl_s)


def test_qm9_b2048_euler():
    cfg, oc, p, z, h = _setup("qm9", 2048)
    x0 = O.base_sample(z, oc)
    feat = np.zeros((2048, cfg.n_nodes), np.int32)
    y, _, nfe, st = h.integrate(g(x0), g(feat, torch.int32), 0.0, 1.0, SolveOptions("euler", 0.1))
    assert (st.cpu().numpy() == 0).all() and (nfe.cpu().numpy() == 10).all()
    idx = np.array([0, 2047])
    ref, _ = O.sample_cnf(p, oc, x0[idx], feat[idx], solver="euler", dt0=0.1, dtype=np.float64)
    assert np.abs(y.cpu().numpy()[idx] - ref).max() <= 1e-4
    y_small, _, _, _ = h.integrate(g(x0[idx]), g(feat[idx], torch.int32), 0.0, 1.0, SolveOptions("euler", 0.1))
    assert torch.equal(y[idx], y_small)
