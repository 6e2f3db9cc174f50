"""Parity at the BASELINE.json batch sizes (configs[1..3]): the full batch runs in one launch, and strided molecules
of it are checked against the fp64 oracle and bitwise against a small-batch run of the same molecules.

  * LJ13, B = 1024, Euler NFE = 100 (the headline workload): 6 strided molecules vs the fp64 oracle, |err| <= 1e-4
  * ALDP, B = 512 real frames of the reference's aldp_500K_train_mini.h5 (zero-CoM centred, setup_training.py:91-94),
    get_log_prob with PIDController(rtol = atol = 1e-5) and Hutchinson: 4 strided molecules held to the adaptive
    envelope of test_gpu_parity.py (within 2x (+2e-4 / +2e-3) the largest distance of the fp32 oracle's own solves
    of x and 3 perturbed copies to an accurate fp64 fixed-step solution)
  * QM9 shape (N = 29, M = 256, L = 4, K = 5), B = 2048, Euler NFE = 10 (the full NFE-100 batch is timed by
    tools/bench_paths.py; 10 steps bound the oracle's CPU time): 2 strided molecules vs fp64, |err| <= 1e-4
"""
import os

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


@pytest.mark.timeout(400)
def test_aldp_b512_adaptive_hutchinson_log_prob():
    cfg, oc, p, _, h = _setup("aldp", 512)
    frames = np.load(os.path.join(HERE, "golden", "aldp_frames.npy")).astype(np.float32)
    assert frames.shape == (512, 22, 3)
    x = (frames - frames.mean(axis=1, keepdims=True)).reshape(512, -1)
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
    assert ek <= 2 * eo_x + 2e-4, (ek, eo_x)
    ek = np.abs(lp[idx] - lp_f).max()
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
