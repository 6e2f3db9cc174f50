"""Golden fixtures (tests/golden/golden_v1.npz, made by tests/golden/make_golden.py from the fp64 oracle).

CPU: the oracle still reproduces them (drift check) and the params generator is unchanged (checksum).
GPU: the HIP kernels reproduce them through the C-ABI, at the tolerances stated in test_gpu_parity.py.
"""
import os

import numpy as np
import pytest
import torch

from oracle import ecnf_oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
G = np.load(os.path.join(HERE, "golden", "golden_v1.npz"))
NAMES = ("dw4", "lj13", "aldp", "qm9")


def _params(name):
    oc = O.CONFIGS[name]
    return oc, O.stress_params(O.init_params(oc, 0), oc)


@pytest.mark.parametrize("name", NAMES)
def test_oracle_reproduces_golden(name):
    oc, p = _params(name)
    pre = name + "/"
    assert abs(float(O.flatten_params(p, oc).astype(np.float64).sum()) - float(G[pre + "param_checksum"])) < 1e-6
    v = O.egnn_vector_field(p, oc, G[pre + "x0"], G[pre + "t"], G[pre + "feat"], dtype=np.float64)
    np.testing.assert_allclose(v, G[pre + "v"], rtol=1e-9, atol=1e-12)
    if pre + "ju" in G:
        _, ju = O.egnn_vector_field(p, oc, G[pre + "x0"], G[pre + "t"], G[pre + "feat"], tangents=G[pre + "u"],
                                    dtype=np.float64)
        np.testing.assert_allclose(ju, G[pre + "ju"], rtol=1e-9, atol=1e-12)
    if name in ("dw4", "lj13"):
        x1, _ = O.sample_cnf(p, oc, G[pre + "x0"], G[pre + "feat"], solver="euler", dt0=0.1, dtype=np.float64)
        np.testing.assert_allclose(x1, G[pre + "euler10_x1"], rtol=1e-9, atol=1e-12)


# ------------------------------------------------------------------------------------------------ GPU
def _handle(name):
    from ecnf_amd import CONFIGS
    from ecnf_amd.engine import EcnfHandle
    oc, p = _params(name)
    return CONFIGS[name], EcnfHandle(CONFIGS[name], p, 0)


def _t(a, dtype=torch.float32):
    return torch.as_tensor(np.asarray(a), device="cuda", dtype=dtype)


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_hip_matches_golden(name):
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    from ecnf_amd import _lib
    from ecnf_amd.engine import SolveOptions
    cfg, h = _handle(name)
    pre = name + "/"
    x0, t, feat = _t(G[pre + "x0"]), _t(G[pre + "t"]), _t(G[pre + "feat"], torch.int32)
    scale = lambda ref: max(1.0, float(np.abs(ref).max()))
    v = h.vector_field(x0, t, feat).cpu().numpy()
    assert np.abs(v - G[pre + "v"]).max() <= 2e-5 * scale(G[pre + "v"])
    if pre + "ju" in G:
        _, ju = h.jvp(x0, t, feat, _t(G[pre + "u"]))
        assert np.abs(ju.cpu().numpy() - G[pre + "ju"]).max() <= 2e-5 * scale(G[pre + "ju"])
    y, _, nfe, _ = h.integrate(x0, feat, 0.0, 1.0, SolveOptions("euler", 0.1))
    assert np.abs(y.cpu().numpy() - G[pre + "euler10_x1"]).max() <= 1e-4 * scale(G[pre + "euler10_x1"])
    if pre + "dopri_x1" in G:
        y, _, nfe, _ = h.integrate(x0, feat, 0.0, 1.0, SolveOptions("dopri5", 0.1))
        assert np.abs(y.cpu().numpy() - G[pre + "dopri_x1"]).max() <= 1e-4
        assert (nfe.cpu().numpy() == 61).all()
        y, dl, _, _ = h.integrate(x0, feat, 0.0, 1.0, SolveOptions("dopri5", 0.1), divergence=_lib.DIV_HUTCHINSON,
                                  eps=_t(G[pre + "z"]))
        lq = (h.base_log_prob(x0) - dl).cpu().numpy()
        assert np.abs(y.cpu().numpy() - G[pre + "hutch_x1"]).max() <= 1e-4
        assert np.abs(lq - G[pre + "hutch_logq"]).max() <= 2e-3
    if pre + "logp_hutch" in G:
        xb, dl, _, _ = h.integrate(x0, feat, 1.0, 0.0, SolveOptions("dopri5", 0.1), divergence=_lib.DIV_HUTCHINSON,
                                   eps=_t(G[pre + "eps"]))
        lp = (h.base_log_prob(xb) + dl).cpu().numpy()
        assert np.abs(xb.cpu().numpy() - G[pre + "logp_hutch_x0"]).max() <= 1e-4
        assert np.abs(lp - G[pre + "logp_hutch"]).max() <= 2e-3
    if pre + "logp_exact" in G:
        xb, dl, _, _ = h.integrate(x0, feat, 1.0, 0.0, SolveOptions("dopri5", 0.1), divergence=_lib.DIV_EXACT)
        lp = (h.base_log_prob(xb) + dl).cpu().numpy()
        assert np.abs(lp - G[pre + "logp_exact"]).max() <= 2e-3
