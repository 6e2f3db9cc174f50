"""Golden fixtures (tests/golden/golden_v1.npz, made by tests/golden/make_golden.py from the fp64 oracle).

CPU: the oracle still reproduces them (drift check) and the params generator is unchanged (checksum).
GPU: the HIP kernels reproduce them through the C-ABI, at the tolerances stated in test_gpu_parity.py; every
log-density is fp32-class (tests/tolerance.py) against the stored fp64 and fp32 oracle values.
"""
import os

import numpy as np
import pytest
import torch

from oracle import ecnf_oracle as O
from tolerance import fp32_class

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
        fp32_class(f"{name} hutch x1", y, G[pre + "hutch_x1"], G[pre + "hutch_x1_f32"])
        fp32_class(f"{name} hutch log_q", lq, G[pre + "hutch_logq"], G[pre + "hutch_logq_f32"])
    if pre + "logp_hutch" in G:
        xb, dl, _, _ = h.integrate(x0, feat, 1.0, 0.0, SolveOptions("dopri5", 0.1), divergence=_lib.DIV_HUTCHINSON,
                                   eps=_t(G[pre + "eps"]))
        lp = (h.base_log_prob(xb) + dl).cpu().numpy()
        assert np.abs(xb.cpu().numpy() - G[pre + "logp_hutch_x0"]).max() <= 1e-4
        fp32_class(f"{name} logp hutch dl", dl, G[pre + "logp_hutch_dl"], G[pre + "logp_hutch_dl_f32"])
        fp32_class(f"{name} logp hutch", lp, G[pre + "logp_hutch"], G[pre + "logp_hutch_f32"])
    if pre + "logp_exact" in G:
        xb, dl, _, _ = h.integrate(x0, feat, 1.0, 0.0, SolveOptions("dopri5", 0.1), divergence=_lib.DIV_EXACT)
        lp = (h.base_log_prob(xb) + dl).cpu().numpy()
        assert np.abs(xb.cpu().numpy() - G[pre + "logp_exact_x0"]).max() <= 1e-4
        fp32_class(f"{name} logp exact dl", dl, G[pre + "logp_exact_dl"], G[pre + "logp_exact_dl_f32"])
        fp32_class(f"{name} logp exact", lp, G[pre + "logp_exact"], G[pre + "logp_exact_f32"])


def test_eval_modes_fixture_inputs():
    """tests/golden/eval_modes_v1.npz (make_eval_modes.py; read by test_gpu_eval_modes.py): every case's inputs and
    params are what the GPU test regenerates (test_gpu_parity.setup's draws, oracle init + stress params), and the
    fp32 envelope is well formed (one solve of the input + perturbed copies, positive step counts)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_eval_modes", os.path.join(HERE, "golden", "make_eval_modes.py"))
    mk = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mk)
    E = np.load(os.path.join(HERE, "golden", "eval_modes_v1.npz"))
    for case, (name, B, mode, n_pert) in mk.CASES.items():
        pre = case + "/"
        oc, params, z, x0, feat = mk.setup(name, B)
        assert abs(float(O.flatten_params(params, oc).astype(np.float64).sum()) - float(E[pre + "param_checksum"])) < 1e-6
        assert np.array_equal(E[pre + "x"], x0) and np.array_equal(E[pre + "feat"], feat)
        if mode == "slp_hutch":
            assert np.array_equal(E[pre + "eps"], z)
        assert E[pre + "o32_x"].shape == (n_pert + 1, B, oc.n_nodes * oc.dim)
        assert E[pre + "o32_nfe"].shape == (n_pert + 1, B) and (E[pre + "o32_nfe"] > 7).all()
        assert np.isfinite(E[pre + "fine_lp"]).all() and E[pre + "fine_lp"].shape == (B,)
