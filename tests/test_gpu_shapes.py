"""Networks of any mlp_units / hidden width on the compiled kernels (params.kernel_config + pad_params: zero-padded
units are exactly inert), against the oracle on the REFERENCE-shaped (unpadded) parameters:

  * the reference's own equivariance-test network (ecnf/nets/egnn_test.py:9-31: n_nodes 5, dim 3, n_blocks 2,
    mlp_units (16, 16), n_invariant_feat_hidden 32) through FlatEgnn (node features through the Embed, a T = 10
    sinusoidal time embedding in place of the test's ones(11) global vector, which FlatEgnn cannot take): KAT-2,
    assert_function_is_equivariant (ecnf/utils/test.py:60-76) on the HIP path at the reference's atol = rtol = 1e-6,
    plus parity of the field with the oracle
  * unequal widths mlp_units (48, 80) with n_invariant_feat_hidden 40 (kernel shape M = 128, H = 64): the field, its
    JVP, an Euler sample and the exact-trace log-density, fp32-class (tests/tolerance.py)
"""
import numpy as np
import pytest
import torch

from oracle import ecnf_oracle as O
from tolerance import fp32_class

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs a ROCm GPU", allow_module_level=True)

from ecnf_amd import cnf as C  # noqa: E402
from ecnf_amd.engine import SolveOptions  # noqa: E402


def _rotation(rng):
    """A random proper rotation (ecnf/utils/test.py:46-57 draws z ~ U(-1, 1) and two angles; any Haar-like draw)."""
    q, r = np.linalg.qr(rng.standard_normal((3, 3)))
    q = q * np.sign(np.diag(r))
    if np.linalg.det(q) < 0:
        q[:, 0] = -q[:, 0]
    return q


def _allclose(a, b, atol, rtol):
    """chex.assert_trees_all_close semantics: |a - b| <= atol + rtol |b|."""
    return bool(np.all(np.abs(a - b) <= atol + rtol * np.abs(b)))


@pytest.mark.parametrize("stress", [False, True])
def test_egnn_test_network_equivariance_kat2(stress):
    cnf = C.build_cnf(n_frames=5, dim=3, sigma_min=0.01, base_scale=1.0, n_blocks_egnn=2, mlp_units=(16, 16),
                      n_invariant_feat_hidden=32, time_embedding_dim=10, n_features=2, device=0)
    assert cnf.cfg.mlp_width == 64 and cnf.cfg.mlp_depth == 2 and cnf.cfg.hidden == 32
    oc = O.CNFConfig(n_nodes=5, dim=3, n_features=2, hidden=32, time_embedding_dim=10, mlp_units=(16, 16), n_blocks=2)
    p = O.init_params(oc, 0)
    if stress:
        p = O.stress_params(p, oc)
    assert {k: v.shape for k, v in p.items()} == {k: v.shape for k, v in cnf.init(0).items()}
    rng = np.random.default_rng(0)
    for trial in range(4):
        x = rng.standard_normal((1, 5, 3)).astype(np.float32)          # test.py:65: normal(key1, (n_nodes, dim))
        R = _rotation(rng).astype(np.float32)
        xg = (x[0] @ R.T)[None]
        feat = np.ones((1, 5), np.int32)
        t = np.array([0.3 + 0.2 * trial], np.float32)
        out = cnf.apply(p, x.reshape(1, -1), t, feat).cpu().numpy().reshape(5, 3)
        g_then_out = cnf.apply(p, xg.reshape(1, -1), t, feat).cpu().numpy().reshape(5, 3)
        out_then_g = out @ R.T
        assert _allclose(out_then_g, g_then_out, 1e-6, 1e-6), np.abs(out_then_g - g_then_out).max()
        ref = O.egnn_vector_field(p, oc, x.reshape(1, -1), t, feat, dtype=np.float64).reshape(5, 3)
        assert np.abs(out - ref).max() <= 2e-5 * max(1.0, np.abs(ref).max())


def test_unequal_widths_parity():
    units, H = (48, 80), 40
    cnf = C.build_cnf(n_frames=7, dim=3, sigma_min=0.01, base_scale=1.0, n_blocks_egnn=2, mlp_units=units,
                      n_invariant_feat_hidden=H, time_embedding_dim=8, n_features=3, device=0)
    assert cnf.cfg.mlp_width == 128 and cnf.cfg.hidden == 64
    oc = O.CNFConfig(n_nodes=7, dim=3, n_features=3, hidden=H, time_embedding_dim=8, mlp_units=units, n_blocks=2)
    p = O.stress_params(O.init_params(oc, 1), oc)
    rng = np.random.default_rng(3)
    B = 6
    x0 = O.base_sample(rng.standard_normal((B, 21)).astype(np.float32), oc)
    feat = rng.integers(0, 3, (B, 7)).astype(np.int32)
    t = np.linspace(0.0, 1.0, B).astype(np.float32)
    v = cnf.apply(p, x0, t, feat)
    fp32_class("unequal eval", v, O.egnn_vector_field(p, oc, x0, t, feat, dtype=np.float64),
               O.egnn_vector_field(p, oc, x0, t, feat, dtype=np.float32))
    h = cnf.to_device(p)
    u = rng.standard_normal((B, 2, 21)).astype(np.float32)
    _, ju = h.jvp(torch.from_numpy(x0).cuda(), torch.from_numpy(t).cuda(), torch.from_numpy(feat).cuda(),
                  torch.from_numpy(u).cuda())
    fp32_class("unequal jvp", ju, O.egnn_vector_field(p, oc, x0, t, feat, tangents=u, dtype=np.float64)[1],
               O.egnn_vector_field(p, oc, x0, t, feat, tangents=u, dtype=np.float32)[1])
    x1 = C.sample_cnf(cnf, p, None, features=feat, use_fixed_step_size=True, step_size=0.1, x0=x0, solver="euler")
    fp32_class("unequal euler-10", x1, O.sample_cnf(p, oc, x0, feat, solver="euler", dt0=0.1, dtype=np.float64)[0],
               O.sample_cnf(p, oc, x0, feat, solver="euler", dt0=0.1, dtype=np.float32)[0])
    lp, lp0, dl = C.get_log_prob(cnf, p, x0, None, features=feat, approx=False, use_fixed_step_size=True,
                                 step_size=0.25, solver="euler")
    r64 = O.get_log_prob(p, oc, x0, feat, approx=False, solver="euler", dt0=0.25, dtype=np.float64)
    r32 = O.get_log_prob(p, oc, x0, feat, approx=False, solver="euler", dt0=0.25, dtype=np.float32)
    fp32_class("unequal exact log_p", lp, r64[0], r32[0])
    fp32_class("unequal exact dl", dl, r64[2], r32[2])
