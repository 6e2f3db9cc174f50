"""CPU tests of the oracle (the checker the GPU parity tests rely on), pinned by the known-answer tests the
reference's own test files imply:

  KAT-1  ecnf/cnf/core_test.py:11-44   linear field v = 3x with a N(0, 100^2 I) base: x1 = e^3 x0 and
                                      log q = log p0(x0) - 3 dim (exact trace); Hutchinson gives 3 |eps|^2.
  KAT-2  ecnf/nets/egnn_test.py:9-31 + ecnf/utils/test.py:60-76: rotation equivariance at atol = rtol = 1e-6.
plus properties implied by the architecture (translation quirk, permutation equivariance), finite-difference
checks of the forward-mode divergence, the closed-form base density, the Dopri5 order, the edge list, targets.
"""
import numpy as np
import pytest
from scipy.spatial.transform import Rotation

from oracle import ecnf_oracle as O


def _stressed(name, seed=0):
    oc = O.CONFIGS[name]
    return oc, O.stress_params(O.init_params(oc, seed), oc)


def _inputs(oc, B, seed=1):
    rng = np.random.default_rng(seed)
    z = rng.standard_normal((B, oc.n_nodes * oc.dim))
    x0 = O.base_sample(z, oc, np.float64)
    feat = rng.integers(0, oc.n_features, (B, oc.n_nodes))
    return z, x0, feat


# ---------------------------------------------------------------------------------------------- KAT-1
def _linear_field(x, t, div_mode, eps):
    v = 3.0 * x
    if div_mode == O.DIV_EXACT:
        div = np.full(x.shape[0], 3.0 * x.shape[1])
    elif div_mode == O.DIV_HUTCH:
        div = 3.0 * np.sum(eps * eps, axis=-1)
    else:
        div = np.zeros(x.shape[0])
    return v, div


def _normal_logp(x, scale=100.0):
    d = x.shape[-1]
    return -0.5 * np.sum((x / scale) ** 2, -1) - d * np.log(scale) - 0.5 * d * np.log(2 * np.pi)


@pytest.mark.parametrize("dt0,tol", [(0.05, 1e-6), (None, 1e-4)])
def test_kat1_linear_field(dt0, tol):
    dim, B = 3, 11
    oc = O.CNFConfig(n_nodes=1, dim=dim)
    x0 = np.random.default_rng(0).standard_normal((B, dim)) * 100.0
    feat = np.zeros((B, 1), np.int64)
    kw = dict(apply_fn=_linear_field, log_prob_base=_normal_logp, solver="dopri5", dt0=dt0, dtype=np.float64)
    x1, log_q, nfe = O.sample_and_log_prob(None, oc, x0, feat, approx=False, **kw)
    assert np.allclose(x1, np.exp(3.0) * x0, rtol=tol, atol=0)
    assert np.allclose(log_q, _normal_logp(x0) - 3.0 * dim, rtol=0, atol=tol * 10)
    if dt0 is not None:
        assert (nfe == 1 + 6 * 20).all()           # FSAL Dopri5, 20 steps of 0.05
    log_p, lp0, delta, _, x_back = O.get_log_prob(None, oc, x1, feat, approx=False, **kw)
    assert np.allclose(x_back, x0, rtol=tol)
    assert np.allclose(log_p, log_q, atol=tol * 10)
    assert np.allclose(delta, -3.0 * dim, atol=tol * 10)


def test_kat1_hutchinson_is_eps_dependent():
    dim, B = 3, 5
    oc = O.CNFConfig(n_nodes=1, dim=dim)
    rng = np.random.default_rng(2)
    x0 = rng.standard_normal((B, dim))
    eps = rng.standard_normal((B, dim))
    _, log_q, _ = O.sample_and_log_prob(None, oc, x0, np.zeros((B, 1)), eps=eps, approx=True, apply_fn=_linear_field,
                                        log_prob_base=_normal_logp, solver="dopri5", dt0=0.05, dtype=np.float64)
    assert np.allclose(log_q, _normal_logp(x0) - 3.0 * np.sum(eps ** 2, -1), atol=1e-6)


def test_dopri5_fifth_order():
    oc = O.CNFConfig(n_nodes=1, dim=2)
    x0 = np.array([[1.0, -2.0]])
    errs = []
    for dt in (0.02, 0.01):
        x1, _ = O.sample_cnf(None, oc, x0, np.zeros((1, 1)), solver="dopri5", dt0=dt, dtype=np.float64,
                             apply_fn=_linear_field)
        errs.append(np.abs(x1 - np.exp(3.0) * x0).max())
    assert 28 < errs[0] / errs[1] < 36       # 2^5 = 32


def test_euler_fixed_grid_nfe_and_first_order():
    oc = O.CNFConfig(n_nodes=1, dim=1)
    x1, nfe = O.sample_cnf(None, oc, np.ones((1, 1)), np.zeros((1, 1)), solver="euler", dt0=0.01,
                           dtype=np.float32, apply_fn=_linear_field)
    assert nfe[0] == 100                       # fp32 accumulated grid 0.99999934 is clipped to t1 (diffrax tol 1e-6)
    assert abs(x1[0, 0] - 1.03 ** 100) < 1e-3 * 1.03 ** 100


# ---------------------------------------------------------------------------------------------- KAT-2 & properties
@pytest.mark.parametrize("name", ["dw4", "lj13", "aldp"])
def test_kat2_rotation_equivariance(name):
    oc, p = _stressed(name)
    z, x0, feat = _inputs(oc, 3)
    t = np.array([0.1, 0.5, 0.9], np.float32)
    if oc.dim == 3:
        R = Rotation.random(random_state=3).as_matrix()
    else:
        a = 1.234
        R = np.array([[np.cos(a), -np.sin(a)], [np.sin(a), np.cos(a)]])
    rot = lambda y: (y.reshape(3, oc.n_nodes, oc.dim) @ R.T).reshape(3, -1)
    v = O.egnn_vector_field(p, oc, x0, t, feat)
    vr = O.egnn_vector_field(p, oc, rot(x0), t, feat)
    np.testing.assert_allclose(rot(v), vr, atol=1e-6, rtol=1e-6)


def test_translation_quirk():
    """v(x + s) = v(x) - s: the output subtracts the INPUT mean (egnn.py:186)."""
    oc, p = _stressed("lj13")
    z, x0, feat = _inputs(oc, 2)
    t = np.array([0.3, 0.6], np.float32)
    s = np.tile([0.5, -1.0, 2.0], oc.n_nodes)[None]
    np.testing.assert_allclose(O.egnn_vector_field(p, oc, x0 + s, t, feat) + s,
                               O.egnn_vector_field(p, oc, x0, t, feat), atol=1e-12)


def test_permutation_equivariance():
    oc, p = _stressed("lj13")            # one feature id: atoms are interchangeable
    z, x0, feat = _inputs(oc, 2)
    t = np.array([0.2, 0.7], np.float32)
    perm = np.random.default_rng(5).permutation(oc.n_nodes)
    P = lambda y: y.reshape(2, oc.n_nodes, 3)[:, perm].reshape(2, -1)
    np.testing.assert_allclose(P(O.egnn_vector_field(p, oc, x0, t, feat)),
                               O.egnn_vector_field(p, oc, P(x0), t, feat), atol=1e-12)


@pytest.mark.parametrize("name", ["dw4", "aldp"])
def test_divergence_matches_finite_differences(name):
    oc, p = _stressed(name)
    z, x0, feat = _inputs(oc, 2)
    t = np.array([0.25, 0.75], np.float32)
    _, div = O.divergence(p, oc, x0, t, feat)
    fd = np.zeros(2)
    e = 1e-6
    for k in range(x0.shape[1]):
        xp, xm = x0.copy(), x0.copy()
        xp[:, k] += e
        xm[:, k] -= e
        fd += (O.egnn_vector_field(p, oc, xp, t, feat)[:, k] - O.egnn_vector_field(p, oc, xm, t, feat)[:, k]) / (2 * e)
    np.testing.assert_allclose(div, fd, rtol=1e-6, atol=1e-6)
    u = np.random.default_rng(0).standard_normal(x0.shape)
    _, hut = O.divergence(p, oc, x0, t, feat, eps=u)
    _, ju = O.egnn_vector_field(p, oc, x0, t, feat, tangents=u[:, None])
    np.testing.assert_allclose(hut, np.sum(ju[:, 0] * u, -1), rtol=1e-12)


def test_fp32_restatement_tracks_fp64():
    oc, p = _stressed("lj13")
    z, x0, feat = _inputs(oc, 4)
    t = np.linspace(0, 1, 4).astype(np.float32)
    v64 = O.egnn_vector_field(p, oc, x0, t, feat, dtype=np.float64)
    v32 = O.egnn_vector_field(p, oc, x0.astype(np.float32), t, feat, dtype=np.float32)
    assert np.abs(v32 - v64).max() <= 2e-5 * max(1, np.abs(v64).max())


# ---------------------------------------------------------------------------------------------- pieces
def test_edge_list_receiver_major():
    s, r = O.fully_connected_edges(4)
    assert r.tolist() == [0, 0, 0, 1, 1, 1, 2, 2, 2, 3, 3, 3]
    assert s.tolist() == [1, 2, 3, 2, 3, 0, 3, 0, 1, 0, 1, 2]


def test_timestep_embedding():
    t = np.array([0.0, 0.3, 1.0], np.float32)
    emb = O.timestep_embedding(t, 8)
    k = np.arange(4)
    w = np.exp(-k * np.log(10000.0) / 3)
    ref = np.concatenate([np.sin(1000 * t[:, None] * w), np.cos(1000 * t[:, None] * w)], 1)
    np.testing.assert_allclose(emb, ref, atol=3e-4)       # fp32 arguments up to 1000 rad
    assert emb.dtype == np.float32 and emb.shape == (3, 8)


@pytest.mark.parametrize("name", ["dw4", "lj13", "aldp"])
def test_base_density_closed_form(name):
    oc = O.CONFIGS[name]
    z, x0, _ = _inputs(oc, 5)
    N, D, s = oc.n_nodes, oc.dim, oc.base_scale
    y = x0.reshape(5, N, D)
    ref = -0.5 * np.sum((y / s) ** 2, (1, 2)) - 0.5 * (N - 1) * D * np.log(2 * np.pi) - (N - 1) * D * np.log(s)
    np.testing.assert_allclose(O.base_log_prob(x0, oc), ref, rtol=1e-12)
    shifted = (y + np.array([1.0, 2.0, 3.0][:D])).reshape(5, -1)          # remove_mean: translation invariant
    np.testing.assert_allclose(O.base_log_prob(shifted, oc), ref, rtol=1e-10)
    assert np.abs(y.mean(axis=1)).max() < 1e-12                            # zero-CoM samples


def test_param_layout():
    oc = O.CONFIGS["lj13"]
    spec = O.param_spec(oc)
    assert spec[0][0] == "EGNN_0/0/Dense_0/bias" and spec[-1][0] == "Embed_0/embedding"
    assert [p for p, _ in spec] == sorted(p for p, _ in spec)     # flat keys here sort like the nested tree
    assert O.param_count(oc) == 510407
    p = O.init_params(oc, 0)
    np.testing.assert_array_equal(O.flatten_params(O.unflatten_params(O.flatten_params(p, oc), oc), oc),
                                  O.flatten_params(p, oc))


def test_targets_and_ess():
    x = np.array([[0.0, 0.0, 0.0], [1.0, 0.0, 0.0]])
    # one pair at r = 1: (1 - 2) per ordered pair, two ordered pairs, eps / (2 tau) = 1/2 -> -1; harmonic 0.5 * 0.5
    assert abs(O.lj_energy(x.reshape(1, -1), 2, 3)[0] - (-1.0 + 0.25)) < 1e-12
    d = np.array([[0.0, 0.0], [4.0, 0.0]])
    assert abs(O.dw_energy(d.reshape(1, -1), 2, 2)[0]) < 1e-12          # |r| = d0
    assert abs(O.forward_ess(np.zeros(10)) - 1.0) < 1e-12
    assert abs(O.reverse_ess(np.zeros(10)) - 1.0) < 1e-12
    lw = np.log(np.array([1.0, 0.0001, 0.0001, 0.0001]))
    assert O.reverse_ess(lw) < 0.3
