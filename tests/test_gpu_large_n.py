"""Molecules of 34 .. 64 atoms (receiver-tiled edges: Net::SR = 64 slots per receiver, every receiver's N - 1 edges on
two whole 32-edge tiles) against the oracle, which has no size limit (graph.py:6-14 for any N):

  * the field, an Euler sample and the Hutchinson and exact-trace log-densities, fp32-class (tests/tolerance.py),
    at N = 34 (33 edges per receiver: 32 + 1), 40 and 64 (63: 32 + 31) with the ALDP widths (mlp_units (64, 64),
    hidden 32) in 3D, and N = 48 in 2D
  * results bitwise independent of the batch position (each molecule owns its edge tiles)
  * the LJ-width network (mlp_units (128, 128, 128), hidden 64) at N = 40 and 64: its tangent kernels run in the wide
    form (Geo BN: per-edge phi_e.0, no per-node P rows, in-place phi_h over two 32-row tiles), at both precisions:
    JVP, Hutchinson and exact-trace log-densities fp32-class (round 5; before, ECNF_E_UNSUPPORTED past 33 atoms)
  * N = 65 is refused (ECNF_E_UNSUPPORTED)
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


def _setup(N, dim, seed=0, units=(64, 64), H=32, blocks=2):
    cnf = C.build_cnf(n_frames=N, dim=dim, sigma_min=0.01, base_scale=1.0, n_blocks_egnn=blocks, mlp_units=units,
                      n_invariant_feat_hidden=H, time_embedding_dim=8, n_features=3, device=0)
    oc = O.CNFConfig(n_nodes=N, dim=dim, n_features=3, hidden=H, time_embedding_dim=8, mlp_units=units,
                     n_blocks=blocks)
    p = O.stress_params(O.init_params(oc, seed), oc)
    return cnf, oc, p


@pytest.mark.parametrize("N,dim", [(34, 3), (40, 3), (64, 3), (48, 2)])
def test_large_n_field_sample_hutchinson(N, dim):
    cnf, oc, p = _setup(N, dim)
    rng = np.random.default_rng(N)
    B, ND = 3, N * dim
    x0 = O.base_sample(rng.standard_normal((B, ND)).astype(np.float32), oc)
    feat = rng.integers(0, 3, (B, N)).astype(np.int32)
    t = np.array([0.1, 0.5, 0.9], np.float32)
    v = cnf.apply(p, x0, t, feat)
    fp32_class(f"N={N} field", v, O.egnn_vector_field(p, oc, x0, t, feat, dtype=np.float64),
               O.egnn_vector_field(p, oc, x0, t, feat, dtype=np.float32))
    x1 = C.sample_cnf(cnf, p, None, features=feat, use_fixed_step_size=True, step_size=0.1, x0=x0, solver="euler")
    fp32_class(f"N={N} euler-10", x1, O.sample_cnf(p, oc, x0, feat, solver="euler", dt0=0.1, dtype=np.float64)[0],
               O.sample_cnf(p, oc, x0, feat, solver="euler", dt0=0.1, dtype=np.float32)[0])
    eps = rng.standard_normal((B, ND)).astype(np.float32)
    lp, lp0, dl = C.get_log_prob(cnf, p, x0, None, features=feat, approx=True, use_fixed_step_size=True,
                                 step_size=0.25, solver="euler", eps=eps)
    r64 = O.get_log_prob(p, oc, x0, feat, eps=eps, approx=True, solver="euler", dt0=0.25, dtype=np.float64)
    r32 = O.get_log_prob(p, oc, x0, feat, eps=eps, approx=True, solver="euler", dt0=0.25, dtype=np.float32)
    fp32_class(f"N={N} hutch log_p", lp, r64[0], r32[0])
    fp32_class(f"N={N} hutch dl", dl, r64[2], r32[2])
    # batch-position independence: molecule 1 alone, and at slot 0 of a reversed batch
    v1 = cnf.apply(p, x0[1:2], t[1:2], feat[1:2])
    vr = cnf.apply(p, x0[::-1].copy(), t[::-1].copy(), feat[::-1].copy())
    assert torch.equal(torch.as_tensor(v1)[0], torch.as_tensor(v)[1])
    assert torch.equal(torch.as_tensor(vr)[1], torch.as_tensor(v)[1])


@pytest.mark.parametrize("N", [40, 64])
def test_large_n_exact_trace(N):
    cnf, oc, p = _setup(N, 3, seed=1)
    rng = np.random.default_rng(7 + N)
    B = 2
    x0 = O.base_sample(rng.standard_normal((B, N * 3)).astype(np.float32), oc)
    feat = rng.integers(0, 3, (B, N)).astype(np.int32)
    lp, lp0, dl = C.get_log_prob(cnf, p, x0, None, features=feat, approx=False, use_fixed_step_size=True,
                                 step_size=0.5, solver="euler")
    r64 = O.get_log_prob(p, oc, x0, feat, approx=False, solver="euler", dt0=0.5, dtype=np.float64)
    r32 = O.get_log_prob(p, oc, x0, feat, approx=False, solver="euler", dt0=0.5, dtype=np.float32)
    fp32_class(f"N={N} exact log_p", lp, r64[0], r32[0])
    fp32_class(f"N={N} exact dl", dl, r64[2], r32[2])


@pytest.mark.parametrize("N", [40, 64])
def test_large_n_m128_divergence(N):
    units, H = (128, 128, 128), 64
    cnf, oc, p = _setup(N, 3, seed=2, units=units, H=H)
    assert cnf.cfg.mlp_width == 128
    rng = np.random.default_rng(11 + N)
    B, ND = 2, N * 3
    x0 = O.base_sample(rng.standard_normal((B, ND)).astype(np.float32), oc)
    feat = rng.integers(0, 3, (B, N)).astype(np.int32)
    t = np.array([0.3, 0.8], np.float32)
    h = cnf.to_device(p)
    assert h.molecules_per_workgroup(True) == 1
    u = rng.standard_normal((B, 2, ND)).astype(np.float32)
    _, ju = h.jvp(torch.from_numpy(x0).cuda(), torch.from_numpy(t).cuda(), torch.from_numpy(feat).cuda(),
                  torch.from_numpy(u).cuda())
    fp32_class(f"N={N} M=128 jvp", ju, O.egnn_vector_field(p, oc, x0, t, feat, tangents=u, dtype=np.float64)[1],
               O.egnn_vector_field(p, oc, x0, t, feat, tangents=u, dtype=np.float32)[1])
    eps = rng.standard_normal((B, ND)).astype(np.float32)
    r64 = O.get_log_prob(p, oc, x0, feat, eps=eps, approx=True, solver="euler", dt0=0.25, dtype=np.float64)
    r32 = O.get_log_prob(p, oc, x0, feat, eps=eps, approx=True, solver="euler", dt0=0.25, dtype=np.float32)
    for prec in ("split_f16", "fp32"):
        h.set_precision(prec)
        assert h.precision == prec
        lp, lp0, dl = C.get_log_prob(cnf, h, x0, None, features=feat, approx=True, use_fixed_step_size=True,
                                     step_size=0.25, solver="euler", eps=eps)   # the handle as is (its precision)
        fp32_class(f"N={N} M=128 hutch log_p ({prec})", lp, r64[0], r32[0])
        fp32_class(f"N={N} M=128 hutch dl ({prec})", dl, r64[2], r32[2])
    h.set_precision("split_f16")
    lp, lp0, dl = C.get_log_prob(cnf, h, x0[:1], None, features=feat[:1], approx=False, use_fixed_step_size=True,
                                 step_size=0.5, solver="euler")
    e64 = O.get_log_prob(p, oc, x0[:1], feat[:1], approx=False, solver="euler", dt0=0.5, dtype=np.float64)
    e32 = O.get_log_prob(p, oc, x0[:1], feat[:1], approx=False, solver="euler", dt0=0.5, dtype=np.float32)
    fp32_class(f"N={N} M=128 exact log_p", lp, e64[0], e32[0])
    fp32_class(f"N={N} M=128 exact dl", dl, e64[2], e32[2])


def test_n65_refused():
    cnf = C.build_cnf(n_frames=65, dim=3, sigma_min=0.01, base_scale=1.0, n_blocks_egnn=2, mlp_units=(64, 64),
                      n_invariant_feat_hidden=32, time_embedding_dim=8, n_features=3, device=0)
    with pytest.raises(Exception, match="n_nodes"):
        cnf.apply(cnf.init(0), np.zeros((1, 195), np.float32), np.zeros(1, np.float32), np.zeros((1, 65), np.int32))
