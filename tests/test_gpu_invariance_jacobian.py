"""GPU checks that complement tests/test_gpu_parity.py:

* bitwise batch-position invariance of every kernel family (split primal M = 64 / 128 / 256, split tangent M = 64 /
  128, the M = 256 tangent kernels): a molecule's output must not depend on its batch slot, on the batch size or on
  the molecules per workgroup the launch picks for that batch size (net_for_batch), so that shards concatenate
  bit-identically across ranks;
* the full Jacobian through ecnf_vf_jvp with N*D unit tangents against the oracle (the exact-trace building block of
  get_log_prob(approx=False), sample_and_log_prob.py:57-66), its trace, and the translation-identity form of the
  trace the exact-divergence solver evaluates from N*D - D columns.

Tolerances: bitwise for invariance; 2e-5 * max(1, |ref|) for the Jacobian (as the JVP parity test)."""
import numpy as np
import pytest
import torch

from oracle import ecnf_oracle as O

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # collected on CPU-only hosts, skipped there
    pytest.skip("needs a ROCm GPU", allow_module_level=True)

from ecnf_amd import CONFIGS  # noqa: E402
from ecnf_amd import _lib  # noqa: E402
from ecnf_amd.engine import SolveOptions  # noqa: E402

from test_gpu_parity import TINY, g, rel_err, setup  # noqa: E402


@pytest.mark.parametrize("name,B", [("lj13", 37), ("aldp", 11), ("qm9", 5), ("dw4", 70)])
def test_batch_position_invariance_all_kernels(name, B):
    cfg = CONFIGS[name]
    oc, params, h, z, x0, feat = setup(cfg, B=B, seed=3)
    eps = np.random.default_rng(9).standard_normal(x0.shape).astype(np.float32)
    X, F, E = g(x0), g(feat, torch.int32), g(eps)
    o = SolveOptions("euler", 0.25)
    y_all, _, _, _ = h.integrate(X, F, 0.0, 1.0, o)
    yh_all, dl_all, _, _ = h.integrate(X, F, 0.0, 1.0, o, _lib.DIV_HUTCHINSON, E)
    for lo, hi in [(0, 1), (B // 2, B // 2 + 3), (1, B)]:
        y, _, _, _ = h.integrate(X[lo:hi], F[lo:hi], 0.0, 1.0, o)
        assert torch.equal(y, y_all[lo:hi]), (name, lo, hi)
        yh, dl, _, _ = h.integrate(X[lo:hi], F[lo:hi], 0.0, 1.0, o, _lib.DIV_HUTCHINSON, E[lo:hi])
        assert torch.equal(yh, yh_all[lo:hi]) and torch.equal(dl, dl_all[lo:hi]), (name, lo, hi)


@pytest.mark.parametrize("name", ["dw4", "tiny"])
def test_full_jacobian_and_trace(name):
    cfg = TINY if name == "tiny" else CONFIGS[name]
    oc, params, h, z, x0, feat = setup(cfg, B=3, seed=5)
    ND = cfg.event_dim
    t = np.array([0.2, 0.5, 0.8], np.float32)
    u = np.broadcast_to(np.eye(ND, dtype=np.float32), (3, ND, ND)).copy()   # tangent k = e_k
    v, J = h.jvp(g(x0), g(t), g(feat, torch.int32), g(u))
    vr, Jr = O.egnn_vector_field(params, oc, x0, t, feat, tangents=u, dtype=np.float64)
    assert rel_err(v, vr) <= 2e-5
    assert rel_err(J, Jr) <= 2e-5, rel_err(J, Jr)
    # row k of the JVP batch is J e_k: its trace is the divergence the exact-trace solver accumulates
    tr = np.trace(J.cpu().numpy(), axis1=1, axis2=2)
    tr_ref = np.trace(Jr, axis1=1, axis2=2)
    assert np.abs(tr - tr_ref).max() <= 2e-5 * max(1.0, np.abs(tr_ref).max())
    # the exact-trace solver's form (ecnf_kernels.hpp joint_field): v(x + s 1) = v(x) - s gives
    # tr J = sum_{k >= D} (J_kk - J_(k mod D),k) - D from the ND - D columns k >= D; it holds to rounding on the
    # device and to fp64 rounding in the oracle
    D = cfg.dim
    def tr_translation(Jm):
        k = np.arange(D, ND)
        return (Jm[:, k, k] - Jm[:, k, k % D]).sum(axis=1) - D   # row k of the JVP batch is J e_k
    assert np.abs(tr_translation(Jr) - tr_ref).max() <= 1e-9 * max(1.0, np.abs(tr_ref).max())
    assert np.abs(tr_translation(J.cpu().numpy().astype(np.float64)) - tr_ref).max() <= 2e-5 * max(1.0, np.abs(tr_ref).max())
