"""Block-1 pair tiles (egnn_eval.hpp PairPlan13): a single-feature 13-atom molecule (LJ13) runs block 1's chains once
per unordered pair and adds each pair's message to both atoms and its shift with opposite signs.  The same network
declared with two node features (every atom given feature 0: the same arithmetic, but the receiver-segment path,
since the kernel cannot assume equal rows) must agree to fp32 rounding, and both with the fp64 oracle; the pair path
must be run-to-run deterministic and independent of the molecules per workgroup (bitwise), as the segment path is."""
import dataclasses

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

DEV = torch.device("cuda", 0)


def _ocfg(cfg):
    return O.CNFConfig(n_nodes=cfg.n_nodes, dim=cfg.dim, n_features=cfg.n_features, hidden=cfg.hidden,
                       time_embedding_dim=cfg.time_embedding_dim, mlp_width=cfg.mlp_width, mlp_depth=cfg.mlp_depth,
                       n_blocks=cfg.n_blocks, base_scale=cfg.base_scale, sigma_min=cfg.sigma_min)


@pytest.fixture(scope="module")
def handles():
    cfg1 = CONFIGS["lj13"]
    assert cfg1.n_features == 1 and cfg1.n_nodes == 13 and cfg1.mlp_width == 128
    cfg2 = dataclasses.replace(cfg1, n_features=2)
    oc1 = _ocfg(cfg1)
    p1 = O.stress_params(O.init_params(oc1, 3), oc1)
    p2 = dict(p1)
    emb = p1["Embed_0/embedding"]
    p2["Embed_0/embedding"] = np.concatenate([emb, emb[::-1] * 0.5 + 0.1], axis=0)   # the second row goes unused
    h1, h2 = EcnfHandle(cfg1, p1, 0), EcnfHandle(cfg2, p2, 0)
    yield cfg1, oc1, p1, h1, h2
    h1.close()
    h2.close()


def _inputs(cfg, B, seed):
    g = torch.Generator("cuda").manual_seed(seed)
    z = torch.randn((B, cfg.event_dim), device=DEV, generator=g)
    t = torch.rand(B, device=DEV, generator=g)
    feat = torch.zeros((B, cfg.n_nodes), device=DEV, dtype=torch.int32)
    return z, t, feat


@pytest.mark.timeout(120)
@pytest.mark.parametrize("B", [1, 5, 37, 1024])
def test_pair_tiles_match_segment_path_and_oracle(handles, B):
    cfg, oc, p, h1, h2 = handles
    z, t, feat = _inputs(cfg, B, 11)
    x = h1.base_sample(z)
    v1 = h1.vector_field(x, t, feat)
    v2 = h2.vector_field(x, t, feat)
    scale = max(1.0, float(v2.abs().max()))
    assert float((v1 - v2).abs().max()) <= 2e-6 * scale
    if B <= 37:
        ref = O.egnn_vector_field(p, oc, x.double().cpu().numpy(), t.cpu().numpy(),
                                  np.zeros((B, cfg.n_nodes), np.int64), dtype=np.float64)
        assert float(np.abs(v1.double().cpu().numpy() - ref).max()) <= 2e-5 * max(1.0, float(np.abs(ref).max()))
    # 20 Euler steps: the trajectories of the two paths stay within fp32 rounding of each other
    o = SolveOptions("euler", 0.05)
    y1 = h1.integrate(x, feat, 0.0, 1.0, o, _lib.DIV_NONE, None)[0]
    y2 = h2.integrate(x, feat, 0.0, 1.0, o, _lib.DIV_NONE, None)[0]
    assert float((y1 - y2).abs().max()) <= 2e-5 * max(1.0, float(y2.abs().max()))


@pytest.mark.timeout(120)
def test_pair_tiles_deterministic_and_batch_independent(handles):
    cfg, _, _, h1, _ = handles
    B = 300
    z, t, feat = _inputs(cfg, B, 12)
    x = h1.base_sample(z)
    o = SolveOptions("euler", 0.1)
    ya = h1.integrate(x, feat, 0.0, 1.0, o, _lib.DIV_NONE, None)[0]
    yb = h1.integrate(x, feat, 0.0, 1.0, o, _lib.DIV_NONE, None)[0]
    assert torch.equal(ya, yb)
    # every molecule's result is its own: the same molecules alone and at other batch positions
    for lo, hi in ((0, 1), (17, 20), (100, 137)):
        ys = h1.integrate(x[lo:hi].contiguous(), feat[lo:hi].contiguous(), 0.0, 1.0, o, _lib.DIV_NONE, None)[0]
        assert torch.equal(ys, ya[lo:hi])
    va = h1.vector_field(x, t, feat)
    vs = h1.vector_field(x[5:9].contiguous(), t[5:9].contiguous(), feat[5:9].contiguous())
    assert torch.equal(vs, va[5:9])


@pytest.mark.timeout(120)
def test_pair_tiles_tangents_match_segment_path(handles):
    """The divergence kernels' pair tiles (the tangent of a pair's message is symmetric too, its shift's tangent
    antisymmetric): JVPs and a Hutchinson log-density against the two-feature (segment-path) network."""
    cfg, _, _, h1, h2 = handles
    B = 64
    z, t, feat = _inputs(cfg, B, 13)
    x = h1.base_sample(z)
    u = torch.randn((B, 2, cfg.event_dim), device=DEV, generator=torch.Generator("cuda").manual_seed(14))
    v1, j1 = h1.jvp(x, t, feat, u)
    v2, j2 = h2.jvp(x, t, feat, u)
    assert float((v1 - v2).abs().max()) <= 2e-6 * max(1.0, float(v2.abs().max()))
    assert float((j1 - j2).abs().max()) <= 2e-6 * max(1.0, float(j2.abs().max()))
    o = SolveOptions("euler", 0.05)
    y1, d1 = h1.integrate(x, feat, 1.0, 0.0, o, _lib.DIV_HUTCHINSON, z)[:2]
    y2, d2 = h2.integrate(x, feat, 1.0, 0.0, o, _lib.DIV_HUTCHINSON, z)[:2]
    assert float((y1 - y2).abs().max()) <= 2e-5 * max(1.0, float(y2.abs().max()))
    assert float((d1 - d2).abs().max()) <= 2e-5 * max(1.0, float(d2.abs().max()))
