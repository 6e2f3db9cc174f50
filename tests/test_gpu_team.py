"""Team (latency) mode of the primal solves (egnn_eval.hpp team_exchange, include/ecnf.h ecnf_set_team): G workgroups
integrate one molecule together, its edge tiles dealt round-robin over them and the edge aggregates exchanged through
global memory after every block's edge phase.  The use case is the reference's own sampling timer, ONE QM9 molecule
per sample_cnf call (examples/load_checkpoint_measure_sampling_time.py:101-119), which the batch path runs on one CU.

The rebuilt aggregates are those a single workgroup holds (a receiver's segment touches at most two tiles; a missing
part is an exact zero), so a team solve must be BITWISE equal to the batch path's solve of the same molecules, for
every G, solver and batch; the batch path itself is pinned to the oracle by test_gpu_parity / test_golden.  One case
checks the team path against the oracle directly (QM9 at B = 1, Euler, 1e-4 as test_euler_sample_short)."""
import numpy as np
import pytest
import torch

from oracle import ecnf_oracle as O

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # collected on CPU-only hosts, skipped there
    pytest.skip("needs a ROCm GPU", allow_module_level=True)

from ecnf_amd import CONFIGS  # noqa: E402
from ecnf_amd import _lib  # noqa: E402
from ecnf_amd import cnf as C  # noqa: E402
from ecnf_amd.engine import SolveOptions  # noqa: E402

from test_gpu_parity import g, setup  # noqa: E402


def _solve(h, x0, feat, opts, mode):
    h.set_team(mode)
    try:
        y, _, nfe, st = h.integrate(g(x0), g(feat, torch.int32), 0.0, 1.0, opts)
    finally:
        h.set_team(0)
    return y, nfe, st


def test_team_sizes():
    """Auto mode: QM9 (M = 256, 26 edge tiles per molecule on 4-wave workgroups) takes G = 7 (one tile round per block)
    for batches up to 32 (B G <= CUs); the M <= 128 shapes keep the batch path unless forced; divergence solves and
    shapes without a team kernel always run the batch path."""
    _, _, hq, _, _, _ = setup(CONFIGS["qm9"], B=1)
    # column-split mode (edge_tile_cols: one tile per member, G = 26 tiles) while B x 26 fits the CUs, then the
    # tile-dealt mode (G = 7)
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    bc = ncu // 26
    assert hq.team_workgroups(1) == 26 and hq.team_workgroups(bc) == 26
    assert hq.team_workgroups(bc + 1) == 7 and hq.team_workgroups(32) == 7
    assert hq.team_workgroups(33) == 1 and hq.team_workgroups(1, with_tangent=True) == 1
    hq.set_team(7)   # forced: the tile-dealt mode
    try:
        assert hq.team_workgroups(1) == 7
    finally:
        hq.set_team(0)
    _, _, hl, _, _, _ = setup(CONFIGS["lj13"], B=1)
    assert hl.team_workgroups(1) == 1
    hl.set_team(3)
    try:
        assert hl.team_workgroups(4) == 3 and hl.team_workgroups(4, with_tangent=True) == 1
    finally:
        hl.set_team(0)
    _, _, hd, _, _, _ = setup(CONFIGS["dw4"], B=1)   # (128, 3, 2): no team kernel
    hd.set_team(2)
    try:
        assert hd.team_workgroups(1) == 1
    finally:
        hd.set_team(0)
    with pytest.raises(ValueError):
        hl.set_team(-1)


@pytest.mark.parametrize("name,B,mode,opts", [
    ("qm9", 1, 0, SolveOptions("euler", 0.1)),      # column-split mode (G = 26)
    ("qm9", 3, 0, SolveOptions("euler", 0.2)),
    ("qm9", 9, 0, SolveOptions("dopri5", 0.25)),
    ("qm9", 1, 7, SolveOptions("euler", 0.1)),      # tile-dealt mode (forced G = 7)
    ("qm9", 12, 0, SolveOptions("euler", 0.25)),    # auto, past the column-split mode's CU budget: G = 7
    ("qm9", 2, 4, SolveOptions("dopri5", 0.25)),
    ("qm9", 1, 0, SolveOptions("dopri5", None)),
    ("lj13", 3, 2, SolveOptions("euler", 0.05)),
    ("lj13", 2, 5, SolveOptions("dopri5", None)),
    ("aldp", 2, 2, SolveOptions("euler", 0.1)),
    ("aldp", 1, 3, SolveOptions("dopri5", None)),
])
def test_team_bitwise_equals_batch_path(name, B, mode, opts):
    cfg = CONFIGS[name]
    oc, params, h, z, x0, feat = setup(cfg, B=B)
    h.set_team(mode)
    G = h.team_workgroups(B)
    h.set_team(0)
    assert G >= 2, (name, B, mode, G)
    y_t, nfe_t, st_t = _solve(h, x0, feat, opts, mode)
    y_b, nfe_b, st_b = _solve(h, x0, feat, opts, 1)
    assert (st_t.cpu().numpy() == 0).all() and (st_b.cpu().numpy() == 0).all()
    assert torch.equal(nfe_t, nfe_b), (nfe_t, nfe_b)
    assert torch.equal(y_t, y_b), float((y_t - y_b).abs().max())


def test_team_qm9_one_molecule_vs_oracle_and_surface():
    """QM9 at B = 1 through the reference-named sample_cnf (the timer's call) runs the team path and matches the oracle
    (Euler, 10 steps, 1e-4 as test_euler_sample_short); the default adaptive call reports a plausible NFE."""
    cfg = CONFIGS["qm9"]
    oc, params, h, z, x0, feat = setup(cfg, B=1)
    assert h.team_workgroups(1) == 26
    cnf = C.build_cnf(n_frames=cfg.n_nodes, dim=cfg.dim, sigma_min=cfg.sigma_min, base_scale=cfg.base_scale,
                      n_blocks_egnn=cfg.n_blocks, mlp_units=(cfg.mlp_width,) * cfg.mlp_depth,
                      n_invariant_feat_hidden=cfg.hidden, time_embedding_dim=cfg.time_embedding_dim,
                      n_features=cfg.n_features, device=0)
    x1 = C.sample_cnf(cnf, h, None, features=feat[0], use_fixed_step_size=True, step_size=0.1, x0=x0[0],
                      solver="euler")
    ref, _ = O.sample_cnf(params, oc, x0, feat, solver="euler", dt0=0.1, dtype=np.float64)
    assert x1.shape == (cfg.event_dim,)
    assert float(np.abs(x1.cpu().numpy() - ref[0]).max()) <= 1e-4
    y, _, nfe, st = h.integrate(g(x0), g(feat, torch.int32), 0.0, 1.0, SolveOptions("dopri5", None))
    assert int(st[0]) == _lib.ECNF_OK and int(nfe[0]) > 7


@pytest.mark.parametrize("B,mode,opts", [
    (1, 2, SolveOptions("euler", 0.1)),
    (5, 4, SolveOptions("euler", 0.1)),
    (3, 3, SolveOptions("dopri5", None)),
    (13, 4, SolveOptions("dopri5", None)),   # two groups of XCD-placed teams (8 + 5)
])
def test_tangent_team_bitwise_equals_batch_path(B, mode, opts):
    """Team mode of the Hutchinson tangent kernels (ALDP's M = 64 shape, forced G; team_exchange also rebuilds the
    tangent message and shift rows): get_log_prob (t = 1 -> 0) is bitwise the batch path's -- y(0), the divergence
    integral, NFE and status.  The exact trace never runs in team mode (its sparse blocks are not exchanged): with a
    forced G it takes the batch path, bitwise too."""
    cfg = CONFIGS["aldp"]
    oc, params, h, z, x0, feat = setup(cfg, B=B)
    eps = g(np.asarray(z, np.float32))

    def run(m, div):
        h.set_team(m)
        try:
            return h.integrate(g(x0), g(feat, torch.int32), 1.0, 0.0, opts, div, eps if div == _lib.DIV_HUTCHINSON
                               else None)
        finally:
            h.set_team(0)

    h.set_team(mode)
    assert h.team_workgroups(B, with_tangent=True) == mode
    h.set_team(0)
    assert h.team_workgroups(B, with_tangent=True) == 1   # tangent teams only when forced (or as re-deal tails)
    for div in (_lib.DIV_HUTCHINSON,) + ((_lib.DIV_EXACT,) if opts.step_size else ()):
        t, b = run(mode, div), run(1, div)
        for p, q in zip(t, b):
            assert torch.equal(p, q), (div, float((p.float() - q.float()).abs().max()))
        assert int(t[3].abs().sum()) == 0
