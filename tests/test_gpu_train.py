"""GPU parity of the flow-matching training step (loss.py:10-32,
gradient_step.py:21-53) through the C-ABI.

Oracle: the fp64 torch restatement (oracle/torch_ref.py) with autograd, itself pinned to central finite
differences of the numpy fp64 oracle (tests/test_train_oracle.py).  Tolerances (fp32 GEMMs on the matrix cores vs
fp64): loss |err| <= 1e-5 relative; every parameter tensor's gradient |err| <= 1e-4 x max|grad of that tensor| +
1e-6 x max|grad| over all tensors.  Adam / EMA against a numpy restatement of optax.adam at 1e-6 relative.
"""
import numpy as np
import pytest
import torch

from oracle import ecnf_oracle as O
from oracle import torch_ref as R

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs a ROCm GPU", allow_module_level=True)

from ecnf_amd import CONFIGS, CNFConfig, param_spec, unflatten_params  # noqa: E402
from ecnf_amd import cnf as C  # noqa: E402
from ecnf_amd import train as TR  # noqa: E402
from ecnf_amd.engine import EcnfHandle  # noqa: E402

TINY = CNFConfig(n_nodes=5, dim=3, n_features=2, hidden=32, mlp_width=64, mlp_depth=2, n_blocks=2, base_scale=0.5)


def _ocfg(cfg):
    return O.CNFConfig(n_nodes=cfg.n_nodes, dim=cfg.dim, n_features=cfg.n_features, hidden=cfg.hidden,
                       time_embedding_dim=cfg.time_embedding_dim, mlp_width=cfg.mlp_width, mlp_depth=cfg.mlp_depth,
                       n_blocks=cfg.n_blocks, base_scale=cfg.base_scale, sigma_min=cfg.sigma_min)


def _case(cfg, B, seed=0):
    oc = _ocfg(cfg)
    p = O.stress_params(O.init_params(oc, seed), oc)
    rng = np.random.default_rng(seed + 5)
    x1 = O.base_sample(rng.standard_normal((B, cfg.event_dim)).astype(np.float32), oc) * np.float32(1.5)
    x0 = O.base_sample(rng.standard_normal((B, cfg.event_dim)).astype(np.float32), oc)
    t = rng.random(B).astype(np.float32)
    feat = rng.integers(0, cfg.n_features, (B, cfg.n_nodes)).astype(np.int32)
    return oc, p, x1, x0, t, feat


def _ref_grad(oc, p, x1, x0, t, feat):
    P = R.to_torch(p, torch.float64, requires_grad=True)
    loss = R.fm_loss(P, oc, torch.from_numpy(x1).double(), torch.from_numpy(x0).double(),
                     torch.from_numpy(t).double(), torch.from_numpy(feat))
    loss.backward()
    # parameters no output depends on (the last block's gate and phi_h) get zero gradients, as under jax.grad
    return float(loss.detach()), {k: (v.grad.numpy() if v.grad is not None else np.zeros(v.shape)) for k, v in P.items()}


@pytest.mark.parametrize("name,B", [("tiny", 6), ("dw4", 16), ("lj13", 8), ("aldp", 4), ("qm9", 2)])
def test_loss_and_grad_match_autograd(name, B):
    cfg = TINY if name == "tiny" else CONFIGS[name]
    oc, p, x1, x0, t, feat = _case(cfg, B)
    tr = TR.Trainer(cfg, max_batch=B + 3, device=0)
    loss, grad = tr.loss_and_grad(p, x1, x0, t, feat)
    loss_ref, g_ref = _ref_grad(oc, p, x1, x0, t, feat)
    assert abs(float(loss) - loss_ref) <= 1e-5 * abs(loss_ref), (float(loss), loss_ref)
    g = unflatten_params(grad.cpu().numpy(), cfg)
    gmax = max(float(np.abs(v).max()) for v in g_ref.values())
    worst = []
    for path, _ in param_spec(cfg):
        ref = g_ref[path].reshape(g[path].shape)
        err = float(np.abs(g[path] - ref).max())
        tol = 1e-4 * float(np.abs(ref).max()) + 1e-6 * gmax
        worst.append((err / max(tol, 1e-30), path, err, tol))
    worst.sort(reverse=True)
    print(name, "worst gradient tensors (err / tol):", [(round(w[0], 3), w[1]) for w in worst[:3]])
    assert worst[0][0] <= 1.0, worst[:3]


@pytest.mark.parametrize("name,B,floats", [("qm9", 2, 150_000), ("lj13", 8, 60_000), ("lj13", 8, 1)])
def test_small_reduction_arena(name, B, floats):
    """A split-reduction arena far below the default (ecnf_trainer_set_reduction_arena) makes the step flush its
    deferred reductions mid-way, between weight-gradient GEMMs and between a GEMM's weight and bias partials' users
    (P and Pb are one reservation, so a flush can never recycle P before it is reduced).  The gradient
    must agree with the default arena's to fp32 rounding (fewer K-splits, another summation order) and with autograd
    at test_loss_and_grad_match_autograd's tolerance."""
    cfg = CONFIGS[name]
    oc, p, x1, x0, t, feat = _case(cfg, B)
    tr = TR.Trainer(cfg, max_batch=B, device=0)
    l_def, g_def = tr.loss_and_grad(p, x1, x0, t, feat)
    used = tr.set_reduction_arena(floats)
    assert 0 < used < tr.set_reduction_arena(0)
    tr.set_reduction_arena(floats)
    l_small, g_small = tr.loss_and_grad(p, x1, x0, t, feat)
    tr.set_reduction_arena(0)
    assert torch.isfinite(g_small).all()
    assert abs(float(l_small) - float(l_def)) <= 1e-6 * abs(float(l_def))
    gd, gs = unflatten_params(g_def.cpu().numpy(), cfg), unflatten_params(g_small.cpu().numpy(), cfg)
    _, g_ref = _ref_grad(oc, p, x1, x0, t, feat)
    gmax = max(float(np.abs(v).max()) for v in g_ref.values())
    for path, _ in param_spec(cfg):
        scale = float(np.abs(gd[path]).max())
        assert float(np.abs(gs[path] - gd[path]).max()) <= 1e-5 * scale + 1e-7 * gmax, path
        ref = g_ref[path].reshape(gs[path].shape)
        assert float(np.abs(gs[path] - ref).max()) <= 1e-4 * float(np.abs(ref).max()) + 1e-6 * gmax, path


def test_step_is_deterministic_and_batch_bounds():
    cfg = CONFIGS["lj13"]
    oc, p, x1, x0, t, feat = _case(cfg, 8)
    tr = TR.Trainer(cfg, max_batch=8, device=0)
    l1, g1 = tr.loss_and_grad(p, x1, x0, t, feat)
    l2, g2 = tr.loss_and_grad(p, x1, x0, t, feat)
    assert torch.equal(l1, l2) and torch.equal(g1, g2)
    with pytest.raises(ValueError):
        tr.loss_and_grad(p, np.concatenate([x1, x1]), np.concatenate([x0, x0]), np.concatenate([t, t]),
                         np.concatenate([feat, feat]))


def test_device_feature_ids_out_of_range():
    """Device-resident features are not validated on the host (no sync): an out-of-range id must never index past the
    embedding table; its molecule makes the loss and the gradient NaN instead of reading other params."""
    cfg = CONFIGS["aldp"]
    oc, p, x1, x0, t, feat = _case(cfg, 4)
    tr = TR.Trainer(cfg, max_batch=4, device=0)
    l_ok, g_ok = tr.loss_and_grad(p, x1, x0, t, torch.from_numpy(feat).cuda())
    assert torch.isfinite(l_ok) and torch.isfinite(g_ok).all()
    for bad_id in (cfg.n_features, -1, 1 << 30):
        bad = torch.from_numpy(feat).cuda()
        bad[2, 5] = bad_id
        l_bad, g_bad = tr.loss_and_grad(p, x1, x0, t, bad)
        assert torch.isnan(l_bad), bad_id
        assert torch.isnan(g_bad).any(), bad_id
    with pytest.raises(ValueError):     # host features: checked before the upload
        f = feat.copy()
        f[0, 0] = cfg.n_features
        tr.loss_and_grad(p, x1, x0, t, f)


def _adam_ref(g, p, mu, nu, lr, count, b1=0.9, b2=0.999, eps=1e-8):
    """optax.scale_by_adam + scale(-lr) + apply_updates (bias corrections with the incremented count)."""
    g, p, mu, nu = (np.asarray(a, np.float64) for a in (g, p, mu, nu))
    mu = b1 * mu + (1 - b1) * g
    nu = b2 * nu + (1 - b2) * g * g
    mh, vh = mu / (1 - b1 ** count), nu / (1 - b2 ** count)
    u = -lr * mh / (np.sqrt(vh) + eps)
    return p + u, mu, nu, u


def test_adam_update_and_ema():
    cfg = TINY
    tr = TR.Trainer(cfg, max_batch=4, device=0)
    n = tr.n_params
    rng = np.random.default_rng(1)
    g = torch.tensor(rng.standard_normal(n).astype(np.float32), device="cuda")
    p0 = rng.standard_normal(n).astype(np.float32)
    p = torch.tensor(p0, device="cuda")
    mu = torch.zeros(n, device="cuda")
    nu = torch.zeros(n, device="cuda")
    ema = p.clone()
    pr, mr, nr = p0.astype(np.float64), np.zeros(n), np.zeros(n)
    er = p0.astype(np.float64)
    for count in (1, 2, 3):
        norms = tr.adam_update(g, p, mu, nu, ema, lr=1e-3 * count, count=count, ema_beta=0.9)
        pr, mr, nr, u = _adam_ref(g.cpu().numpy(), pr, mr, nr, 1e-3 * count, count)
        er = er * 0.9 + 0.1 * pr
        assert np.abs(p.cpu().numpy() - pr).max() <= 1e-6 * np.abs(pr).max()
        assert np.abs(ema.cpu().numpy() - er).max() <= 1e-6 * np.abs(er).max()
        nv = norms.cpu().numpy()
        assert abs(nv[0] - np.linalg.norm(g.cpu().numpy().astype(np.float64))) <= 1e-5 * nv[0]
        assert abs(nv[1] - np.linalg.norm(u)) <= 1e-5 * nv[1]


def test_update_fn_trains_and_refreshes_the_sampler():
    """gradient_step.flow_matching_update_fn on LJ13 (lj13.yaml: Adam, batch 64): 40 steps on a fixed synthetic
    data set lower the loss; the trained params re-packed into a sampling handle (ecnf_update_params) give the
    vector field of the oracle with those params."""
    cfg = CONFIGS["lj13"]
    cnf = C.build_cnf(n_frames=13, dim=3, sigma_min=cfg.sigma_min, base_scale=cfg.base_scale, n_blocks_egnn=3,
                      mlp_units=(128, 128, 128), n_invariant_feat_hidden=64, time_embedding_dim=8, n_features=1)
    oc = _ocfg(cfg)
    p0 = O.init_params(oc, 0)
    rng = np.random.default_rng(3)
    data = O.base_sample(rng.standard_normal((64, 39)).astype(np.float32), oc) * np.float32(0.6)   # zero CoM
    feat = np.zeros((64, 13), np.int32)
    opt = TR.adam(TR.warmup_cosine_decay_schedule(0.0, 3e-3, 5, 40, 0.0))
    state = TR.init_training_state(cnf, p0, opt, key=7, use_ema=True)
    losses = []
    for i in range(40):
        state, info = TR.flow_matching_update_fn(cnf, opt, state, data, feat, ema_beta=0.9)
        losses.append(float(info["loss"]))
        # the schedule starts at init_value 0: the first update is zero, as in optax
        assert np.isfinite(float(info["grad_norm"])) and (float(info["update_norm"]) > 0) == (i > 0)
    assert state.opt_state.count == 40
    assert np.mean(losses[-5:]) < 0.9 * np.mean(losses[:5]), losses
    h = EcnfHandle(cfg, p0, 0)
    h.update_params(state.params)
    trained = unflatten_params(state.params.cpu().numpy(), cfg)
    t = np.full(4, 0.3, np.float32)
    v = h.vector_field(torch.from_numpy(data[:4]).cuda(), torch.from_numpy(t).cuda(),
                       torch.from_numpy(feat[:4]).cuda()).cpu().numpy()
    ref = O.egnn_vector_field(trained, oc, data[:4], t, feat[:4], dtype=np.float64)
    assert np.abs(v - ref).max() <= 2e-5 * max(1.0, np.abs(ref).max())
