"""CPU oracle: a numpy restatement of the reference's equivariant-CNF sample / log_prob path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this module, and only as the checker (or as the timed CPU
baseline).  The product path (``ecnf_amd``) never imports it and fails loudly when the HIP
library is missing.

What it restates (all paths relative to the reference snapshot, Kalyan0821/ecnf-baseline-neurips-2023):

* ``ecnf/cnf/build_cnf.py:18-32``        get_timestep_embedding           -> :func:`timestep_embedding`
* ``ecnf/cnf/build_cnf.py:46-61``        scaled zero-CoM base (distrax)   -> :func:`base_sample`, :func:`base_log_prob`
* ``ecnf/cnf/build_cnf.py:65-93``        FlatEgnn.__call__                -> :func:`egnn_vector_field`
* ``ecnf/nets/egnn.py:49-114``           EGCL.__call__                    -> :func:`_egcl`
* ``ecnf/nets/egnn.py:144-190``          EGNN.call_single                 -> :func:`egnn_vector_field`
* ``ecnf/nets/mlp.py:7-19``              MLP                              -> :func:`_mlp`
* ``ecnf/utils/graph.py:6-14``           fully connected edge list        -> :func:`fully_connected_edges`
* ``ecnf/utils/numerical.py:7-10``       safe_norm                        -> inside :func:`_egcl`
* ``ecnf/cnf/zero_com_base.py:10-93``    zero-CoM Gaussian                -> :func:`base_sample`, :func:`base_log_prob`
* ``ecnf/cnf/sample_and_log_prob.py:11-149``  sample_cnf / get_log_prob / sample_and_log_prob_cnf
                                          -> :func:`sample_cnf`, :func:`get_log_prob`, :func:`sample_and_log_prob`
* ``ecnf/cnf/core.py:35-39``             optimal_transport_conditional_vf -> :func:`ot_conditional_vf`
* ``ecnf/targets/target_energy/leonard_jones.py:10-35`` / ``double_well.py:9-28`` -> :func:`lj_energy`, :func:`dw_energy`
* ``ecnf/utils/evaluation.py:10-22``, ``ecnf/setup_training.py:182``  -> :func:`forward_ess`, :func:`reverse_ess`
* ``ecnf/utils/evaluation.py:25-115``, ``ecnf/setup_training.py:190-215``, ``ecnf/utils/numerical.py:43-52``
                                          -> :func:`setup_padded_reshaped_data`, :func:`eval_test_set`,
                                             :func:`maybe_masked_mean`

Third-party arithmetic restated from its published algorithm (none of these packages is importable
here and ``requirements.txt:1-16`` pins no versions):

* diffrax (2023 API): ``Dopri5`` tableau with the Shampine embedded pair (b_error ends in -1/60), FSAL,
  ``ConstantStepSize`` (t_{n+1} = t_n + dt accumulated in fp32, clipped to t1 within 1e-6),
  ``PIDController`` defaults (I-controller, safety 0.9, factormin 0.2, factormax 10, error order 5,
  rms norm over every leaf of the state — (x, logp) for the joint solves, x alone for sample_cnf —
  ``force_dtmin``) and Hairer's initial step
  selection; reversed time (t0 > t1) by reparametrisation tau = -t.
* flax ``Dense``/``Embed`` (x @ kernel + bias, kernel [in, out]); e3nn-jax ``scatter_sum`` (segment sum);
  distrax ``ScalarAffine``/``Lambda``/``Transformed`` log-det conventions.

PARITY STATUS.  The reference cannot run here (``import jax`` fails) and its own tests
assert no numeric values, so this oracle is pinned by the known-answer tests the reference's tests imply:
KAT-1 (``ecnf/cnf/core_test.py:11-44``: linear field v = 3x, analytic e^3 flow and log-det -3*dim),
KAT-2 (``ecnf/nets/egnn_test.py:9-31`` + ``ecnf/utils/test.py:60-76``: rotation equivariance at 1e-6),
the closed-form base log-density, translation/permutation properties and finite-difference checks of the
forward-mode divergence.  diffrax-internal numerics (tableau variant, controller details) are
"parity unpinned" beyond those KATs.

Divergences are computed in FORWARD mode (J e_k, eps^T J eps) where the reference uses ``jax.vjp``
(``sample_and_log_prob.py:64-66,75-77``): the same quantity, different rounding.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import numpy as np

Params = Dict[str, np.ndarray]


# ----------------------------------------------------------------------------------------------
# configuration (examples/config/*.yaml `flow:` keys)
# ----------------------------------------------------------------------------------------------
@dataclass(frozen=True)
class CNFConfig:
    n_nodes: int                 # n_frames (N)
    dim: int                     # D
    n_features: int = 1          # Embed vocabulary size
    hidden: int = 64             # n_invariant_feat_hidden (H)
    time_embedding_dim: int = 8  # T
    mlp_width: int = 128         # every entry of mlp_units (M)
    mlp_depth: int = 3           # len(mlp_units) (L)
    n_blocks: int = 3            # n_blocks_egnn (K)
    base_scale: float = 1.0
    sigma_min: float = 0.01
    normalization_constant: float = 1.0   # egnn.py:127
    variance_scaling_init: float = 0.001  # egnn.py:128
    mlp_units: Optional[Tuple[int, ...]] = None   # unequal widths (egnn.py:43-47); None: (mlp_width,) * mlp_depth

    @property
    def n_edges(self) -> int:
        return self.n_nodes * (self.n_nodes - 1)

    @property
    def units(self) -> Tuple[int, ...]:
        return tuple(self.mlp_units) if self.mlp_units else (self.mlp_width,) * self.mlp_depth


# the configs of BASELINE.json, with shapes from examples/config/{dw4,lj13,aldp,qm9}.yaml
CONFIGS = {
    "dw4": CNFConfig(n_nodes=4, dim=2, n_features=1, hidden=64, mlp_width=128, mlp_depth=3, n_blocks=3,
                     base_scale=1.0, sigma_min=0.01),
    "lj13": CNFConfig(n_nodes=13, dim=3, n_features=1, hidden=64, mlp_width=128, mlp_depth=3, n_blocks=3,
                      base_scale=1.0, sigma_min=0.01),
    "aldp": CNFConfig(n_nodes=22, dim=3, n_features=22, hidden=32, mlp_width=64, mlp_depth=2, n_blocks=3,
                      base_scale=0.2, sigma_min=1e-6),
    "qm9": CNFConfig(n_nodes=29, dim=3, n_features=1, hidden=32, mlp_width=256, mlp_depth=4, n_blocks=5,
                     base_scale=2.0, sigma_min=1e-6),
}


# ----------------------------------------------------------------------------------------------
# parameters: flax path names, canonical (= jax tree-flatten, i.e. sorted-key) order
# ----------------------------------------------------------------------------------------------
def param_spec(cfg: CNFConfig) -> List[Tuple[str, Tuple[int, ...]]]:
    """Ordered (flax path, shape) list.  Order = sorted-key pytree flatten order, so that
    ``jax.flatten_util.ravel_pytree(params["params"])[0]`` of a reference checkpoint is the flat blob.

    Names follow flax auto-naming at ``build_cnf.py:79,85``, ``egnn.py:42-47,83,99,167-168,188``,
    ``mlp.py:13-16``."""
    H, T, K = cfg.hidden, cfg.time_embedding_dim, cfg.n_blocks
    U = cfg.units                           # mlp_units (egnn.py:43-47); m_ij has width U[-1]
    L = len(U)
    tree: Dict[str, Tuple[int, ...]] = {}

    def dense(prefix, fan_in, fan_out):
        tree[prefix + "/bias"] = (fan_out,)
        tree[prefix + "/kernel"] = (fan_in, fan_out)

    for k in range(K):
        blk = f"EGNN_0/{k}"
        dense(f"{blk}/Dense_0", U[-1], 1)   # phi_x output layer (egnn.py:83-85)
        dense(f"{blk}/Dense_1", U[-1], 1)   # gate (egnn.py:99)
        for l in range(L):                  # phi_e (egnn.py:43)
            dense(f"{blk}/phi_e/Dense_{l}", 2 * H + 1 if l == 0 else U[l - 1], U[l])
        hu = U + (H,)
        for l in range(L + 1):              # phi_h = MLP((*mlp_units, H)) (egnn.py:46)
            dense(f"{blk}/phi_h/Dense_{l}", U[-1] + H if l == 0 else hu[l - 1], hu[l])
        for l in range(L):                  # phi_x_torso (egnn.py:45)
            dense(f"{blk}/phi_x_torso/Dense_{l}", U[-1] if l == 0 else U[l - 1], U[l])
        dense(f"EGNN_0/Dense_{k}", H + T, H)  # per-block node Dense (egnn.py:167)
    tree["EGNN_0/final_scaling"] = ()
    tree["Embed_0/embedding"] = (cfg.n_features, H)

    def sort_key(path: str):
        # flax flattens nested dicts level by level with sorted keys
        return tuple(path.split("/"))

    return [(p, tree[p]) for p in sorted(tree, key=sort_key)]


def param_count(cfg: CNFConfig) -> int:
    return int(sum(int(np.prod(s)) for _, s in param_spec(cfg)))


def init_params(cfg: CNFConfig, seed: int = 0, x_out_scale: float = 1.0) -> Params:
    """flax-default-like init with numpy's PCG64 (JAX threefry cannot be reproduced offline).

    Kernels: lecun-normal (truncated normal, std = 1/sqrt(fan_in)/0.8796); biases zero; phi_x output
    kernel: variance_scaling(0.001, fan_avg, uniform) (egnn.py:83-85) times ``x_out_scale``;
    Embed: normal(1/sqrt(n_features)); final_scaling = 1 (egnn.py:188)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    p: Params = {}
    for path, shape in param_spec(cfg):
        if path.endswith("/bias"):
            p[path] = np.zeros(shape, np.float32)
        elif path.endswith("final_scaling"):
            p[path] = np.ones(shape, np.float32)
        elif path.endswith("embedding"):
            p[path] = (rng.standard_normal(shape) / np.sqrt(shape[0])).astype(np.float32)
        elif path.endswith("Dense_0/kernel") and path.count("/") == 3 and "/phi_" not in path:
            # EGNN_0/{k}/Dense_0/kernel: phi_x output layer
            fan_in, fan_out = shape
            lim = np.sqrt(3.0 * cfg.variance_scaling_init / ((fan_in + fan_out) / 2.0))
            p[path] = (rng.uniform(-lim, lim, shape) * x_out_scale).astype(np.float32)
        else:
            fan_in = shape[0]
            z = rng.standard_normal(shape)
            while np.any(np.abs(z) > 2):
                bad = np.abs(z) > 2
                z[bad] = rng.standard_normal(int(bad.sum()))
            p[path] = (z * np.sqrt(1.0 / fan_in) / 0.87962566103423978).astype(np.float32)
    return p


def stress_params(params: Params, cfg: CNFConfig, seed: int = 7, bias_std: float = 0.05) -> Params:
    """A 'trained-looking' variant: nonzero biases and a phi_x output scaled x100 so the flow moves
    particles by O(0.3) (the default init's field is ~1e-3; egnn.py:128)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    out = {}
    for k, v in params.items():
        v = v.copy()
        if k.endswith("/bias"):
            v = (rng.standard_normal(v.shape) * bias_std).astype(np.float32)
        if k.count("/") == 3 and k.split("/")[2] == "Dense_0" and k.endswith("kernel"):
            v = (v * 100.0).astype(np.float32)
        out[k] = v
    return out


def flatten_params(params: Params, cfg: CNFConfig) -> np.ndarray:
    return np.concatenate([np.asarray(params[p], np.float32).reshape(-1) for p, _ in param_spec(cfg)])


def unflatten_params(flat: np.ndarray, cfg: CNFConfig) -> Params:
    out, off = {}, 0
    for p, s in param_spec(cfg):
        n = int(np.prod(s))
        out[p] = np.asarray(flat[off:off + n], np.float32).reshape(s)
        off += n
    assert off == flat.size
    return out


# ----------------------------------------------------------------------------------------------
# building blocks
# ----------------------------------------------------------------------------------------------
def fully_connected_edges(n_nodes: int) -> Tuple[np.ndarray, np.ndarray]:
    """graph.py:6-14: receiver-major; receivers = i repeated N-1 times, senders = (i+1+j) % N."""
    receivers = np.repeat(np.arange(n_nodes), n_nodes - 1)
    senders = np.array([(i + 1 + j) % n_nodes for i in range(n_nodes) for j in range(n_nodes - 1)],
                       dtype=np.int64)
    return senders, receivers


def timestep_embedding(t: np.ndarray, dim: int, dtype=np.float32) -> np.ndarray:
    """build_cnf.py:18-32 (fp32 op order of the JAX code: t*1000, log(1e4)/(half-1), exp(k * -e))."""
    f = np.dtype(dtype).type
    t = np.asarray(t, dtype) * f(1000)
    half = dim // 2
    e = f(np.log(f(10000))) / f(half - 1)
    freqs = np.exp(np.arange(half).astype(dtype) * -e).astype(dtype)
    arg = t[:, None] * freqs[None, :]
    return np.concatenate([np.sin(arg), np.cos(arg)], axis=1).astype(dtype)


def timestep_frequencies(dim: int) -> np.ndarray:
    """The fp32 frequency table used by :func:`timestep_embedding` (exported for the device side)."""
    f = np.float32
    half = dim // 2
    e = f(np.log(f(10000))) / f(half - 1)
    return np.exp(np.arange(half).astype(f) * -e).astype(f)


def _sigmoid(z):
    return 1.0 / (1.0 + np.exp(-z))


def _silu_dual(z, dz):
    s = _sigmoid(z)
    y = z * s
    if dz is None:
        return y, None
    ds = s * (1.0 + z * (1.0 - s))
    return y, ds[:, None] * dz


def _dense(x, dx, params, prefix, dtype):
    W = params[prefix + "/kernel"].astype(dtype)
    b = params[prefix + "/bias"].astype(dtype)
    y = x @ W + b
    dy = None if dx is None else dx @ W
    return y, dy


def _mlp(x, dx, params, prefix, n_layers, activate_final, dtype):
    """mlp.py:7-19 (SiLU between layers, optional final SiLU)."""
    for l in range(n_layers):
        x, dx = _dense(x, dx, params, f"{prefix}/Dense_{l}", dtype)
        if l < n_layers - 1 or activate_final:
            x, dx = _silu_dual(x, dx)
    return x, dx


def _egcl(cfg, params, blk, vec, dvec, h, dh, dtype):
    """egnn.py:49-114 for a batch [B, N, ...]; tangents carry an extra K axis at position 1."""
    f = np.dtype(dtype).type
    N = cfg.n_nodes
    senders, receivers = fully_connected_edges(N)
    nn1 = N - 1                                                  # avg_num_neighbours (egnn.py:69)

    r = vec[:, receivers] - vec[:, senders]                      # egnn.py:73
    x2 = np.sum(r ** 2, axis=-1, keepdims=True)                  # numerical.py:9
    zero = x2 == 0
    length = np.sqrt(np.where(zero, f(1), x2))                   # numerical.py:10
    len2 = length ** 2                                           # egnn.py:76 (lengths**2)
    dr = dlength = dlen2 = None
    if dvec is not None:
        dr = dvec[:, :, receivers] - dvec[:, :, senders]
        rdr = np.sum(r[:, None] * dr, axis=-1, keepdims=True)    # d(x2)/2
        dlength = np.where(zero[:, None], f(0), rdr / length[:, None])
        dlen2 = f(2) * length[:, None] * dlength

    edge_in = np.concatenate([h[:, senders], h[:, receivers], len2], axis=-1)   # egnn.py:76
    dedge_in = None
    if dh is not None:
        dedge_in = np.concatenate([dh[:, :, senders], dh[:, :, receivers], dlen2], axis=-1)

    L = len(cfg.units)
    m, dm = _mlp(edge_in, dedge_in, params, f"{blk}/phi_e", L, True, dtype)          # egnn.py:79
    px, dpx = _mlp(m, dm, params, f"{blk}/phi_x_torso", L, True, dtype)               # egnn.py:82
    px, dpx = _dense(px, dpx, params, f"{blk}/Dense_0", dtype)                         # egnn.py:83-85

    denom = f(cfg.normalization_constant) + length
    shifts = px * r / denom                                                            # egnn.py:87-91
    shift_i = shifts.reshape(shifts.shape[0], N, nn1, -1).sum(axis=2)                  # scatter_sum
    vec_out = shift_i / f(nn1)                                                         # egnn.py:95
    dvec_out = None
    if dvec is not None:
        dshifts = (dpx * r[:, None] + px[:, None] * dr) / denom[:, None] \
            - (px * r)[:, None] * dlength / (denom[:, None] ** 2)
        dvec_out = dshifts.reshape(dshifts.shape[:2] + (N, nn1, -1)).sum(axis=3) / f(nn1)

    e, de = _dense(m, dm, params, f"{blk}/Dense_1", dtype)                             # egnn.py:99
    g = _sigmoid(e)                                                                    # egnn.py:101
    gm = m * g
    sq = f(np.sqrt(f(nn1)))
    m_i = gm.reshape(gm.shape[0], N, nn1, -1).sum(axis=2) / sq                         # egnn.py:102-104
    dm_i = None
    if dm is not None:
        dg = (g * (1 - g))[:, None] * de
        dgm = dg * m[:, None] + g[:, None] * dm
        dm_i = dgm.reshape(dgm.shape[:2] + (N, nn1, -1)).sum(axis=3) / sq

    phi_h_in = np.concatenate([m_i, h], axis=-1)                                       # egnn.py:105
    dphi_h_in = None if dh is None else np.concatenate([dm_i, dh], axis=-1)
    hout, dhout = _mlp(phi_h_in, dphi_h_in, params, f"{blk}/phi_h", L + 1, False, dtype)  # egnn.py:106
    h_new = hout + h                                                                   # egnn.py:111
    dh_new = None if dh is None else dhout + dh
    vec_new = vec + vec_out                                                            # egnn.py:113
    dvec_new = None if dvec is None else dvec + dvec_out
    return vec_new, dvec_new, h_new, dh_new


def egnn_vector_field(params: Params, cfg: CNFConfig, x: np.ndarray, t: np.ndarray, feat: np.ndarray,
                      tangents: Optional[np.ndarray] = None, dtype=np.float64):
    """FlatEgnn.__call__ (build_cnf.py:68-93) + EGNN.call_single (egnn.py:144-190), batched.

    x [B, N*D], t [B], feat int [B, N]; tangents [B, K, N*D] (forward-mode directions) or None.
    Returns v [B, N*D] and, with tangents, J @ tangents [B, K, N*D]."""
    f = np.dtype(dtype).type
    N, D, K = cfg.n_nodes, cfg.dim, cfg.n_blocks
    B = x.shape[0]
    pos = np.asarray(x, dtype).reshape(B, N, D)
    feat = np.asarray(feat).reshape(B, N)
    h = params["Embed_0/embedding"].astype(dtype)[feat]                   # build_cnf.py:79-80
    temb = timestep_embedding(np.asarray(t, np.float32), cfg.time_embedding_dim).astype(dtype)

    mean_in = pos.mean(axis=1, keepdims=True)                             # egnn.py:160
    vec = pos - mean_in
    vec0 = vec
    dvec = dvec0 = dh = dmean_in = None
    if tangents is not None:
        tp = np.asarray(tangents, dtype).reshape(B, -1, N, D)
        dmean_in = tp.mean(axis=2, keepdims=True)
        dvec = tp - dmean_in
        dvec0 = dvec
        dh = np.zeros((B, tp.shape[1], N, cfg.hidden), dtype)

    for k in range(K):                                                    # egnn.py:165-178
        hin = np.concatenate([h, np.repeat(temb[:, None], N, axis=1)], axis=-1)
        dhin = None if dh is None else np.concatenate(
            [dh, np.zeros(dh.shape[:3] + (cfg.time_embedding_dim,), dtype)], axis=-1)
        h, dh = _dense(hin, dhin, params, f"EGNN_0/Dense_{k}", dtype)
        vec, dvec, h, dh = _egcl(cfg, params, f"EGNN_0/{k}", vec, dvec, h, dh, dtype)

    fs = params["EGNN_0/final_scaling"].astype(dtype)
    v = ((vec - vec0) - mean_in) * fs                                     # egnn.py:183-188
    v = v.reshape(B, N * D)
    if tangents is None:
        return v
    dv = ((dvec - dvec0) - dmean_in) * fs
    return v, dv.reshape(B, -1, N * D)


def divergence(params, cfg, x, t, feat, eps=None, dtype=np.float64):
    """Exact trace over the full N*D space (sample_and_log_prob.py:64-66) when ``eps`` is None,
    Hutchinson eps^T J eps otherwise (:75-77).  Returns (v, div)."""
    B, ND = x.shape
    if eps is None:
        tang = np.broadcast_to(np.eye(ND, dtype=dtype), (B, ND, ND))
        v, jv = egnn_vector_field(params, cfg, x, t, feat, tang, dtype)
        return v, np.einsum("bkk->b", jv)
    v, jv = egnn_vector_field(params, cfg, x, t, feat, np.asarray(eps, dtype)[:, None], dtype)
    return v, np.sum(jv[:, 0] * np.asarray(eps, dtype), axis=-1)


# ----------------------------------------------------------------------------------------------
# base distribution (zero_com_base.py + build_cnf.py:46-61)
# ----------------------------------------------------------------------------------------------
def base_sample(z: np.ndarray, cfg: CNFConfig, dtype=np.float32) -> np.ndarray:
    """x0 = s * (z - mean_N z) for a standard-normal draw z [B, N*D] (zero_com_base.py:88-93 then the
    ScalarAffine forward of build_cnf.py:46)."""
    N, D = cfg.n_nodes, cfg.dim
    z = np.asarray(z, dtype).reshape(-1, N, D)
    x = z - z.mean(axis=1, keepdims=True)
    return (np.dtype(dtype).type(cfg.base_scale) * x).reshape(-1, N * D)


def base_log_prob(y: np.ndarray, cfg: CNFConfig, dtype=np.float64) -> np.ndarray:
    """Transformed(FlatZeroCoMGaussian, Lambda(ScalarAffine)).log_prob:
    log N_{(N-1)D}(remove_mean(y/s)) - (N-1) D log s   (zero_com_base.py:64-84, build_cnf.py:50-57)."""
    f = np.dtype(dtype).type
    N, D = cfg.n_nodes, cfg.dim
    s = f(cfg.base_scale)
    u = np.asarray(y, dtype).reshape(-1, N, D) * (f(1) / s)
    u = u - u.mean(axis=1, keepdims=True)
    r2 = np.sum(u ** 2, axis=(-1, -2))
    dof = (N - 1) * D
    log_norm = f(-0.5) * f(dof) * f(np.log(f(2) * f(np.pi)))
    ildj = -f(N * D) * f(np.log(s)) * f(N - 1) / f(N)
    return (f(-0.5) * r2 + log_norm + ildj).astype(dtype)


def ot_conditional_vf(x0, x1, t, sigma_min):
    """core.py:35-39."""
    t = np.asarray(t)[..., None]
    x_t = (1 - (1 - sigma_min) * t) * x0 + t * x1
    u_t = x1 - (1 - sigma_min) * x0
    return x_t, u_t


# ----------------------------------------------------------------------------------------------
# ODE solvers (diffrax semantics, restated; see module docstring)
# ----------------------------------------------------------------------------------------------
DOPRI5_A = [
    [1 / 5],
    [3 / 40, 9 / 40],
    [44 / 45, -56 / 15, 32 / 9],
    [19372 / 6561, -25360 / 2187, 64448 / 6561, -212 / 729],
    [9017 / 3168, -355 / 33, 46732 / 5247, 49 / 176, -5103 / 18656],
    [35 / 384, 0.0, 500 / 1113, 125 / 192, -2187 / 6784, 11 / 84],
]
DOPRI5_C = [0.0, 1 / 5, 3 / 10, 4 / 5, 8 / 9, 1.0, 1.0]
DOPRI5_B = [35 / 384, 0.0, 500 / 1113, 125 / 192, -2187 / 6784, 11 / 84, 0.0]
DOPRI5_BERR = [35 / 384 - 1951 / 21600, 0.0, 500 / 1113 - 22642 / 50085, 125 / 192 - 451 / 720,
               -2187 / 6784 + 12231 / 42400, 11 / 84 - 649 / 6300, -1.0 / 60.0]

SOLVERS = ("euler", "dopri5")
DIV_NONE, DIV_HUTCH, DIV_EXACT = "none", "hutchinson", "exact"


def _clip_to_end(tnext, t1, f):
    tol = f(1e-6) if f == np.float32 else f(1e-10)
    return np.where(tnext > t1 - tol, t1, tnext)


def _rms(xs):
    tot = sum(np.sum(np.asarray(a) ** 2, axis=-1) for a in xs)
    n = sum(a.shape[-1] for a in xs)
    return np.sqrt(tot / n)


class _Field:
    """Joint field on (x, logp) in reparametrised time tau = dir * t (diffrax reverse-time handling)."""

    def __init__(self, params, cfg, feat, div_mode, eps, direction, dtype, apply_fn=None):
        self.params, self.cfg, self.feat = params, cfg, feat
        self.div_mode, self.eps, self.dir, self.dtype = div_mode, eps, direction, dtype
        self.apply_fn = apply_fn
        self.nfe = 0

    def __call__(self, tau, x, idx):
        f = np.dtype(self.dtype).type
        t = (f(self.dir) * tau).astype(self.dtype)
        self.nfe += 1
        feat = self.feat[idx]
        if self.apply_fn is not None:   # a user-supplied field (KAT-1's linear field)
            v, div = self.apply_fn(x, t, self.div_mode, None if self.eps is None else self.eps[idx])
        elif self.div_mode == DIV_NONE:
            v = egnn_vector_field(self.params, self.cfg, x, t, feat, dtype=self.dtype)
            div = np.zeros(x.shape[0], self.dtype)
        elif self.div_mode == DIV_EXACT:
            v, div = divergence(self.params, self.cfg, x, t, feat, None, self.dtype)
        else:
            v, div = divergence(self.params, self.cfg, x, t, feat, self.eps[idx], self.dtype)
        return (f(self.dir) * v).astype(self.dtype), (f(self.dir) * div).astype(self.dtype)


def odeint(field: _Field, x0, tau0: float, tau1: float, solver: str, dt0: Optional[float],
           rtol=1e-5, atol=1e-5, dtmin=1e-5, max_steps=4096, track_logp=False):
    """Integrate the joint field from tau0 to tau1 (tau0 < tau1) for a batch; every molecule keeps its own
    (tau, dt) when adaptive, exactly as under jax.vmap (finished lanes are frozen).

    Returns x1 [B, ND], logp1 [B], nfe [B]."""
    dtype = field.dtype
    f = np.dtype(dtype).type
    x = np.array(x0, dtype, copy=True)
    B = x.shape[0]
    lp = np.zeros(B, dtype)
    tau = np.full(B, f(tau0), dtype)
    T1 = f(tau1)
    nfe = np.zeros(B, np.int64)
    idx_all = np.arange(B)

    def F(tt, xx, idx):
        v, d = field(tt, xx, idx)
        nfe[idx] += 1
        return v, (d if track_logp else np.zeros_like(d))

    if solver == "euler":
        assert dt0 is not None, "Euler needs a fixed step"
        dt = f(dt0)
        tnext = _clip_to_end(tau + dt, T1, f)
        steps = 0
        while np.any(tau < T1):
            steps += 1
            if steps > max_steps:
                raise RuntimeError("max_steps exceeded")
            h = (tnext - tau).astype(dtype)
            v, d = F(tau, x, idx_all)
            x = (x + h[:, None] * v).astype(dtype)
            lp = (lp + h * d).astype(dtype)
            tau = tnext
            tnext = _clip_to_end(tau + dt, T1, f)
        return x, lp, nfe

    assert solver == "dopri5"
    A = [[f(a) for a in row] for row in DOPRI5_A]
    Cc = [f(c) for c in DOPRI5_C]
    Bs = [f(b) for b in DOPRI5_B]
    Be = [f(b) for b in DOPRI5_BERR]

    if dt0 is None:
        # Hairer's initial step (diffrax _select_initial_step), error order 5
        kx0, kl0 = F(tau, x, idx_all)
        sx = f(atol) + np.abs(x) * f(rtol)
        sl = f(atol) + np.abs(lp) * f(rtol)
        # rms over the leaves of y: (x, logp) for the joint solves, x alone for sample_cnf (y0 = x0)
        leaves = (lambda a, b: [a, b[:, None]]) if track_logp else (lambda a, b: [a])
        d0 = _rms(leaves(x / sx, lp / sl))
        d1 = _rms(leaves(kx0 / sx, kl0 / sl))
        cond = (d0 < 1e-5) | (d1 < 1e-5)
        d1s = np.where(cond, f(1), d1)
        h0 = np.where(cond, f(1e-6), f(0.01) * (d0 / d1s)).astype(dtype)
        x1 = x + h0[:, None] * kx0
        l1 = lp + h0 * kl0
        kx1, kl1 = F(tau + h0, x1, idx_all)
        d2 = _rms(leaves((kx1 - kx0) / sx, (kl1 - kl0) / sl)) / h0
        maxd = np.maximum(d1, d2)
        h1 = np.where(maxd <= 1e-15, np.maximum(f(1e-6), h0 * f(1e-3)),
                      (f(0.01) / np.maximum(maxd, f(1e-30))) ** f(1 / 5)).astype(dtype)
        dt = np.minimum(f(100) * h0, h1).astype(dtype)
        at_dtmin = dt <= f(dtmin)
        dt = np.maximum(dt, f(dtmin)).astype(dtype)
    else:
        dt = np.full(B, f(dt0), dtype)
        at_dtmin = np.zeros(B, bool)
    tnext = _clip_to_end(np.minimum(tau + dt, T1), T1, f).astype(dtype)

    # FSAL: k1 = f(t0, y0) (solver init)
    k1x, k1l = F(tau, x, idx_all)
    steps = np.zeros(B, np.int64)
    while True:
        active = tau < T1
        if not np.any(active):
            break
        steps += active
        if np.any(steps > max_steps):
            raise RuntimeError("max_steps exceeded")
        idx = idx_all[active]
        t0a, x0a, l0a = tau[active], x[active], lp[active]
        h = (tnext[active] - t0a).astype(dtype)
        kx = [k1x[active]]
        kl = [k1l[active]]
        for s in range(1, 7):
            ax = sum(A[s - 1][j] * kx[j] for j in range(s))
            al = sum(A[s - 1][j] * kl[j] for j in range(s))
            ys = (x0a + h[:, None] * ax).astype(dtype)
            ls = (l0a + h * al).astype(dtype)
            vx, vl = F((t0a + Cc[s] * h).astype(dtype), ys, idx)
            kx.append(vx)
            kl.append(vl)
        # stage 7 is evaluated at y1 (a_7 = b): ys == y1
        x1 = ys
        l1 = ls
        ex = h[:, None] * sum(Be[j] * kx[j] for j in range(7))
        el = h * sum(Be[j] * kl[j] for j in range(7))
        if dt0 is not None:
            keep = np.ones(len(idx), bool)
            new_dt = np.full(len(idx), f(dt0), dtype)
            new_atmin = np.zeros(len(idx), bool)
        else:
            scx = f(atol) + np.maximum(np.abs(x0a), np.abs(x1)) * f(rtol)
            scl = f(atol) + np.maximum(np.abs(l0a), np.abs(l1)) * f(rtol)
            err = _rms([ex / scx, (el / scl)[:, None]] if track_logp else [ex / scx])
            keep = (err < 1) | at_dtmin[active]
            with np.errstate(divide="ignore"):
                inv = f(1) / err
            factor = np.clip(f(0.9) * inv ** f(1 / 5), np.where(keep, f(1), f(0.2)), f(10)).astype(dtype)
            factor = np.where(np.isnan(factor), f(1), factor)
            new_dt = (h * factor).astype(dtype)
            new_atmin = new_dt <= f(dtmin)
            new_dt = np.maximum(new_dt, f(dtmin)).astype(dtype)
        # commit
        tn = np.where(keep, tnext[active], t0a).astype(dtype)
        x[active] = np.where(keep[:, None], x1, x0a)
        lp[active] = np.where(keep, l1, l0a)
        k1x_a = np.where(keep[:, None], kx[6], kx[0])
        k1l_a = np.where(keep, kl[6], kl[0])
        k1x[active] = k1x_a
        k1l[active] = k1l_a
        tau[active] = tn
        at_dtmin[active] = new_atmin
        if dt0 is not None:
            tnext[active] = _clip_to_end(tn + f(dt0), T1, f)
        else:
            tnext[active] = _clip_to_end(np.minimum(tn + new_dt, T1), T1, f)
    return x, lp, nfe


# ----------------------------------------------------------------------------------------------
# the CNF API (sample_and_log_prob.py), batched with explicit noise
# ----------------------------------------------------------------------------------------------
def sample_cnf(params, cfg, x0, feat, solver="dopri5", dt0=0.05, rtol=1e-5, atol=1e-5,
               dtmin=1e-5, dtype=np.float32, apply_fn=None):
    """sample_and_log_prob.py:11-38 with x0 supplied (= cnf.sample_base, see :func:`base_sample`).
    ``dt0=None`` selects the adaptive PID path (:34-37)."""
    field = _Field(params, cfg, np.asarray(feat), DIV_NONE, None, 1.0, dtype, apply_fn)
    x1, _, nfe = odeint(field, x0, 0.0, 1.0, solver, dt0, rtol, atol, dtmin)
    return x1, nfe


def get_log_prob(params, cfg, x, feat, eps=None, approx=False, solver="dopri5", dt0=0.05,
                 rtol=1e-5, atol=1e-5, dtmin=1e-5, dtype=np.float32, apply_fn=None, log_prob_base=None):
    """sample_and_log_prob.py:41-94: solve t=1 -> 0 on (x, 0); returns (log_p, log_p0, delta, nfe)."""
    div_mode = DIV_HUTCH if approx else DIV_EXACT
    field = _Field(params, cfg, np.asarray(feat), div_mode, eps, -1.0, dtype, apply_fn)
    x0, dl, nfe = odeint(field, x, -1.0, 0.0, solver, dt0, rtol, atol, dtmin, track_logp=True)
    lp0 = (log_prob_base or (lambda y: base_log_prob(y, cfg, dtype)))(x0)
    return (lp0 + dl).astype(dtype), lp0, dl, nfe, x0


def sample_and_log_prob(params, cfg, x0, feat, eps=None, approx=False, solver="dopri5", dt0=None,
                        rtol=1e-5, atol=1e-5, dtmin=1e-5, dtype=np.float32, apply_fn=None, log_prob_base=None):
    """sample_and_log_prob.py:97-149 (fixed-step branch repaired to y0=(x0, 0)).
    Returns (x1, log_q, nfe) with log_q = log p0(x0) - l(1) (:147)."""
    div_mode = DIV_HUTCH if approx else DIV_EXACT
    field = _Field(params, cfg, np.asarray(feat), div_mode, eps, 1.0, dtype, apply_fn)
    x1, dl, nfe = odeint(field, x0, 0.0, 1.0, solver, dt0, rtol, atol, dtmin, track_logp=True)
    lp0 = (log_prob_base or (lambda y: base_log_prob(y, cfg, dtype)))(x0)
    return x1, (lp0 - dl).astype(dtype), nfe


# ----------------------------------------------------------------------------------------------
# targets and eval reductions ("next" rows of SURVEY.md section 8f)
# ----------------------------------------------------------------------------------------------
def lj_energy(x, n_nodes, dim, epsilon=1.0, tau=1.0, r=1.0, harmonic_potential_coef=0.5):
    """leonard_jones.py:10-27 (ordered-pair double count, eps/(2 tau), harmonic CoM term)."""
    x = np.asarray(x, np.float64).reshape(-1, n_nodes, dim)
    s, rcv = fully_connected_edges(n_nodes)
    vec = x[:, s] - x[:, rcv]
    x2 = np.sum(vec ** 2, -1)
    d = np.sqrt(np.where(x2 == 0, 1.0, x2))
    r = np.asarray(r, np.float64)
    rr = r[rcv] if r.ndim else r     # per-node r: the receiver's (leonard_jones.py:14-16,20)
    term = (rr / d) ** 12 - 2 * (rr / d) ** 6
    e = epsilon / (2 * tau) * term.sum(-1)
    com = x.mean(axis=1, keepdims=True)
    return e + harmonic_potential_coef * np.sum((x - com) ** 2, axis=(-1, -2))


def dw_energy(x, n_nodes, dim, a=0.0, b=-4.0, c=0.9, d0=4.0, tau=1.0):
    """double_well.py:9-19."""
    x = np.asarray(x, np.float64).reshape(-1, n_nodes, dim)
    s, rcv = fully_connected_edges(n_nodes)
    vec = x[:, s] - x[:, rcv]
    x2 = np.sum(vec ** 2, -1)
    d = np.sqrt(np.where(x2 == 0, 1.0, x2)) - d0
    return np.sum(a * d + b * d ** 2 + c * d ** 4, axis=-1) / tau / 2


def _logsumexp(a, b=None):
    """jax.nn.logsumexp(a, b): the max shift is replaced by 0 when it is not finite, so +inf entries give +inf and
    -inf entries weight 0 (no exp(inf - inf) = NaN)."""
    a = np.asarray(a, np.float64)
    m = np.max(a)
    m0 = m if np.isfinite(m) else 0.0
    w = np.ones_like(a) if b is None else np.asarray(b, np.float64)
    with np.errstate(over="ignore", divide="ignore"):
        return m0 + np.log(np.sum(w * np.exp(a - m0)))


def forward_ess(log_w, mask=None):
    """evaluation.py:10-22."""
    log_w = np.asarray(log_w, np.float64)
    mask = np.ones_like(log_w) if mask is None else np.asarray(mask, np.float64)
    log_w = np.where(mask > 0, log_w, 0.0)
    n = mask.sum()
    log_z_inv = _logsumexp(-log_w, mask) - np.log(n)
    log_z_exp = _logsumexp(log_w, mask) - np.log(n)
    return float(np.exp(-log_z_inv - log_z_exp))


def reverse_ess(log_w):
    """setup_training.py:182: 1 / sum(softmax(log_w)^2) / n."""
    log_w = np.asarray(log_w, np.float64)
    return float(np.exp(2 * _logsumexp(log_w) - _logsumexp(2 * log_w)) / log_w.size)


# ----------------------------------------------------------------------------------------------
# the test-set evaluation leg: evaluation.py:25-115, setup_training.py:190-215
# ----------------------------------------------------------------------------------------------
def setup_padded_reshaped_data(data, interval_length, reshape_axis=0):
    """evaluation.py:25-50: pad the leading axis with zeros to a multiple of interval_length and reshape;
    returns (reshaped data, mask) with mask 1 on the real rows."""
    data = np.asarray(data)
    n = data.shape[0]
    pad = (interval_length - n % interval_length) % interval_length
    padded = np.concatenate([data, np.zeros((pad,) + data.shape[1:], data.dtype)], axis=0)
    mask = np.zeros(n + pad, dtype=int)
    mask[:n] = 1
    npad = n + pad
    if reshape_axis == 0:
        shape = (interval_length, npad // interval_length)
    else:
        assert reshape_axis == 1
        shape = (npad // interval_length, interval_length)
    return padded.reshape(shape + data.shape[1:]), mask.reshape(shape)


def maybe_masked_mean(array, mask=None):
    """numerical.py:43-52."""
    array = np.asarray(array, np.float64)
    if mask is None:
        return float(array.mean())
    mask = np.asarray(mask, np.float64)
    divisor = mask.sum()
    return float(np.where(mask > 0, array, 0.0).sum() * (0.0 if divisor == 0 else 1.0 / divisor))


def eval_test_set(params, cfg, x, feat, batch_size, eps=None, approx=False, solver="euler", dt0=0.05,
                  dtype=np.float64, target_log_prob=None):
    """eval_fn (evaluation.py:59-115) with eval_on_data_batch_fn (setup_training.py:190-215) and, with a target,
    calculate_forward_ess on the flattened log_w and mask (setup_training.py:239-241).  Per padded batch:
    get_log_prob of every molecule (vmap), masked means of log_q / log_prob_base / delta; the batches' infos are
    weighted by their share of the real rows (evaluation.py:92-97).  Padded rows never enter a mean (their values are
    replaced by 0 under the mask), so only the real rows are solved here.  eps: [n, N*D] Hutchinson probes of the
    real rows (approx=True)."""
    x = np.asarray(x, np.float32)
    n = x.shape[0]
    xb, mask = setup_padded_reshaped_data(x, batch_size, reshape_axis=1)
    lp, lp0, dl, _, _ = get_log_prob(params, cfg, x, feat, eps=eps, approx=approx, solver=solver, dt0=dt0,
                                     dtype=dtype)
    pad = xb.shape[0] * batch_size - n
    full = lambda a: np.concatenate([np.asarray(a, np.float64), np.zeros(pad)]).reshape(mask.shape)
    lq_b, lp0_b, dl_b = full(lp), full(lp0), full(dl)
    w = mask.sum(-1) / mask.sum()
    info = {"test_log_lik": float(sum(w[b] * maybe_masked_mean(lq_b[b], mask[b]) for b in range(len(w)))),
            "test_log_prob_base": float(sum(w[b] * maybe_masked_mean(lp0_b[b], mask[b]) for b in range(len(w)))),
            "test_delta_log_lik": float(sum(w[b] * maybe_masked_mean(dl_b[b], mask[b]) for b in range(len(w))))}
    if target_log_prob is not None:
        log_w = full(np.asarray(target_log_prob(x), np.float64) - np.asarray(lp, np.float64))
        info["forward_ess"] = forward_ess(log_w.reshape(-1), mask.reshape(-1))
    return info
