"""Parameter layout of the EGNN vector field: flax path names in jax tree-flatten order.

The flat fp32 blob handed to ``ecnf_create`` is ``jax.flatten_util.ravel_pytree(params["params"])[0]`` of a
reference checkpoint: sorted keys at every level, bias before kernel.  Names are the flax auto-names of
``ecnf/cnf/build_cnf.py:79,85``, ``ecnf/nets/egnn.py:42-47,83,99,167-168,188`` and ``ecnf/nets/mlp.py:13-16``.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Mapping, Tuple

import numpy as np


@dataclass(frozen=True)
class CNFConfig:
    """build_cnf(...) arguments (build_cnf.py:34-44) with mlp_units = (mlp_width,) * mlp_depth."""
    n_nodes: int
    dim: int
    n_features: int = 1
    hidden: int = 64                 # n_invariant_feat_hidden
    time_embedding_dim: int = 8
    mlp_width: int = 128
    mlp_depth: int = 3
    n_blocks: int = 3                # n_blocks_egnn
    base_scale: float = 1.0
    sigma_min: float = 0.01
    normalization_constant: float = 1.0
    # the reference network's widths when this (kernel) shape zero-pads them (kernel_config); () / 0: not padded.
    # flatten_params pads reference-shaped params onto this shape by itself, so every entry point that takes params
    # (EcnfHandle, update_params, the Trainer, dataio) accepts them
    ref_mlp_units: Tuple[int, ...] = ()
    ref_hidden: int = 0

    @property
    def event_dim(self) -> int:
        return self.n_nodes * self.dim

    @property
    def mlp_units(self) -> Tuple[int, ...]:
        return (self.mlp_width,) * self.mlp_depth


# examples/config/{dw4,lj13,aldp,qm9}.yaml (`flow:` block); QM9 at the BASELINE shape N = 29
CONFIGS: Dict[str, CNFConfig] = {
    "dw4": CNFConfig(n_nodes=4, dim=2, n_features=1, hidden=64, mlp_width=128, mlp_depth=3, n_blocks=3,
                     base_scale=1.0, sigma_min=0.01),
    "lj13": CNFConfig(n_nodes=13, dim=3, n_features=1, hidden=64, mlp_width=128, mlp_depth=3, n_blocks=3,
                      base_scale=1.0, sigma_min=0.01),
    "aldp": CNFConfig(n_nodes=22, dim=3, n_features=22, hidden=32, mlp_width=64, mlp_depth=2, n_blocks=3,
                      base_scale=0.2, sigma_min=1e-6),
    "qm9": CNFConfig(n_nodes=29, dim=3, n_features=1, hidden=32, mlp_width=256, mlp_depth=4, n_blocks=5,
                     base_scale=2.0, sigma_min=1e-6),
}


def param_spec(cfg: CNFConfig) -> List[Tuple[str, Tuple[int, ...]]]:
    H, T, M, L, K = cfg.hidden, cfg.time_embedding_dim, cfg.mlp_width, cfg.mlp_depth, cfg.n_blocks
    if K > 10:
        raise ValueError("n_blocks > 10 changes the lexicographic order of the block names")
    shapes: Dict[Tuple[str, ...], Tuple[int, ...]] = {}

    def dense(path, fan_in, fan_out):
        shapes[path + ("bias",)] = (fan_out,)
        shapes[path + ("kernel",)] = (fan_in, fan_out)

    for k in range(K):
        blk = ("EGNN_0", str(k))
        dense(blk + ("Dense_0",), M, 1)                      # phi_x output Dense(1)
        dense(blk + ("Dense_1",), M, 1)                      # gate Dense(1)
        for l in range(L):
            dense(blk + ("phi_e", f"Dense_{l}"), 2 * H + 1 if l == 0 else M, M)
        for l in range(L + 1):
            dense(blk + ("phi_h", f"Dense_{l}"), M + H if l == 0 else M, H if l == L else M)
        for l in range(L):
            dense(blk + ("phi_x_torso", f"Dense_{l}"), M, M)
        dense(("EGNN_0", f"Dense_{k}"), H + T, H)
    shapes[("EGNN_0", "final_scaling")] = ()
    shapes[("Embed_0", "embedding")] = (cfg.n_features, H)
    return [("/".join(p), shapes[p]) for p in sorted(shapes)]


def param_count(cfg: CNFConfig) -> int:
    return int(sum(int(np.prod(s)) for _, s in param_spec(cfg)))


def _flat_lookup(params: Mapping) -> Dict[str, np.ndarray]:
    """Accept {'EGNN_0/0/...': array} or a nested flax dict (optionally under a 'params' key)."""
    if "params" in params and isinstance(params["params"], Mapping):
        params = params["params"]
    out: Dict[str, np.ndarray] = {}

    def walk(d, prefix):
        for k, v in d.items():
            key = f"{prefix}/{k}" if prefix else str(k)
            if isinstance(v, Mapping):
                walk(v, key)
            else:
                out[key] = np.asarray(v)
    walk(params, "")
    return out


def _reference_shaped(flat: Mapping, cfg: CNFConfig) -> bool:
    """Whether `flat` holds the reference-shaped tree of a padded kernel config (every shape of ref_param_spec)."""
    if not cfg.ref_mlp_units:
        return False
    spec = ref_param_spec(cfg.n_features, cfg.ref_hidden, cfg.time_embedding_dim, cfg.ref_mlp_units, cfg.n_blocks)
    return all(path in flat and np.asarray(flat[path]).shape == shape for path, shape in spec)


def flatten_params(params: Mapping, cfg: CNFConfig) -> np.ndarray:
    """Flat fp32 blob in ravel_pytree order; raises ValueError on a missing key or a wrong shape.  For a padded
    kernel config (kernel_config), reference-shaped params are zero-padded first (pad_params)."""
    flat = _flat_lookup(params)
    if _reference_shaped(flat, cfg):
        flat = pad_params(flat, cfg.ref_hidden, cfg.time_embedding_dim, cfg.ref_mlp_units, cfg)
    chunks = []
    for path, shape in param_spec(cfg):
        if path not in flat:
            raise ValueError(f"missing parameter {path}")
        a = np.asarray(flat[path], np.float32)
        if a.shape != shape:
            raise ValueError(f"parameter {path} has shape {a.shape}, expected {shape}")
        chunks.append(a.reshape(-1))
    return np.ascontiguousarray(np.concatenate(chunks))


def unflatten_params(blob: np.ndarray, cfg: CNFConfig, reference_shapes: bool = False) -> Dict[str, np.ndarray]:
    """Flat blob -> flax-path dict of cfg's (kernel) shapes; reference_shapes=True crops a padded config's params back
    to the reference network's shapes (crop_params)."""
    if reference_shapes and cfg.ref_mlp_units:
        return crop_params(unflatten_params(blob, cfg), cfg)
    out, off = {}, 0
    for path, shape in param_spec(cfg):
        n = int(np.prod(shape))
        out[path] = np.asarray(blob[off:off + n], np.float32).reshape(shape)
        off += n
    if off != blob.size:
        raise ValueError(f"blob has {blob.size} floats, expected {off}")
    return out


def init_params(cfg: CNFConfig, seed: int = 0) -> Dict[str, np.ndarray]:
    """flax-default-like initialisation (cnf.init, build_cnf.py:97): lecun-normal kernels, zero biases,
    variance_scaling(0.001, fan_avg, uniform) for the phi_x output layer (egnn.py:83-85), final_scaling 1.
    numpy PCG64 stands in for JAX threefry (not bit-compatible)."""
    return init_from_spec(param_spec(cfg), seed)


def init_from_spec(spec: List[Tuple[str, Tuple[int, ...]]], seed: int = 0) -> Dict[str, np.ndarray]:
    """init_params over any (path, shape) tree (param_spec, or ref_param_spec for unequal widths)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    p: Dict[str, np.ndarray] = {}
    for path, shape in spec:
        parts = path.split("/")
        if parts[-1] == "bias":
            p[path] = np.zeros(shape, np.float32)
        elif parts[-1] == "final_scaling":
            p[path] = np.ones(shape, np.float32)
        elif parts[-1] == "embedding":
            p[path] = (rng.standard_normal(shape) / np.sqrt(shape[0])).astype(np.float32)
        elif len(parts) == 4 and parts[2] == "Dense_0":
            lim = np.sqrt(3.0 * 0.001 / ((shape[0] + shape[1]) / 2.0))
            p[path] = rng.uniform(-lim, lim, shape).astype(np.float32)
        else:
            z = rng.standard_normal(shape)
            while np.any(np.abs(z) > 2):
                bad = np.abs(z) > 2
                z[bad] = rng.standard_normal(int(bad.sum()))
            p[path] = (z / np.sqrt(shape[0]) / 0.87962566103423978).astype(np.float32)
    return p


# ---------------------------------------------------------------------------------------------------------------
# networks of any mlp_units / hidden width on the compiled kernel shapes (zero padding)
# ---------------------------------------------------------------------------------------------------------------
# (M, L, D) of the compiled kernels (ecnf_kernels.hpp ECNF_SHAPES / ECNF_SHAPES_WIDE_TAN)
COMPILED_SHAPES = {(128, 3, 3), (128, 3, 2), (128, 2, 3), (128, 2, 2), (64, 2, 3), (64, 2, 2), (64, 3, 3), (64, 3, 2),
                   (256, 4, 3), (256, 3, 3)}


def ref_param_spec(n_features: int, hidden: int, time_embedding_dim: int, mlp_units, n_blocks: int
                   ) -> List[Tuple[str, Tuple[int, ...]]]:
    """The reference's parameter tree for ANY mlp_units (egnn.py:43-47: phi_e = MLP(mlp_units), phi_x_torso =
    MLP(mlp_units) on m_ij of width mlp_units[-1], phi_h = MLP((*mlp_units, H)) on [m_i | h]; build_cnf.py:79,85)."""
    H, T, K, U = hidden, time_embedding_dim, n_blocks, tuple(int(u) for u in mlp_units)
    L = len(U)
    shapes: Dict[Tuple[str, ...], Tuple[int, ...]] = {}

    def dense(path, fan_in, fan_out):
        shapes[path + ("bias",)] = (fan_out,)
        shapes[path + ("kernel",)] = (fan_in, fan_out)

    hu = U + (H,)
    for k in range(K):
        blk = ("EGNN_0", str(k))
        dense(blk + ("Dense_0",), U[-1], 1)
        dense(blk + ("Dense_1",), U[-1], 1)
        for l in range(L):
            dense(blk + ("phi_e", f"Dense_{l}"), 2 * H + 1 if l == 0 else U[l - 1], U[l])
        for l in range(L + 1):
            dense(blk + ("phi_h", f"Dense_{l}"), U[-1] + H if l == 0 else hu[l - 1], hu[l])
        for l in range(L):
            dense(blk + ("phi_x_torso", f"Dense_{l}"), U[-1] if l == 0 else U[l - 1], U[l])
        dense(("EGNN_0", f"Dense_{k}"), H + T, H)
    shapes[("EGNN_0", "final_scaling")] = ()
    shapes[("Embed_0", "embedding")] = (n_features, H)
    return [("/".join(p), shapes[p]) for p in sorted(shapes)]


def kernel_config(n_nodes: int, dim: int, n_features: int, hidden: int, time_embedding_dim: int, mlp_units,
                  n_blocks: int, base_scale: float = 1.0, sigma_min: float = 0.01) -> CNFConfig:
    """The compiled kernel shape that runs a network of these widths: every MLP layer padded to the smallest compiled
    width M >= max(mlp_units) for its depth and dim, the node features to a multiple of 32.  Zero-padded units are
    inert: their pre-activations are exactly 0, SiLU(0) = 0, and every weight reading them is 0, so the padded network
    computes the same function (the extra terms add exact zeros)."""
    U = tuple(int(u) for u in mlp_units)
    if not U or min(U) < 1:
        raise ValueError("mlp_units must be a non-empty sequence of positive widths")
    L = len(U)
    fits = sorted(m for (m, l, d) in COMPILED_SHAPES if l == L and d == dim and m >= max(U))
    if not fits:
        raise ValueError(f"no compiled kernel for mlp_units={U} (depth {L}, width <= 256) at dim {dim}; compiled "
                         f"(M, L, D): {sorted(COMPILED_SHAPES)}")
    Hp = 32 * ((int(hidden) + 31) // 32)
    padded = U != (fits[0],) * L or Hp != int(hidden)
    return CNFConfig(n_nodes=n_nodes, dim=dim, n_features=n_features, hidden=Hp,
                     time_embedding_dim=time_embedding_dim, mlp_width=fits[0], mlp_depth=L, n_blocks=n_blocks,
                     base_scale=base_scale, sigma_min=sigma_min, ref_mlp_units=U if padded else (),
                     ref_hidden=int(hidden) if padded else 0)


def pad_params(params: Mapping, hidden: int, time_embedding_dim: int, mlp_units, kcfg: CNFConfig
               ) -> Dict[str, np.ndarray]:
    """Reference-shaped params (ref_param_spec) -> the zero-padded params of the kernel shape kcfg (kernel_config):
    every [in, out] matrix is placed into the padded one by the row / column maps of its concatenated inputs
    ([h_s | h_r | |r|^2] for phi_e.0, [m_i | h] for phi_h.0, [h | temb] for the node Dense)."""
    flat = _flat_lookup(params)
    H, T, U = int(hidden), int(time_embedding_dim), tuple(int(u) for u in mlp_units)
    Hp, Mp, L = kcfg.hidden, kcfg.mlp_width, len(U)
    hu, hup = U + (H,), (Mp,) * L + (Hp,)
    spec = dict(ref_param_spec(kcfg.n_features, H, T, U, kcfg.n_blocks))
    for path, shape in spec.items():
        if path not in flat:
            raise ValueError(f"missing parameter {path}")
        if np.asarray(flat[path]).shape != shape:
            raise ValueError(f"parameter {path} has shape {np.asarray(flat[path]).shape}, expected {shape}")
    out: Dict[str, np.ndarray] = {}

    def place(path, pshape, rows=None):
        """rows: list of (src_lo, src_hi, dst_lo) row segments of a kernel (None: rows 0..n -> 0..n)."""
        a = np.asarray(flat[path], np.float32)
        z = np.zeros(pshape, np.float32)
        if a.ndim == 1:
            z[: a.shape[0]] = a
        elif rows is None:
            z[: a.shape[0], : a.shape[1]] = a
        else:
            for s0, s1, d0 in rows:
                z[d0:d0 + s1 - s0, : a.shape[1]] = a[s0:s1]
        out[path] = z

    for k in range(kcfg.n_blocks):
        b = f"EGNN_0/{k}"
        for nm in ("Dense_0", "Dense_1"):
            place(f"{b}/{nm}/kernel", (Mp, 1))
            place(f"{b}/{nm}/bias", (1,))
        for l in range(L):
            if l == 0:
                place(f"{b}/phi_e/Dense_0/kernel", (2 * Hp + 1, Mp), [(0, H, 0), (H, 2 * H, Hp), (2 * H, 2 * H + 1, 2 * Hp)])
            else:
                place(f"{b}/phi_e/Dense_{l}/kernel", (Mp, Mp))
            place(f"{b}/phi_e/Dense_{l}/bias", (Mp,))
            place(f"{b}/phi_x_torso/Dense_{l}/kernel", (Mp, Mp))
            place(f"{b}/phi_x_torso/Dense_{l}/bias", (Mp,))
        for l in range(L + 1):
            if l == 0:
                place(f"{b}/phi_h/Dense_0/kernel", (Mp + Hp, Mp), [(0, U[-1], 0), (U[-1], U[-1] + H, Mp)])
            else:
                place(f"{b}/phi_h/Dense_{l}/kernel", (Mp, hup[l]))
            place(f"{b}/phi_h/Dense_{l}/bias", (hup[l],))
        place(f"EGNN_0/Dense_{k}/kernel", (Hp + T, Hp), [(0, H, 0), (H, H + T, Hp)])
        place(f"EGNN_0/Dense_{k}/bias", (Hp,))
    out["EGNN_0/final_scaling"] = np.asarray(flat["EGNN_0/final_scaling"], np.float32).reshape(())
    e = np.asarray(flat["Embed_0/embedding"], np.float32)
    out["Embed_0/embedding"] = np.zeros((kcfg.n_features, Hp), np.float32)
    out["Embed_0/embedding"][:, :H] = e
    del hu
    return out


def crop_params(params: Mapping, kcfg: CNFConfig) -> Dict[str, np.ndarray]:
    """The inverse of pad_params for a padded kernel config: the reference-shaped params (ref_param_spec) read out of
    the padded ones by the same row / column maps (the padded rows / columns are dropped)."""
    if not kcfg.ref_mlp_units:
        return dict(_flat_lookup(params))
    flat = _flat_lookup(params)
    H, T, U = kcfg.ref_hidden, kcfg.time_embedding_dim, kcfg.ref_mlp_units
    Hp, Mp, L = kcfg.hidden, kcfg.mlp_width, len(U)
    spec = dict(ref_param_spec(kcfg.n_features, H, T, U, kcfg.n_blocks))
    out: Dict[str, np.ndarray] = {}

    def take(path, rows=None):
        a = np.asarray(flat[path], np.float32)
        shape = spec[path]
        if a.ndim == 0:
            out[path] = a.reshape(())
        elif a.ndim == 1:
            out[path] = a[: shape[0]].copy()
        elif rows is None:
            out[path] = a[: shape[0], : shape[1]].copy()
        else:
            out[path] = np.concatenate([a[d0:d0 + s1 - s0, : shape[1]] for s0, s1, d0 in rows], axis=0)

    for k in range(kcfg.n_blocks):
        b = f"EGNN_0/{k}"
        for nm in ("Dense_0", "Dense_1"):
            take(f"{b}/{nm}/kernel")
            take(f"{b}/{nm}/bias")
        for l in range(L):
            if l == 0:
                take(f"{b}/phi_e/Dense_0/kernel", [(0, H, 0), (H, 2 * H, Hp), (2 * H, 2 * H + 1, 2 * Hp)])
            else:
                take(f"{b}/phi_e/Dense_{l}/kernel")
            take(f"{b}/phi_e/Dense_{l}/bias")
            take(f"{b}/phi_x_torso/Dense_{l}/kernel")
            take(f"{b}/phi_x_torso/Dense_{l}/bias")
        for l in range(L + 1):
            if l == 0:
                take(f"{b}/phi_h/Dense_0/kernel", [(0, U[-1], 0), (U[-1], U[-1] + H, Mp)])
            else:
                take(f"{b}/phi_h/Dense_{l}/kernel")
            take(f"{b}/phi_h/Dense_{l}/bias")
        take(f"EGNN_0/Dense_{k}/kernel", [(0, H, 0), (H, H + T, Hp)])
        take(f"EGNN_0/Dense_{k}/bias")
    take("EGNN_0/final_scaling")
    take("Embed_0/embedding")
    return out
