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


def flatten_params(params: Mapping, cfg: CNFConfig) -> np.ndarray:
    """Flat fp32 blob in ravel_pytree order; raises ValueError on a missing key or a wrong shape."""
    flat = _flat_lookup(params)
    chunks = []
    for path, shape in param_spec(cfg):
        if path not in flat:
            raise ValueError(f"missing parameter {path}")
        a = np.asarray(flat[path], np.float32)
        if a.shape != shape:
            raise ValueError(f"parameter {path} has shape {a.shape}, expected {shape}")
        chunks.append(a.reshape(-1))
    return np.ascontiguousarray(np.concatenate(chunks))


def unflatten_params(blob: np.ndarray, cfg: CNFConfig) -> Dict[str, np.ndarray]:
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
    rng = np.random.Generator(np.random.PCG64(seed))
    p: Dict[str, np.ndarray] = {}
    for path, shape in param_spec(cfg):
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
