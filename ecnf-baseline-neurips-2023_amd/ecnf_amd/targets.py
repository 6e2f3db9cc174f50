"""Target densities and eval reductions on the device.

  * :func:`lj_log_prob` / :func:`dw_log_prob`  <- log_prob_fn = -energy of ecnf/targets/target_energy/
    leonard_jones.py:10-35 and double_well.py:9-28 (ecnf_target_log_prob, one thread per molecule)
  * :func:`lse_partials`  <- the log-sum-exp reductions of evaluation.py:10-22 and setup_training.py:182
    (ecnf_lse_partials, one workgroup); ecnf_amd.distributed combines the partials across ranks
  * :func:`log_weights`   <- log_w = log p_target(x) - log q(x) (evaluation.py:59-115 usage)

Every function takes device tensors and runs on libecnf_hip.so; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import numpy as np
import torch

from . import _lib


def _target(kind: int, n_nodes: int, dim: int, **kw) -> _lib.EcnfTarget:
    t = _lib.EcnfTarget()
    t.kind, t.n_nodes, t.dim = kind, int(n_nodes), int(dim)
    t.epsilon = float(kw.get("epsilon", 1.0))
    t.tau = float(kw.get("tau", 1.0))
    t.r = float(kw.get("r", 1.0))
    t.harmonic_coef = float(kw.get("harmonic_potential_coef", 0.5))
    t.a, t.b, t.c, t.d0 = float(kw.get("a", 0.0)), float(kw.get("b", -4.0)), float(kw.get("c", 0.9)), float(kw.get("d0", 4.0))
    return t


def _flat(x: torch.Tensor, n_nodes: int, dim: int) -> torch.Tensor:
    if not (torch.is_tensor(x) and x.is_cuda):
        raise ValueError("x must be a device (cuda) tensor")
    x = x.reshape(-1, n_nodes * dim)
    return x.float().contiguous() if x.dtype != torch.float32 else x.contiguous()


def _log_prob(t: _lib.EcnfTarget, x: torch.Tensor, r_nodes: Optional[torch.Tensor] = None) -> torch.Tensor:
    lib = _lib.load()
    xf = _flat(x, t.n_nodes, t.dim)
    if r_nodes is not None:
        r_nodes = torch.as_tensor(r_nodes, device=xf.device, dtype=torch.float32).reshape(-1).contiguous()
        if r_nodes.numel() != t.n_nodes:
            raise ValueError(f"r must be a scalar or have n_nodes = {t.n_nodes} entries")
        t.r_nodes = r_nodes.data_ptr()
    out = torch.empty(xf.shape[0], device=xf.device, dtype=torch.float32)
    stream = torch.cuda.current_stream(xf.device).cuda_stream
    _lib.check(lib.ecnf_target_log_prob(ctypes.byref(t), xf.data_ptr(), out.data_ptr(), xf.shape[0], stream))
    return out


def lj_log_prob(x: torch.Tensor, n_nodes: int = 13, dim: int = 3, epsilon: float = 1.0, tau: float = 1.0,
                r=1.0, harmonic_potential_coef: float = 0.5) -> torch.Tensor:
    """leonard_jones.log_prob_fn: -energy(x) for x [..., n_nodes*dim] or [..., n_nodes, dim]; r is a float or a
    per-node array [n_nodes] (leonard_jones.py:10-20: pair (receiver i, sender j) uses r[i])."""
    # a Python / numpy scalar or a 0-d array / tensor is the scalar r; anything with n_nodes entries is per node
    scalar = (torch.as_tensor(r).dim() == 0) if torch.is_tensor(r) else np.ndim(r) == 0
    t = _target(_lib.TARGET_LJ, n_nodes, dim, epsilon=epsilon, tau=tau, r=float(r) if scalar else 1.0,
                harmonic_potential_coef=harmonic_potential_coef)
    return _log_prob(t, x, None if scalar else r)


def dw_log_prob(x: torch.Tensor, n_nodes: int = 4, dim: int = 2, temperature: float = 1.0, a: float = 0.0,
                b: float = -4.0, c: float = 0.9, d0: float = 4.0) -> torch.Tensor:
    """double_well.log_prob_fn(x, temperature): -energy(x, tau=temperature)."""
    return _log_prob(_target(_lib.TARGET_DW, n_nodes, dim, tau=temperature, a=a, b=b, c=c, d0=d0), x)


def log_weights(log_p_target: torch.Tensor, log_q: torch.Tensor) -> torch.Tensor:
    """Importance log-weights log_w = log p(x) - log q(x) of flow samples."""
    return log_p_target - log_q


def lse_partials(v: torch.Tensor, mask: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Device float[7]: (max, sum exp(s v - max)) for s = +1, -1, +2, then the count of unmasked entries."""
    if not (torch.is_tensor(v) and v.is_cuda):
        raise ValueError("v must be a device (cuda) tensor")
    lib = _lib.load()
    vf = v.reshape(-1).float().contiguous()
    mf = None if mask is None else mask.reshape(-1).to(device=vf.device, dtype=torch.float32).contiguous()
    if mf is not None and mf.numel() != vf.numel():
        raise ValueError("mask must match v")
    out = torch.empty(7, device=vf.device, dtype=torch.float32)
    stream = torch.cuda.current_stream(vf.device).cuda_stream
    _lib.check(lib.ecnf_lse_partials(vf.data_ptr(), None if mf is None else mf.data_ptr(), vf.numel(), out.data_ptr(),
                                     stream))
    return out
