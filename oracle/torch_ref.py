"""torch restatement of the EGNN vector field and the fixed-step sampler, batched like XLA's vmap.

TEST INFRASTRUCTURE ONLY (see ecnf_oracle.py's header for the rules): ``bench.py``'s ``cpu_baseline`` leg times it
on the host cores as the reported CPU baseline ("torch-CPU fp32 batched restatement of the
identical math"), and ``tests/`` use it as the reverse-mode checker of the training path (torch autograd, itself
checked against finite differences of the fp64 numpy oracle).  Never imported by ``ecnf_amd``.

Follows the same reference lines as the numpy oracle:
  * ``ecnf/cnf/build_cnf.py:18-32,68-93``  time embedding, FlatEgnn       -> :func:`vector_field`
  * ``ecnf/nets/egnn.py:49-114,144-190``   EGCL, EGNN.call_single         -> :func:`_egcl`, :func:`vector_field`
  * ``ecnf/nets/mlp.py:7-19``              MLP                            -> :func:`_mlp`
  * ``ecnf/utils/graph.py:6-14``           receiver-major edges           -> :func:`edges`
  * ``ecnf/utils/numerical.py:7-10``       safe_norm                      -> inside :func:`_egcl`
  * ``ecnf/cnf/core.py:35-39``, ``ecnf/cnf/loss.py:10-32``  flow-matching loss -> :func:`fm_loss`
  * ``ecnf/cnf/sample_and_log_prob.py:28-33`` with a ConstantStepSize Euler solver -> :func:`sample_euler`
"""
from __future__ import annotations

import math
from typing import Dict, Mapping

import numpy as np
import torch


def edges(n: int):
    """graph.py:6-14: receivers = i repeated N-1 times, senders = (i+1+j) mod N."""
    recv = torch.arange(n).repeat_interleave(n - 1)
    send = torch.tensor([(i + 1 + j) % n for i in range(n) for j in range(n - 1)], dtype=torch.long)
    return send, recv


def to_torch(params: Mapping, dtype=torch.float32, requires_grad: bool = False) -> Dict[str, torch.Tensor]:
    out = {}
    for k, v in params.items():
        t = torch.as_tensor(np.asarray(v), dtype=dtype).clone()
        out[k] = t.requires_grad_(requires_grad)
    return out


def time_embedding(t: torch.Tensor, dim: int) -> torch.Tensor:
    """build_cnf.py:18-32 (1000 t, ln(1e4) / (dim/2 - 1)); frequencies in fp32 like the reference."""
    half = dim // 2
    ex = np.float32(np.log(10000.0) / (half - 1))
    freqs = torch.as_tensor(np.exp(np.arange(half, dtype=np.float32) * -ex), dtype=torch.float32)
    arg = (t.float() * 1000.0)[:, None] * freqs[None]
    return torch.cat([torch.sin(arg), torch.cos(arg)], dim=-1).to(t.dtype)


def _dense(x, P, prefix):
    return x @ P[prefix + "/kernel"] + P[prefix + "/bias"]


def _mlp(x, P, prefix, n_layers, activate_final):
    for l in range(n_layers):
        x = _dense(x, P, f"{prefix}/Dense_{l}")
        if l < n_layers - 1 or activate_final:
            x = torch.nn.functional.silu(x)
    return x


def _egcl(cfg, P, blk, vec, h, send, recv):
    """egnn.py:49-114 on [B, N, ...]."""
    N, L = cfg.n_nodes, cfg.mlp_depth
    nn1 = N - 1
    r = vec[:, recv] - vec[:, send]                                        # egnn.py:73
    x2 = (r * r).sum(-1, keepdim=True)
    length = torch.sqrt(torch.where(x2 == 0, torch.ones_like(x2), x2))    # numerical.py:7-10
    e_in = torch.cat([h[:, send], h[:, recv], length * length], dim=-1)   # egnn.py:76
    m = _mlp(e_in, P, f"{blk}/phi_e", L, True)                             # egnn.py:79
    px = _dense(_mlp(m, P, f"{blk}/phi_x_torso", L, True), P, f"{blk}/Dense_0")   # egnn.py:82-85
    shifts = px * r / (cfg.normalization_constant + length)                # egnn.py:87-91
    B = vec.shape[0]
    vec = vec + shifts.reshape(B, N, nn1, -1).sum(2) / nn1                 # egnn.py:92-95,113
    g = torch.sigmoid(_dense(m, P, f"{blk}/Dense_1"))                      # egnn.py:99-101
    m_i = (m * g).reshape(B, N, nn1, -1).sum(2) / math.sqrt(nn1)           # egnn.py:102-104
    h = _mlp(torch.cat([m_i, h], dim=-1), P, f"{blk}/phi_h", L + 1, False) + h   # egnn.py:105-111
    return vec, h


def vector_field(P: Mapping[str, torch.Tensor], cfg, x: torch.Tensor, t: torch.Tensor,
                 feat: torch.Tensor) -> torch.Tensor:
    """FlatEgnn.__call__ (build_cnf.py:68-93) + EGNN.call_single (egnn.py:144-190) for x [B, N*D]."""
    N, D, K = cfg.n_nodes, cfg.dim, cfg.n_blocks
    B = x.shape[0]
    send, recv = edges(N)
    pos = x.reshape(B, N, D)
    h = P["Embed_0/embedding"][feat.long()]                                 # build_cnf.py:79-80
    temb = time_embedding(t, cfg.time_embedding_dim).to(x.dtype)
    mean = pos.mean(1, keepdim=True)                                        # egnn.py:160
    vec = pos - mean
    vec0 = vec
    for k in range(K):                                                      # egnn.py:165-178
        h = _dense(torch.cat([h, temb[:, None].expand(B, N, -1)], dim=-1), P, f"EGNN_0/Dense_{k}")
        vec, h = _egcl(cfg, P, f"EGNN_0/{k}", vec, h, send, recv)
    return (((vec - vec0) - mean) * P["EGNN_0/final_scaling"]).reshape(B, N * D)   # egnn.py:183-188


def sample_euler(P, cfg, x0: torch.Tensor, feat: torch.Tensor, n_steps: int) -> torch.Tensor:
    """ODE 0 -> 1 with ConstantStepSize Euler (t accumulated in fp32 and clipped to 1 within 1e-6)."""
    x = x0.clone()
    dt = np.float32(1.0 / n_steps)
    tau = np.float32(0.0)
    with torch.no_grad():
        while tau < 1.0:
            tn = np.float32(tau + dt)
            tn = np.float32(1.0) if tn > np.float32(1.0) - np.float32(1e-6) else tn
            v = vector_field(P, cfg, x, torch.full((x.shape[0],), float(tau), dtype=x.dtype), feat)
            x = x + float(np.float32(tn - tau)) * v
            tau = tn
    return x


def fm_loss(P, cfg, x_data: torch.Tensor, x0: torch.Tensor, t: torch.Tensor, feat: torch.Tensor) -> torch.Tensor:
    """loss.py:10-32 with the noise given: x_t, u_t from the OT conditional path (core.py:35-39), then
    mean((v(x_t, t) - u_t)^2) over batch and coordinates."""
    s = cfg.sigma_min
    tt = t[:, None]
    x_t = (1 - (1 - s) * tt) * x0 + tt * x_data
    u_t = x_data - (1 - s) * x0
    v = vector_field(P, cfg, x_t, t, feat)
    return ((v - u_t) ** 2).mean()
