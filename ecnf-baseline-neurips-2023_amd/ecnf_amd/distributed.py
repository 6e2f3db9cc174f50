"""Multi-GPU sampling: one process per GPU, the batch sharded contiguously, eval statistics reduced over
torch.distributed (backend "nccl" = RCCL over xGMI on MI355X; "gloo" for the CPU tests).

The reference is single-device; its batch statistics are the only cross-sample math:
  * test log-likelihood: masked means of log_q, log p0, delta over the test batches
    (setup_training.py:206-209, numerical.py:43-52)                   -> :func:`masked_mean`
  * forward ESS: log-sum-exp of -log_w and log_w over the test set (evaluation.py:10-22) -> :func:`forward_ess`
  * reverse ESS: 1 / sum softmax(log_w)^2 / n (setup_training.py:182)  -> :func:`reverse_ess`
Each is one MAX and/or one SUM all-reduce of a few scalars — latency-bound, no data-path collective.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch
import torch.distributed as dist


def world() -> Tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def shard_bounds(n_total: int, rank: int, world_size: int) -> Tuple[int, int]:
    """Contiguous shard [lo, hi) of rank; shard sizes differ by at most one molecule."""
    base, rem = divmod(int(n_total), int(world_size))
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def global_normal(n_total: int, event_dim: int, seed: int, lo: int, hi: int, device) -> torch.Tensor:
    """Rows [lo, hi) of one seeded standard-normal draw of shape [n_total, event_dim]: the noise a molecule gets
    does not depend on the world size (results concatenate bit-identically across 1/2/4/8 GPUs, because the
    kernels' per-molecule results do not depend on batch position)."""
    g = torch.Generator(device=device)
    g.manual_seed(int(seed))
    z = torch.randn((int(n_total), int(event_dim)), generator=g, device=device, dtype=torch.float32)
    return z[lo:hi].contiguous()


def _allreduce(t: torch.Tensor, op) -> torch.Tensor:
    # every initialised group reduces, one rank included (an identity, but the RCCL path then runs on one GPU)
    if dist.is_available() and dist.is_initialized():
        if t.is_cuda and dist.get_backend() == "gloo":
            # gloo rehearsals (tests, several ranks folded onto one GPU): reduce a host copy
            h = t.cpu()
            dist.all_reduce(h, op=op)
            t.copy_(h)
        else:
            dist.all_reduce(t, op=op)
    return t


def logsumexp(values: torch.Tensor, weights: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Global log(sum_i w_i exp(v_i)) over every rank's local values (fp64): one MAX + one SUM all-reduce."""
    v = values.detach().to(torch.float64).reshape(-1)
    w = torch.ones_like(v) if weights is None else weights.detach().to(torch.float64).reshape(-1)
    valid = w > 0
    m_local = v[valid].max() if bool(valid.any()) else torch.tensor(-math.inf, dtype=torch.float64, device=v.device)
    m = _allreduce(m_local.reshape(1).clone(), dist.ReduceOp.MAX)
    m0 = torch.where(torch.isfinite(m), m, torch.zeros_like(m))
    s = _allreduce((w * torch.exp(v - m0)).sum().reshape(1), dist.ReduceOp.SUM)
    return (m0 + torch.log(s))[0]


def masked_mean(values: torch.Tensor, mask: Optional[torch.Tensor] = None) -> torch.Tensor:
    """numerical.py:43-52 over the global batch (0 when fully masked)."""
    v = values.detach().to(torch.float64).reshape(-1)
    m = torch.ones_like(v) if mask is None else mask.detach().to(torch.float64).reshape(-1)
    acc = _allreduce(torch.stack([(torch.where(m > 0, v, torch.zeros_like(v))).sum(), m.sum()]), dist.ReduceOp.SUM)
    return torch.where(acc[1] == 0, torch.zeros_like(acc[0]), acc[0] / torch.clamp(acc[1], min=1.0))


def combine_partials(p: torch.Tensor) -> torch.Tensor:
    """Global [LSE(v), LSE(-v), LSE(2v), count] (fp64) from every rank's float[7] log-sum-exp partials
    (targets.lse_partials / ecnf_lse_partials): one MAX all-reduce of the three maxima, then one SUM all-reduce of
    the rescaled sums and the count."""
    p = p.detach().to(torch.float64).reshape(7)
    m_local = p[[0, 2, 4]]
    m = _allreduce(m_local.clone(), dist.ReduceOp.MAX)
    finite = torch.isfinite(m)
    m0 = torch.where(finite, m, torch.zeros_like(m))
    # a rank whose maximum is the global one contributes its sum as is (this also keeps +inf maxima, whose sums
    # count the +inf entries, free of exp(inf - inf)); empty ranks (-inf) contribute nothing
    scale = torch.where(m_local == m, torch.ones_like(m_local),
                        torch.where(torch.isfinite(m_local), torch.exp(m_local - m0), torch.zeros_like(m_local)))
    s = _allreduce(torch.cat([p[[1, 3, 5]] * scale, p[6:7]]), dist.ReduceOp.SUM)
    # jax.nn.logsumexp: a +inf maximum gives +inf, no entries (-inf) gives -inf, NaN stays NaN
    return torch.cat([torch.where(finite, m0 + torch.log(s[:3]), m), s[3:]])


def ess_from_device(log_w: torch.Tensor, mask: Optional[torch.Tensor] = None):
    """(forward ESS, reverse ESS) of the global log_w from the HIP log-sum-exp partials of each rank's shard
    (ecnf_lse_partials) and two scalar all-reduces.  Forward ESS follows evaluation.py:10-22 (masked);
    reverse ESS setup_training.py:182 (over the unmasked entries)."""
    from .targets import lse_partials
    g = combine_partials(lse_partials(log_w, mask))
    lse, lse_neg, lse_2, n = g[0], g[1], g[2], g[3]
    fwd = torch.exp(-(lse_neg - torch.log(n)) - (lse - torch.log(n)))
    rev = torch.exp(2 * lse - lse_2) / n
    return fwd, rev


def forward_ess(log_w: torch.Tensor, mask: Optional[torch.Tensor] = None) -> torch.Tensor:
    """evaluation.py:10-22: exp(-(LSE(-log_w) - log n) - (LSE(log_w) - log n))."""
    lw = log_w.detach().to(torch.float64).reshape(-1)
    m = torch.ones_like(lw) if mask is None else mask.detach().to(torch.float64).reshape(-1)
    lw = torch.where(m > 0, lw, torch.zeros_like(lw))
    n = _allreduce(m.sum().reshape(1), dist.ReduceOp.SUM)[0]
    log_z_inv = logsumexp(-lw, m) - torch.log(n)
    log_z_exp = logsumexp(lw, m) - torch.log(n)
    return torch.exp(-log_z_inv - log_z_exp)


def reverse_ess(log_w: torch.Tensor) -> torch.Tensor:
    """setup_training.py:182: 1 / sum(softmax(log_w)^2) / n = exp(2 LSE(log_w) - LSE(2 log_w)) / n."""
    lw = log_w.detach().to(torch.float64).reshape(-1)
    n = _allreduce(torch.tensor([float(lw.numel())], dtype=torch.float64, device=lw.device), dist.ReduceOp.SUM)[0]
    return torch.exp(2 * logsumexp(lw) - logsumexp(2 * lw)) / n


def all_gather_rows(x: torch.Tensor) -> torch.Tensor:
    """Concatenate every rank's [n_r, ...] rows in rank order (shards may differ by one row)."""
    rank, ws = world()
    if ws == 1:
        return x
    n = torch.tensor([x.shape[0]], device=x.device, dtype=torch.int64)
    sizes = [torch.zeros_like(n) for _ in range(ws)]
    dist.all_gather(sizes, n)
    nmax = int(max(int(s) for s in sizes))
    pad = torch.zeros((nmax,) + tuple(x.shape[1:]), device=x.device, dtype=x.dtype)
    pad[: x.shape[0]] = x
    bufs = [torch.empty_like(pad) for _ in range(ws)]
    dist.all_gather(bufs, pad)
    return torch.cat([b[: int(s)] for b, s in zip(bufs, sizes)], dim=0)
