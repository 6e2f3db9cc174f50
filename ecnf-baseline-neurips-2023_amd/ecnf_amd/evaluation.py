"""The test-set evaluation leg on the HIP engine.

Mirrors (names, argument meaning):
  * ``setup_padded_reshaped_data``   ecnf/utils/evaluation.py:25-50 (zero padding to whole batches + a mask)
  * ``calculate_forward_ess``        ecnf/utils/evaluation.py:10-22
  * ``eval_test_set``                eval_fn (ecnf/utils/evaluation.py:59-115) driving eval_on_data_batch_fn
                                     (ecnf/setup_training.py:190-215): get_log_prob of every test molecule, the masked
                                     means test_log_lik / test_log_prob_base / test_delta_log_lik, and with a target
                                     the forward ESS of log_w = log p_target - log_q (setup_training.py:239-241)

The reference scans the padded batches one after the other (lax.scan, vmap inside a batch) and weights each batch's
masked means by its share of the real rows; that is the global masked mean, which is what is computed here.  On the
GPU the batches are not a memory constraint: each rank solves all of its whole batches in ONE ecnf_integrate launch
(molecules are independent and their results do not depend on their batch position), then the statistics are
reduced over torch.distributed (RCCL over xGMI on MI355X, gloo in the CPU tests):
  * one SUM all-reduce of [sum log_q, sum log p0, sum delta, count] (masked)      -> distributed.masked_mean
  * one MAX + one SUM all-reduce of the log-sum-exp partials of +-log_w            -> distributed.ess_from_device
Batches are dealt to ranks contiguously (whole batches), so the padded tail batch lives on the last rank.
"""
from __future__ import annotations

from typing import Callable, Dict, Optional

import torch

from . import _lib
from . import distributed as D
from .engine import EcnfHandle, SolveOptions


def setup_padded_reshaped_data(data: torch.Tensor, interval_length: int, reshape_axis: int = 0):
    """evaluation.py:25-50: pad the leading axis with zero rows to a multiple of ``interval_length`` and reshape to
    [interval_length, n/interval] (reshape_axis 0, the pmap layout) or [n/interval, interval_length] (1, the
    minibatch layout).  Returns (data, mask) with mask 1 on the real rows."""
    n = data.shape[0]
    pad = (interval_length - n % interval_length) % interval_length
    padded = torch.cat([data, torch.zeros((pad,) + tuple(data.shape[1:]), dtype=data.dtype, device=data.device)])
    mask = torch.zeros(n + pad, dtype=torch.int32, device=data.device)
    mask[:n] = 1
    m = (n + pad) // interval_length
    if reshape_axis == 0:
        shape = (interval_length, m)
    else:
        if reshape_axis != 1:
            raise ValueError("reshape_axis must be 0 or 1")
        shape = (m, interval_length)
    return padded.reshape(shape + tuple(data.shape[1:])), mask.reshape(shape)


def calculate_forward_ess(log_w: torch.Tensor, mask: torch.Tensor) -> Dict[str, torch.Tensor]:
    """evaluation.py:10-22 over every rank's entries (device log-sum-exp partials + one MAX and one SUM all-reduce)."""
    if log_w.shape != mask.shape:
        raise ValueError("log_w and mask must have the same shape (chex.assert_equal_shape)")
    fwd, _ = D.ess_from_device(log_w.reshape(-1).float().contiguous(), mask.reshape(-1).float().contiguous())
    return {"forward_ess": fwd}


def reduce_test_stats(log_q: torch.Tensor, log_prob_base: torch.Tensor, delta: torch.Tensor,
                      mask: Optional[torch.Tensor] = None) -> Dict[str, torch.Tensor]:
    """The masked means of eval_on_data_batch_fn (setup_training.py:206-209) over every rank's rows (fp64, one SUM
    all-reduce each)."""
    return {"test_log_lik": D.masked_mean(log_q, mask),
            "test_log_prob_base": D.masked_mean(log_prob_base, mask),
            "test_delta_log_lik": D.masked_mean(delta, mask)}


def eval_test_set(h: EcnfHandle, x, features, batch_size: int, approx: bool = False,
                  opts: Optional[SolveOptions] = None, eps: Optional[torch.Tensor] = None, seed: int = 0,
                  target_log_prob_fn: Optional[Callable[[torch.Tensor], torch.Tensor]] = None) -> Dict[str, float]:
    """eval_fn + eval_on_data_batch_fn on the whole test set ``x`` [n, N*D] (GLOBAL: every rank passes the same
    array; each solves its contiguous share of the padded batches).  approx=False: the exact trace
    (eval_exact_log_prob: true, lj13.yaml:33); approx=True: Hutchinson with ``eps`` [n, N*D] (GLOBAL rows), or one
    seeded global draw.  Returns floats: test_log_lik, test_log_prob_base, test_delta_log_lik and, with a target,
    forward_ess."""
    cfg = h.cfg
    x = torch.as_tensor(x, device=h.device, dtype=torch.float32).reshape(-1, cfg.event_dim)
    n = x.shape[0]
    if n == 0:
        raise ValueError("empty test set")
    feats = torch.as_tensor(features)
    if feats.dim() == 1:
        feats = feats.reshape(1, -1).expand(n, -1)
    feats = feats.to(h.device, torch.int32).reshape(n, cfg.n_nodes)
    xb, mask = setup_padded_reshaped_data(x, int(batch_size), reshape_axis=1)
    n_batches = xb.shape[0]
    rank, ws = D.world()
    blo, bhi = D.shard_bounds(n_batches, rank, ws)
    # this rank's rows: whole batches [blo, bhi); only the real rows among them are solved (padded rows are masked
    # out of every statistic, and a zero-coordinate row could only cost solver steps)
    lo, hi = min(blo * batch_size, n), min(bhi * batch_size, n)
    opts = opts or SolveOptions(solver="dopri5", step_size=None)
    div = _lib.DIV_HUTCHINSON if approx else _lib.DIV_EXACT
    e = None
    if approx:
        e = (torch.as_tensor(eps, device=h.device, dtype=torch.float32).reshape(n, cfg.event_dim)[lo:hi]
             if eps is not None else D.global_normal(n, cfg.event_dim, seed, lo, hi, h.device))
    if hi > lo:
        x0, dl, _, _ = h.integrate(x[lo:hi], feats[lo:hi], 1.0, 0.0, opts, divergence=div, eps=e)
        lp0 = h.base_log_prob(x0)
        log_q = lp0 + dl                                          # sample_and_log_prob.py:90-94
    else:
        dl = lp0 = log_q = torch.zeros(0, device=h.device)
    info = reduce_test_stats(log_q, lp0, dl)
    out = {k: float(v) for k, v in info.items()}
    if target_log_prob_fn is not None:
        log_w = (target_log_prob_fn(x[lo:hi]) - log_q) if hi > lo else torch.zeros(0, device=h.device)
        m = torch.ones_like(log_w)
        out["forward_ess"] = float(calculate_forward_ess(log_w, m)["forward_ess"])
    out["n_test"] = n
    out["n_batches"] = n_batches
    return out


def main(argv=None) -> None:
    """Command-line eval of a test set (one JSON line on rank 0); under torch.distributed.run each rank solves its
    share of the batches.  --data: an .npy of positions [n, N, D] or [n, N*D] (e.g. tests/golden/aldp_frames.npy,
    zero-CoM centred here as setup_training.py:91-94 does); weights: the seeded synthetic init of the config
    (params.init_params) unless --params names a flax-path .npz (dataio)."""
    import argparse
    import json
    import os
    import time

    import numpy as np
    import torch.distributed as dist

    from . import CONFIGS, dataio, init_params
    from . import targets as T
    ap = argparse.ArgumentParser(prog="python -m ecnf_amd.evaluation")
    ap.add_argument("--config", default="aldp")
    ap.add_argument("--data", required=True)
    ap.add_argument("--n", type=int, default=0, help="first n molecules of the data (0 = all)")
    ap.add_argument("--batch-size", type=int, default=64)
    ap.add_argument("--approx", action="store_true", help="Hutchinson instead of the exact trace")
    ap.add_argument("--step-size", type=float, default=0.0,
                    help="> 0: fixed steps of this size (the reference's use_fixed_step_size: Dopri5 with a constant "
                         "dt0, sample_and_log_prob.py:84-85), else Dopri5 + PID")
    ap.add_argument("--solver", choices=("dopri5", "euler"), default="dopri5",
                    help="fixed-step solver (euler: NFE = 1 / step size; not the reference's)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--params", default="", help="flax-path .npz (dataio.load_params_npz)")
    ap.add_argument("--dist-backend", default="nccl")
    args = ap.parse_args(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.dist_backend)
    cfg = CONFIGS[args.config]
    if args.params:
        params = dataio.load_params_npz(args.params, cfg)
    else:
        params = init_params(cfg, args.seed)
    x = np.load(args.data).astype(np.float32)
    if args.n:
        x = x[: args.n]
    x = x.reshape(x.shape[0], cfg.n_nodes, cfg.dim)
    x = (x - x.mean(axis=1, keepdims=True)).reshape(x.shape[0], -1)
    feats = (np.arange(cfg.n_nodes, dtype=np.int32) if args.config == "aldp"     # data.py:146
             else np.zeros(cfg.n_nodes, np.int32))
    h = EcnfHandle(cfg, params, local)
    if args.solver == "euler" and args.step_size <= 0:
        ap.error("--solver euler needs --step-size > 0")
    opts = (SolveOptions(args.solver, args.step_size) if args.step_size > 0 else SolveOptions("dopri5", None))
    target = None
    if args.config == "lj13":
        target = lambda y: T.lj_log_prob(y, cfg.n_nodes, cfg.dim)
    elif args.config == "dw4":
        target = lambda y: T.dw_log_prob(y, cfg.n_nodes, cfg.dim)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    info = eval_test_set(h, x, feats, args.batch_size, approx=args.approx, opts=opts, seed=args.seed,
                         target_log_prob_fn=target)
    torch.cuda.synchronize()
    info["seconds"] = time.perf_counter() - t0
    info["world"] = D.world()[1]
    if D.world()[0] == 0:
        print(json.dumps(info), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
