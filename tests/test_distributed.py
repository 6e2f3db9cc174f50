"""Multi-process (gloo, world size 2, CPU) tests of the sharding and the eval-statistic reductions that run over
RCCL on the GPU node: sharded results must equal the single-process (oracle) statistics."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ecnf_amd import distributed as D
from oracle import ecnf_oracle as O


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _np_partials(v, mask=None):
    """The float[7] output contract of ecnf_lse_partials (include/ecnf.h), restated in numpy for host-side tests of
    the cross-rank combine: (max s v, sum exp(s v - max)) for s = +1, -1, +2 over unmasked entries, then count."""
    v = np.asarray(v, np.float64)
    if mask is not None:
        v = v[np.asarray(mask) > 0]
    out = []
    for s in (1.0, -1.0, 2.0):
        if v.size:
            m = (s * v).max()
            out += [m, np.exp(s * v - m).sum()]
        else:
            out += [-np.inf, 0.0]
    return torch.tensor(out + [float(v.size)], dtype=torch.float32)


def _ess_from_partials(p):
    g = D.combine_partials(p)
    lse, lse_neg, lse_2, n = (float(x) for x in g)
    return np.exp(-(lse_neg - np.log(n)) - (lse - np.log(n))), np.exp(2 * lse - lse_2) / n


def _worker(rank, world, port, log_w, mask, q, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, hi = D.shard_bounds(len(log_w), rank, world)
        lw = torch.from_numpy(log_w[lo:hi])
        mk = torch.from_numpy(mask[lo:hi])
        res = {
            "fess": float(D.forward_ess(lw, mk)),
            "ress": float(D.reverse_ess(lw)),
            "mean": float(D.masked_mean(torch.from_numpy(q[lo:hi]), mk)),
            "lse": float(D.logsumexp(lw)),
            "gathered": D.all_gather_rows(torch.from_numpy(q[lo:hi]).reshape(-1, 1)).numpy().ravel(),
            "z": D.global_normal(9, 3, 7, *D.shard_bounds(9, rank, world), device="cpu").numpy(),
            "ess_partials": _ess_from_partials(_np_partials(log_w[lo:hi], mask[lo:hi])),
            "ress_partials": _ess_from_partials(_np_partials(log_w[lo:hi]))[1],
        }
        out_q.put((rank, res))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gloo_reductions_match_single_process(world):
    rng = np.random.default_rng(0)
    n = 37                                           # ragged: shards of 19 and 18
    log_w = rng.standard_normal(n) * 3.0
    mask = (rng.random(n) > 0.2).astype(np.float64)
    q = rng.standard_normal(n)
    ctx = mp.get_context("spawn")
    out_q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, log_w, mask, q, out_q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(out_q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        res = results[r]
        assert abs(res["fess"] - O.forward_ess(log_w, mask)) < 1e-10
        assert abs(res["ress"] - O.reverse_ess(log_w)) < 1e-10
        assert abs(res["mean"] - (q * mask).sum() / mask.sum()) < 1e-12
        m = log_w.max()
        assert abs(res["lse"] - (m + np.log(np.exp(log_w - m).sum()))) < 1e-10
        np.testing.assert_array_equal(res["gathered"], q)
        # the device-partials path (fp32 partials, as ecnf_lse_partials returns them)
        assert abs(res["ess_partials"][0] - O.forward_ess(log_w, mask)) < 1e-5
        assert abs(res["ress_partials"] - O.reverse_ess(log_w)) < 1e-5
    z_full = D.global_normal(9, 3, 7, 0, 9, device="cpu").numpy()
    np.testing.assert_array_equal(np.concatenate([results[r]["z"] for r in range(world)]), z_full)


def test_shard_bounds_cover():
    for n in (0, 1, 7, 1024, 65536):
        for w in (1, 2, 3, 8):
            bounds = [D.shard_bounds(n, r, w) for r in range(w)]
            assert bounds[0][0] == 0 and bounds[-1][1] == n
            assert all(bounds[i][1] == bounds[i + 1][0] for i in range(w - 1))
            sizes = [b - a for a, b in bounds]
            assert max(sizes) - min(sizes) <= 1


def test_single_process_reductions_without_init():
    lw = torch.tensor([0.0, -1.0, 2.0], dtype=torch.float64)
    assert abs(float(D.reverse_ess(lw)) - O.reverse_ess(lw.numpy())) < 1e-12
    assert abs(float(D.forward_ess(lw)) - O.forward_ess(lw.numpy())) < 1e-12
    assert float(D.masked_mean(lw, torch.zeros(3))) == 0.0


def test_combine_partials_single_process_and_empty_shard():
    rng = np.random.default_rng(3)
    lw = rng.standard_normal(50) * 4.0
    fwd, rev = _ess_from_partials(_np_partials(lw))
    assert abs(fwd - O.forward_ess(lw)) < 1e-5 and abs(rev - O.reverse_ess(lw)) < 1e-5
    # an empty shard contributes (-inf, 0) partials and must not poison the combine
    g = D.combine_partials(_np_partials(np.zeros(0)))
    assert float(g[3]) == 0.0
