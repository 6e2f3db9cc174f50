"""CPU tests of the test-set evaluation leg's host logic (ecnf_amd.evaluation; evaluation.py:10-115,
setup_training.py:190-215): the padded / reshaped batching against the oracle's restatement, and the statistics of
whole batches sharded over a gloo world of 2 against the oracle's per-batch-weighted eval_fn (no GPU here; the device
path is tests/test_gpu_evaluation.py)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ecnf_amd import distributed as D
from ecnf_amd import evaluation as EV
from oracle import ecnf_oracle as O


@pytest.mark.parametrize("n,bs", [(37, 16), (32, 16), (5, 16), (1, 1), (64, 7)])
@pytest.mark.parametrize("axis", [0, 1])
def test_padded_reshaped_data_matches_oracle(n, bs, axis):
    x = np.random.default_rng(n).standard_normal((n, 6)).astype(np.float32)
    got, gm = EV.setup_padded_reshaped_data(torch.from_numpy(x), bs, reshape_axis=axis)
    ref, rm = O.setup_padded_reshaped_data(x, bs, reshape_axis=axis)
    assert got.shape == ref.shape and gm.shape == rm.shape
    np.testing.assert_array_equal(got.numpy(), ref)
    np.testing.assert_array_equal(gm.numpy(), rm)
    assert int(gm.sum()) == n


def test_masked_mean_matches_reference_definition():
    a = np.array([1.0, 2.0, 5.0, 7.0])
    m = np.array([1, 0, 1, 0])
    assert O.maybe_masked_mean(a, m) == 3.0
    assert O.maybe_masked_mean(a, np.zeros(4)) == 0.0          # fully masked: 0, not NaN (numerical.py:50-51)
    assert float(D.masked_mean(torch.tensor(a), torch.tensor(m))) == 3.0
    assert float(D.masked_mean(torch.tensor(a), torch.zeros(4))) == 0.0


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, lq, lp0, dl, lw, bs, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = len(lq)
        nb = (n + bs - 1) // bs
        blo, bhi = D.shard_bounds(nb, rank, world)           # whole batches per rank, as eval_test_set deals them
        lo, hi = min(blo * bs, n), min(bhi * bs, n)
        st = EV.reduce_test_stats(torch.from_numpy(lq[lo:hi]), torch.from_numpy(lp0[lo:hi]), torch.from_numpy(dl[lo:hi]))
        fwd = D.forward_ess(torch.from_numpy(lw[lo:hi]))
        out_q.put((rank, {k: float(v) for k, v in st.items()}, float(fwd), hi - lo))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n,bs", [(37, 8), (40, 8), (9, 16)])
def test_sharded_test_stats_match_oracle_eval_fn(n, bs):
    """eval_fn's per-batch weighting (evaluation.py:92-97) of masked batch means == the global masked mean the
    sharded leg computes; forward ESS over the flattened log_w with the padding masked (setup_training.py:239-241)."""
    rng = np.random.default_rng(n)
    lq = rng.normal(-50, 5, n)
    lp0 = rng.normal(-40, 3, n)
    dl = lq - lp0
    lw = rng.normal(0, 2, n)
    # the oracle's eval_fn aggregation over the padded batches
    _, mask = O.setup_padded_reshaped_data(np.zeros((n, 1)), bs, reshape_axis=1)
    pad = mask.size - n
    full = lambda a: np.concatenate([a, np.zeros(pad)]).reshape(mask.shape)
    w = mask.sum(-1) / mask.sum()
    ref = {k: float(sum(w[b] * O.maybe_masked_mean(full(a)[b], mask[b]) for b in range(len(w))))
           for k, a in (("test_log_lik", lq), ("test_log_prob_base", lp0), ("test_delta_log_lik", dl))}
    ref_fwd = O.forward_ess(full(lw).reshape(-1), mask.reshape(-1))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, lq, lp0, dl, lw, bs, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sum(r[3] for r in res) == n
    for _, st, fwd, _ in res:
        for k, v in ref.items():
            assert abs(st[k] - v) <= 1e-12 * max(1.0, abs(v)), (k, st[k], v)
        assert abs(fwd - ref_fwd) <= 1e-12 * ref_fwd, (fwd, ref_fwd)
