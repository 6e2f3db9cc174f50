"""The test-set evaluation leg on the GPU (ecnf_amd.evaluation) against the oracle's
eval_fn restatement (oracle.eval_test_set: evaluation.py:10-115, setup_training.py:190-215):

  * ALDP, 37 real frames of the reference's aldp_500K_train_mini.h5 in padded batches of 16 (the last batch ragged),
    get_log_prob with Hutchinson, fixed-step Euler: test_log_lik / test_log_prob_base / test_delta_log_lik
    fp32-class (tests/tolerance.py) against the fp64 / fp32 oracle
  * LJ13, 21 molecules in batches of 8, the exact trace (eval_exact_log_prob: true, lj13.yaml:33): the same
    statistics plus the forward ESS of log_w = log p_target - log_q (relative 1e-4: the ESS is a ratio of log-sum-exps
    of log_w values the log-density bound already holds).  The target is a smooth stand-in (the base density): the
    LJ energy of random inputs spreads log_w over hundreds of nats and the ESS underflows to exactly 0 in fp64
  * the same ALDP eval over 2 ranks (torch.distributed.run, gloo, both ranks on this GPU): equal to 1 rank
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from oracle import ecnf_oracle as O
from tolerance import fp32_class

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs a ROCm GPU", allow_module_level=True)

from ecnf_amd import CONFIGS, dataio  # noqa: E402
from ecnf_amd import evaluation as EV  # noqa: E402
from ecnf_amd.engine import EcnfHandle, SolveOptions  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
FRAMES = os.path.join(HERE, "golden", "aldp_frames.npy")


def _params(name):
    oc = O.CONFIGS[name]
    return O.stress_params(O.init_params(oc, 0), oc)


def _aldp(n):
    f = np.load(FRAMES).astype(np.float32)[:n]
    return (f - f.mean(axis=1, keepdims=True)).reshape(n, -1)


def _check_stats(name, got, r64, r32):
    for k in ("test_log_lik", "test_log_prob_base", "test_delta_log_lik"):
        fp32_class(f"{name} {k}", np.array([got[k]]), np.array([r64[k]]), np.array([r32[k]]))


def test_aldp_test_set_hutchinson():
    cfg, oc = CONFIGS["aldp"], O.CONFIGS["aldp"]
    p = _params("aldp")
    x = _aldp(37)
    feat = np.arange(22, dtype=np.int32)
    eps = np.random.default_rng(11).standard_normal(x.shape).astype(np.float32)
    h = EcnfHandle(cfg, p, 0)
    got = EV.eval_test_set(h, x, feat, 16, approx=True, opts=SolveOptions("euler", 0.1), eps=eps)
    assert got["n_batches"] == 3
    ftile = np.tile(feat, (37, 1))
    r64 = O.eval_test_set(p, oc, x, ftile, 16, eps=eps, approx=True, solver="euler", dt0=0.1, dtype=np.float64)
    r32 = O.eval_test_set(p, oc, x, ftile, 16, eps=eps, approx=True, solver="euler", dt0=0.1, dtype=np.float32)
    _check_stats("aldp", got, r64, r32)


def test_lj13_test_set_exact_forward_ess():
    cfg, oc = CONFIGS["lj13"], O.CONFIGS["lj13"]
    p = _params("lj13")
    rng = np.random.default_rng(5)
    x = (1.4 * O.base_sample(rng.standard_normal((21, cfg.event_dim)).astype(np.float32), oc)).astype(np.float32)
    feat = np.zeros(13, np.int32)
    h = EcnfHandle(cfg, p, 0)
    target = lambda y: h.base_log_prob(y)
    got = EV.eval_test_set(h, x, feat, 8, approx=False, opts=SolveOptions("euler", 0.25), target_log_prob_fn=target)
    ftile = np.zeros((21, 13), np.int32)
    tgt = lambda y: O.base_log_prob(y, oc)
    r64 = O.eval_test_set(p, oc, x, ftile, 8, solver="euler", dt0=0.25, dtype=np.float64, target_log_prob=tgt)
    r32 = O.eval_test_set(p, oc, x, ftile, 8, solver="euler", dt0=0.25, dtype=np.float32, target_log_prob=tgt)
    _check_stats("lj13", got, r64, r32)
    print(f"forward ESS: hip {got['forward_ess']:.6g}, oracle fp64 {r64['forward_ess']:.6g}")
    assert 1e-4 < r64["forward_ess"] < 1.0
    assert abs(got["forward_ess"] - r64["forward_ess"]) <= 1e-4 * r64["forward_ess"]


@pytest.mark.timeout(300)
def test_aldp_test_set_two_ranks_equal_one(tmp_path):
    npz = tmp_path / "aldp.npz"
    dataio.save_params_npz(npz, _params("aldp"), CONFIGS["aldp"])
    frames = tmp_path / "frames.npy"
    np.save(frames, np.load(FRAMES)[:45])
    args = ["--config", "aldp", "--data", str(frames), "--batch-size", "8", "--approx", "--step-size", "0.125",
            "--params", str(npz), "--dist-backend", "gloo"]
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["PYTHONPATH"] = os.pathsep.join([os.path.join(ROOT, "ecnf-baseline-neurips-2023_amd"),
                                         env.get("PYTHONPATH", "")])

    def run(n):
        import socket
        with socket.socket() as so:
            so.bind(("127.0.0.1", 0))
            port = so.getsockname()[1]
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
               "--master-addr=127.0.0.1", f"--master-port={port}", "-m", "ecnf_amd.evaluation", *args]
        out = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
        assert out.returncode == 0, out.stderr[-3000:]
        lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
        assert len(lines) == 1, out.stdout
        return json.loads(lines[0])

    one, two = run(1), run(2)
    assert one["world"] == 1 and two["world"] == 2 and one["n_batches"] == 6
    for k in ("test_log_lik", "test_log_prob_base", "test_delta_log_lik"):
        # the same molecules with the same seeded noise; only the fp64 summation order of the all-reduce differs
        assert abs(one[k] - two[k]) <= 1e-12 * max(1.0, abs(one[k])), (k, one[k], two[k])
