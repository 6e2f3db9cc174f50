"""Rehearsal of the multi-GPU bench path (BASELINE.json configs[4]: LJ13 sharded over ranks, the eval leg's ESS
reduced across ranks) with 2 ranks folded onto one GPU over gloo.

`bench.py --gpus 2` (WORLD_SIZE unset) must start the 2 rank processes itself, the JSON line must report the world the
process group formed, each rank's shard must be bitwise equal to the same rows of a 1-rank run (one global noise draw;
per-molecule results independent of batch position), and the cross-rank reverse / forward ESS and mean log q must
match the single-process oracle over the concatenated log weights (setup_training.py:166-185, evaluation.py:10-22)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from oracle import ecnf_oracle as O

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs a ROCm GPU", allow_module_level=True)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--batch", "96", "--nfe", "10", "--steps", "1", "--warmup", "1", "--logprob", "1", "--fp32-steps", "0", "--train-steps", "0",
        "--cpu-molecules", "0", "--pmc", "0"]


def _run(gpus, dump, backend="gloo"):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--dist-backend",
                          backend, "--dump", str(dump), *ARGS], capture_output=True, text=True, timeout=240, env=env,
                         cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    return json.loads(lines[0])


@pytest.mark.timeout(400)
def test_two_ranks_match_one_rank(tmp_path):
    one = _run(1, tmp_path / "w1")
    two = _run(2, tmp_path / "w2")
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert two["config"]["global_batch"] == one["config"]["global_batch"] == 96
    assert two["config"]["batch_per_gpu"] == 48
    r1 = np.load(tmp_path / "w1" / "rank0.npz")
    parts = [np.load(tmp_path / "w2" / f"rank{r}.npz") for r in range(2)]
    assert all(int(p["world"]) == 2 for p in parts)
    assert [int(p["lo"]) for p in parts] == [0, 48] and [int(p["hi"]) for p in parts] == [48, 96]
    for key in ("x1", "x1_lp", "log_q", "log_w"):
        cat = np.concatenate([p[key] for p in parts])
        assert np.array_equal(cat, r1[key]), key
    log_w = r1["log_w"].astype(np.float64)
    rev = O.reverse_ess(log_w)
    for res in (one, two):
        lp = res["logprob"]
        assert lp["status_ok"]
        assert abs(lp["rev_ess"] - rev) <= 1e-5 * rev + 1e-9, (lp["rev_ess"], rev)
        assert abs(lp["mean_log_q"] - float(r1["log_q"].astype(np.float64).mean())) <= 1e-4


@pytest.mark.timeout(600)
def test_configs4_per_gpu_size_two_ranks(tmp_path):
    """BASELINE.json configs[4] at its per-GPU size on one GPU: `bench.py --gpus 2 --dist-backend gloo --batch 16384`
    runs 8192 LJ13 molecules per rank (65,536 / 8, the per-GPU share of the 8-GPU run) at the headline NFE = 100 plus
    the eval leg (Hutchinson sample_and_log_prob_cnf -> LJ13 target -> reverse ESS over the process group,
    setup_training.py:166-185).  Checks: each shard is bitwise the same rows of a 1-rank run of the same global batch;
    4 strided molecules per shard match the oracle (x1 within 1e-4 of fp64, log q fp32-class); the cross-rank reverse
    ESS and mean log q match the oracle's reductions over the concatenated log weights.  Only the hardware 8-GPU run
    (RCCL over xGMI) is left untested."""
    from tolerance import fp32_class
    args = ["--batch", "16384", "--nfe", "100", "--steps", "1", "--warmup", "1", "--logprob", "1", "--fp32-steps", "0",
            "--train-steps", "0", "--cpu-molecules", "0", "--pmc", "0", "--ref-latency-samples", "0"]

    def run(gpus, dump):
        env = dict(os.environ)
        for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
            env.pop(k, None)
        out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--dist-backend",
                              "gloo", "--dump", str(dump), *args], capture_output=True, text=True, timeout=280,
                             env=env, cwd=ROOT)
        assert out.returncode == 0, out.stderr[-3000:]
        lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
        assert len(lines) == 1, out.stdout
        return json.loads(lines[0])

    two = run(2, tmp_path / "w2")
    one = run(1, tmp_path / "w1")
    assert two["n_gpus"] == 2 and two["config"]["batch_per_gpu"] == 8192 and two["config"]["nfe"] == 100
    r1 = np.load(tmp_path / "w1" / "rank0.npz")
    parts = [np.load(tmp_path / "w2" / f"rank{r}.npz") for r in range(2)]
    assert [int(p["lo"]) for p in parts] == [0, 8192] and [int(p["hi"]) for p in parts] == [8192, 16384]
    for key in ("z", "x0", "x1", "x1_lp", "log_q", "log_w"):
        assert np.array_equal(np.concatenate([p[key] for p in parts]), r1[key]), key
    # 4 strided molecules per shard against the oracle (the bench's weights: init_params(lj13, 0), zero features)
    oc = O.CONFIGS["lj13"]
    params = O.init_params(oc, 0)
    for p in parts:
        rows = np.arange(4) * 2048 + 1234            # strided rows of the shard
        x0, z = p["x0"][rows], p["z"][rows]
        feat = np.zeros((4, oc.n_nodes), np.int32)
        x64, _ = O.sample_cnf(params, oc, x0, feat, solver="euler", dt0=0.01, dtype=np.float64)
        assert np.abs(p["x1"][rows] - x64).max() <= 1e-4
        _, lq64, _ = O.sample_and_log_prob(params, oc, x0, feat, eps=z, approx=True, solver="euler", dt0=0.01,
                                           dtype=np.float64)
        _, lq32, _ = O.sample_and_log_prob(params, oc, x0, feat, eps=z, approx=True, solver="euler", dt0=0.01,
                                           dtype=np.float32)
        fp32_class(f"configs4 shard {int(p['lo'])} log_q", p["log_q"][rows], lq64, lq32)
    log_w = r1["log_w"].astype(np.float64)
    rev = O.reverse_ess(log_w)
    for res in (one, two):
        lp = res["logprob"]
        assert lp["status_ok"]
        assert abs(lp["rev_ess"] - rev) <= 1e-5 * rev + 1e-9, (lp["rev_ess"], rev)
        assert abs(lp["mean_log_q"] - float(r1["log_q"].astype(np.float64).mean())) <= 1e-4


@pytest.mark.timeout(900)
def test_configs4_full_workload_eight_ranks(tmp_path):
    """BASELINE.json configs[4] at its FULL workload on one GPU: `bench.py --gpus 8 --dist-backend gloo` (defaults:
    global batch 65,536, 8,192 LJ13 molecules per rank, Euler NFE = 100, the eval leg -- Hutchinson
    sample_and_log_prob_cnf -> LJ13 target -> reverse ESS and mean log q reduced across the 8 ranks;
    setup_training.py:166-185, evaluation.py:10-22), the 8 ranks folded onto the one GPU.  Checks: world = 8 reported;
    each rank's shard is bitwise the same rows of a 1-rank run of the whole 65,536-molecule batch; 2 strided molecules
    of every shard match the oracle (x1 within 1e-4 of fp64, log q fp32-class); the 8-rank reverse ESS and mean log q
    equal the single-process values.  Only the placement on 8 devices with RCCL over xGMI is left to the hardware run
    (RCCL itself: tests/test_gpu_rccl.py)."""
    from tolerance import fp32_class
    args = ["--nfe", "100", "--steps", "1", "--warmup", "1", "--logprob", "1", "--fp32-steps", "0",
            "--train-steps", "0", "--cpu-molecules", "0", "--pmc", "0", "--ref-latency-samples", "0"]

    def run(gpus, dump, extra=()):
        env = dict(os.environ)
        for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
            env.pop(k, None)
        out = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", str(gpus),
                              "--dist-backend", "gloo", "--dump", str(dump), *args, *extra], capture_output=True,
                             text=True, timeout=420, env=env, cwd=ROOT)
        assert out.returncode == 0, out.stderr[-3000:]
        lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
        assert len(lines) == 1, out.stdout
        return json.loads(lines[0])

    eight = run(8, tmp_path / "w8")                             # default global batch at world > 1: 65,536
    one = run(1, tmp_path / "w1", ("--batch", "65536"))
    assert eight["n_gpus"] == 8 and eight["config"]["global_batch"] == 65536
    assert eight["config"]["batch_per_gpu"] == 8192 and eight["config"]["nfe"] == 100
    assert eight["config"]["dist_backend"] == "gloo" and eight["logprob"]["reduced_by"] == "gloo"
    r1 = np.load(tmp_path / "w1" / "rank0.npz")
    parts = [np.load(tmp_path / "w8" / f"rank{r}.npz") for r in range(8)]
    assert all(int(p["world"]) == 8 for p in parts)
    assert [int(p["lo"]) for p in parts] == [8192 * r for r in range(8)]
    for key in ("z", "x0", "x1", "x1_lp", "log_q", "log_w"):
        assert np.array_equal(np.concatenate([p[key] for p in parts]), r1[key]), key
    oc = O.CONFIGS["lj13"]
    params = O.init_params(oc, 0)
    for r, p in enumerate(parts):
        rows = np.array([(977 * r + 131) % 8192, (3571 * r + 4099) % 8192])   # strided rows of every shard
        x0, z = p["x0"][rows], p["z"][rows]
        feat = np.zeros((2, oc.n_nodes), np.int32)
        x64, _ = O.sample_cnf(params, oc, x0, feat, solver="euler", dt0=0.01, dtype=np.float64)
        assert np.abs(p["x1"][rows] - x64).max() <= 1e-4
        _, lq64, _ = O.sample_and_log_prob(params, oc, x0, feat, eps=z, approx=True, solver="euler", dt0=0.01,
                                           dtype=np.float64)
        _, lq32, _ = O.sample_and_log_prob(params, oc, x0, feat, eps=z, approx=True, solver="euler", dt0=0.01,
                                           dtype=np.float32)
        fp32_class(f"configs4 rank {r} log_q", p["log_q"][rows], lq64, lq32)
    l1, l8 = one["logprob"], eight["logprob"]
    assert l1["status_ok"] and l8["status_ok"]
    # (fp32 log-sum-exp partials per rank on the device, combined in fp64: equal up to the partials' rounding)
    assert abs(l8["rev_ess"] - l1["rev_ess"]) <= 1e-5 * l1["rev_ess"] + 1e-12, (l8["rev_ess"], l1["rev_ess"])
    assert abs(l8["mean_log_q"] - l1["mean_log_q"]) <= 1e-9 * max(1.0, abs(l1["mean_log_q"]))
    rev = O.reverse_ess(r1["log_w"].astype(np.float64))
    assert abs(l8["rev_ess"] - rev) <= 1e-5 * rev + 1e-9, (l8["rev_ess"], rev)
