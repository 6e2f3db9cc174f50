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
