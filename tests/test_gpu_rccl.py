"""RCCL on the GPU (the multi-GPU path's collective backend): `bench.py` under torch.distributed.run with
ONE rank forms an nccl (= RCCL) process group, and the eval leg's reductions (reverse ESS, mean log q: one MAX and one
SUM all-reduce each, ecnf_amd.distributed) then run through RCCL on device tensors.  Two ranks cannot share one GPU
under RCCL, so this is the size the 1-GPU box can run; the 8-GPU run is the driver's.  The rank's outputs must be
bitwise those of a plain single-process run (no process group) and the RCCL-reduced statistics equal to them."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs a ROCm GPU", allow_module_level=True)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--batch", "96", "--nfe", "10", "--steps", "1", "--warmup", "1", "--logprob", "1", "--fp32-steps", "0",
        "--train-steps", "0", "--cpu-molecules", "0", "--pmc", "0", "--ref-latency-samples", "0"]


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _line(out):
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.timeout(300)
def test_bench_eval_leg_over_rccl_one_rank(tmp_path):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    bench = os.path.join(ROOT, "bench.py")
    plain = _line(subprocess.run([sys.executable, bench, "--dump", str(tmp_path / "plain"), *ARGS],
                                 capture_output=True, text=True, timeout=240, env=env, cwd=ROOT))
    rccl = _line(subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
                                 "--master-addr=127.0.0.1", f"--master-port={_port()}", bench, "--dist-backend", "nccl",
                                 "--dump", str(tmp_path / "rccl"), *ARGS],
                                capture_output=True, text=True, timeout=240, env=env, cwd=ROOT))
    assert plain["config"]["dist_backend"] is None
    assert rccl["config"]["dist_backend"] == "nccl" and rccl["n_gpus"] == 1
    a, b = np.load(tmp_path / "plain" / "rank0.npz"), np.load(tmp_path / "rccl" / "rank0.npz")
    for key in ("x1", "x1_lp", "log_q", "log_w"):
        assert np.array_equal(a[key], b[key]), key
    for key in ("rev_ess", "mean_log_q"):
        assert rccl["logprob"][key] == plain["logprob"][key], key
    assert rccl["logprob"]["status_ok"]
