"""Training step alone (loss + reverse-mode gradient + Adam, lj13.yaml batch 64) for rocprofv3 kernel traces and
A/B timing of the training kernels: prints one JSON line with the HIP-event ms per step and the loss.
Usage: python tools/train_step.py [--config lj13] [--batch 64] [--steps 20]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ecnf-baseline-neurips-2023_amd"))

import torch  # noqa: E402

from ecnf_amd import CONFIGS, init_params  # noqa: E402
from ecnf_amd import train as TRN  # noqa: E402
from ecnf_amd.engine import EcnfHandle  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="lj13")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    cfg = CONFIGS[args.config]
    dev = torch.device("cuda", 0)
    h = EcnfHandle(cfg, init_params(cfg, 0), 0)
    tr = TRN.Trainer(cfg, max_batch=args.batch, device=0)
    p = tr.device_params(init_params(cfg, 0))
    mu, nu = torch.zeros_like(p), torch.zeros_like(p)
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    xd = h.base_sample(torch.randn((args.batch, cfg.event_dim), generator=g, device=dev))
    xb = h.base_sample(torch.randn((args.batch, cfg.event_dim), generator=g, device=dev))
    tt = torch.rand((args.batch,), generator=g, device=dev)
    ft = torch.zeros((args.batch, cfg.n_nodes), device=dev, dtype=torch.int32)
    stream = torch.cuda.current_stream()
    losses = []
    for i in range(args.steps + 2):
        if i == 2:
            torch.cuda.synchronize(dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
        loss, grad = tr.loss_and_grad(p, xd, xb, tt, ft)
        tr.adam_update(grad, p, mu, nu, None, lr=1e-4, count=i + 1)
        if i < 2:
            losses.append(float(loss))
    e1.record(stream)
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / args.steps
    print(json.dumps({"config": args.config, "batch": args.batch, "ms_per_step": ms, "loss0": losses[0],
                      "loss1": losses[1], "grad_abs_sum": float(grad.double().abs().sum())}), flush=True)


if __name__ == "__main__":
    main()
