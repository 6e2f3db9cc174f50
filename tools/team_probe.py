"""Diagnostic: team (latency) mode timing (include/ecnf.h ecnf_set_team) for small batches.

For each config and batch, the kernel time (HIP events) of a fixed-step Euler solve at several workgroups per molecule
(G = 1 is the batch path), reported per evaluation, and the wall time of the reference timer's call (Dopri5 + PID,
one molecule per call, the sample copied to the host).  Usage: python tools/team_probe.py [qm9|lj13|aldp] [B ...]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ecnf-baseline-neurips-2023_amd"))

import torch  # noqa: E402
from ecnf_amd import CONFIGS, init_params  # noqa: E402
from ecnf_amd.engine import EcnfHandle, SolveOptions  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "qm9"
batches = [int(b) for b in sys.argv[2:]] or [1, 4]
cfg = CONFIGS[name]
h = EcnfHandle(cfg, init_params(cfg, 0), 0)
g = torch.Generator(device="cuda")
out = {"config": name}
for B in batches:
    g.manual_seed(0)
    x0 = h.base_sample(torch.randn((B, cfg.event_dim), generator=g, device="cuda"))
    feat = torch.zeros((B, cfg.n_nodes), device="cuda", dtype=torch.int32)
    steps = 20
    rows = {}
    ref = None
    modes = [int(m) for m in os.environ.get("TP_MODES", "1,0,2,4,7,13").split(",")]
    for mode in modes:   # 1: batch path, 0: auto (QM9 B <= 9: column-split, G = 26), >= 2: tile-dealt
        h.set_team(mode)
        G = h.team_workgroups(B)
        key = f"{'auto' if mode == 0 else 'forced'}_G{G}"
        if mode != 1 and (G == 1 or key in rows):
            continue
        y, _, _, _ = h.integrate(x0, feat, 0.0, 1.0, SolveOptions("euler", 1.0 / steps))
        ref = y if ref is None else ref
        ts = []
        for _ in range(5):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            y, _, _, _ = h.integrate(x0, feat, 0.0, 1.0, SolveOptions("euler", 1.0 / steps), check_status=False)
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        ms = sorted(ts)[2]
        rows[key] = {"kernel_ms": ms, "us_per_eval": 1e3 * ms / steps, "bitwise_vs_batch": bool(torch.equal(y, ref))}
    if os.environ.get("TP_DUMP"):   # the batch-path (or first mode's) sample, for cross-library comparison
        import numpy as np
        np.save(f"{os.environ['TP_DUMP']}_B{B}.npy", ref.cpu().numpy())
    h.set_team(0)
    # the reference timer's call: PID, one molecule, host copy
    walls, nfes = [], []
    for i in range(6):
        zq = torch.randn((1, cfg.event_dim), generator=g, device="cuda")
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        xq, _, nq, _ = h.integrate(h.base_sample(zq), feat[:1], 0.0, 1.0, SolveOptions("dopri5", None))
        xq.cpu()
        if i:
            walls.append(1e3 * (time.perf_counter() - t1))
            nfes.append(int(nq[0]))
    out[f"B{B}"] = {"euler20": rows, "pid_call_ms": walls, "pid_nfe": nfes, "auto_G": h.team_workgroups(B)}
    print(json.dumps({f"B{B}": out[f"B{B}"]}), flush=True)
print(json.dumps(out))
