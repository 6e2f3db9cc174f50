"""Diagnostic: are two ALDP tangent workgroups co-resident on one CU?  Fixed-step Euler Hutchinson solves (every molecule
the same NFE, one launch, no workspace) of ALDP at B = 64 ... 1024 molecules: with one workgroup per CU the time steps
at multiples of the CU count, with two it stays flat up to twice the CU count.  Same for the LJ13 primal (MPW = 2) and
tangent kernels as controls.  Usage: python tools/diag/occupancy_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "ecnf-baseline-neurips-2023_amd"))

import torch  # noqa: E402
from ecnf_amd import CONFIGS, init_params, _lib  # noqa: E402
from ecnf_amd.engine import EcnfHandle, SolveOptions  # noqa: E402

ncu = torch.cuda.get_device_properties(0).multi_processor_count
print("CUs", ncu, flush=True)
for name, div, dt in (("aldp", _lib.DIV_HUTCHINSON, 0.125), ("aldp", _lib.DIV_NONE, 0.125),
                      ("lj13", _lib.DIV_HUTCHINSON, 0.125)):
    cfg = CONFIGS[name]
    h = EcnfHandle(cfg, init_params(cfg, 0), 0)
    for B in (64, 128, 192, 256, 320, 384, 448, 512, 640, 768, 1024):
        g = torch.Generator("cuda").manual_seed(3)
        z = torch.randn((B, cfg.event_dim), device="cuda", generator=g)
        x = h.base_sample(z)
        feat = (torch.arange(cfg.n_nodes, device="cuda", dtype=torch.int32) % cfg.n_features).expand(B, -1).contiguous()
        eps = z if div == _lib.DIV_HUTCHINSON else None
        ts = []
        for _ in range(4):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            h.integrate(x, feat, 1.0, 0.0, SolveOptions("euler", dt), div, eps, check_status=False)
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        wg, launches = h.integrate_plan(B, 1.0, 0.0, SolveOptions("euler", dt), div)
        print(f"{name} div={div} B={B:5d} workgroups={wg:5d} ms={sorted(ts)[1]:.3f}", flush=True)
    h.close()
