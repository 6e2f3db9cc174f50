"""Time the LJ13 B=1024 Euler-100 Hutchinson sample+logp solve (tangent kernel) for one molecules-per-workgroup
override (ECNF_MPW_TANGENT, read by ecnf_create's choose_mpw).  Usage: ECNF_MPW_TANGENT=3 python tools/mpw_sweep.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ecnf-baseline-neurips-2023_amd"))
import torch  # noqa: E402
from ecnf_amd import CONFIGS, init_params, _lib  # noqa: E402
from ecnf_amd.engine import EcnfHandle, SolveOptions  # noqa: E402

cfg = CONFIGS["lj13"]
B = 1024
h = EcnfHandle(cfg, init_params(cfg, 0), 0)
g = torch.Generator("cuda").manual_seed(0)
z = torch.randn((B, cfg.event_dim), device="cuda", generator=g)
x0 = h.base_sample(z)
feat = torch.zeros((B, cfg.n_nodes), device="cuda", dtype=torch.int32)
o = SolveOptions("euler", 0.01)
h.integrate(x0, feat, 0.0, 1.0, o, _lib.DIV_HUTCHINSON, z, check_status=False)
ts = []
for _ in range(3):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    y, dl, _, _ = h.integrate(x0, feat, 0.0, 1.0, o, _lib.DIV_HUTCHINSON, z, check_status=False)
    b.record()
    torch.cuda.synchronize()
    ts.append(a.elapsed_time(b))
print(json.dumps({"mpw_tangent": os.environ.get("ECNF_MPW_TANGENT", "auto"), "ms": sorted(ts)[1],
                  "dlogp_sum": float(dl.double().sum())}))
