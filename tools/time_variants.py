"""A/B timing of tools/libt_*.so (tools/build_timing.sh): integrate launches of one workload (default LJ13 B=1024
Euler NFE=100; TV_CASE=aldp_sample / aldp_hutch / lj13_hutch select ALDP B=512 PID sample, ALDP B=512 PID
Hutchinson log_prob, LJ13 B=1024 Euler Hutchinson, qm9: QM9 B=2048 Euler NFE=20 sample, qm9_hutch: QM9 B=512 Euler NFE=20 Hutchinson), each library in its own subprocess, ROUNDS interleaved rounds
(A B C A B C ...) so clock drift hits all alike.  Prints the median ms per launch of each library."""
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import os, sys, json, torch
sys.path.insert(0, os.path.join(%r, "ecnf-baseline-neurips-2023_amd"))
from ecnf_amd import CONFIGS, init_params
from ecnf_amd.engine import EcnfHandle, SolveOptions
from ecnf_amd import _lib
case = os.environ.get("TV_CASE", "lj13")
name, B = ("aldp", 512) if case.startswith("aldp") else \
    ("qm9", 512 if case.endswith("hutch") else 2048) if case.startswith("qm9") else ("lj13", 1024)
cfg = CONFIGS[name]
h = EcnfHandle(cfg, init_params(cfg, 0), 0)
z = torch.randn((B, cfg.event_dim), device="cuda", generator=torch.Generator("cuda").manual_seed(0))
x0 = h.base_sample(z)
feat = (torch.arange(cfg.n_nodes, device="cuda", dtype=torch.int32).remainder(cfg.n_features)).expand(B, -1).contiguous()
o = SolveOptions("euler", 0.01) if name == "lj13" else SolveOptions("euler", 0.05) if name == "qm9" else \
    SolveOptions("dopri5", None)
div = _lib.DIV_HUTCHINSON if case.endswith("hutch") else _lib.DIV_NONE
t0, t1 = (1.0, 0.0) if case == "aldp_hutch" else (0.0, 1.0)
eps = z if div else None
for _ in range(2): h.integrate(x0, feat, t0, t1, o, div, eps, check_status=False)
ts = []
for _ in range(5):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(); y = h.integrate(x0, feat, t0, t1, o, div, eps, check_status=False)[0]; b.record(); torch.cuda.synchronize()
    ts.append(a.elapsed_time(b))
print(json.dumps({"ms": sorted(ts)[2], "sum": float(y.double().abs().sum())}))
""" % ROOT

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
libs = sorted(glob.glob(os.path.join(ROOT, "tools", os.environ.get("TV_GLOB", "libt_*.so"))))
res = {os.path.basename(l)[5:-3]: [] for l in libs}
for r in range(rounds):
    for lib in libs:
        env = dict(os.environ, ECNF_LIB=lib)
        envf = lib[:-3] + ".env"   # optional KEY=VALUE lines for this library (e.g. ECNF_MPW)
        if os.path.exists(envf):
            env.update(dict(l.strip().split("=", 1) for l in open(envf) if "=" in l))
        out = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=120)
        if out.returncode != 0:
            print(out.stderr[-2000:])
            sys.exit(out.returncode)
        d = json.loads(out.stdout.strip().splitlines()[-1])
        res[os.path.basename(lib)[5:-3]].append(round(d["ms"], 3))
        print(os.path.basename(lib), r, d, flush=True)
for k, v in res.items():
    print(f"{k:>12}: {sorted(v)[len(v) // 2]:.3f} ms  {v}")
