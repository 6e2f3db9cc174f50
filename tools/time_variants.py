"""A/B timing of tools/libt_*.so (tools/build_timing.sh): LJ13 B=1024 Euler NFE=100 integrate launches, each
library in its own subprocess, ROUNDS interleaved rounds (A B C A B C ...) so clock drift hits all alike.
Prints the median ms per launch of each library."""
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
cfg = CONFIGS["lj13"]
h = EcnfHandle(cfg, init_params(cfg, 0), 0)
z = torch.randn((1024, cfg.event_dim), device="cuda", generator=torch.Generator("cuda").manual_seed(0))
x0 = h.base_sample(z)
feat = torch.zeros((1024, cfg.n_nodes), device="cuda", dtype=torch.int32)
o = SolveOptions("euler", 0.01)
for _ in range(2): h.integrate(x0, feat, 0.0, 1.0, o, check_status=False)
ts = []
for _ in range(5):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(); y = h.integrate(x0, feat, 0.0, 1.0, o, check_status=False)[0]; b.record(); torch.cuda.synchronize()
    ts.append(a.elapsed_time(b))
print(json.dumps({"ms": sorted(ts)[2], "sum": float(y.double().abs().sum())}))
""" % ROOT

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
libs = sorted(glob.glob(os.path.join(ROOT, "tools", "libt_*.so")))
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
