"""Diagnostic: the LJ13 vector field of two libraries (ECNF_LIB_A, ECNF_LIB_B; e.g. tools/libt_head.so and a block-1 pair
tile build) on the same seeded molecules, each library in its own subprocess: per-atom max |dv| and the relative error
against the fp64 oracle.  Usage: python tools/diag/pair_diff.py [B]"""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CHILD = r"""
import os, sys, numpy as np, torch
sys.path.insert(0, os.path.join(%r, "ecnf-baseline-neurips-2023_amd"))
sys.path.insert(0, %r)
from ecnf_amd import CONFIGS
from ecnf_amd.engine import EcnfHandle
from oracle import ecnf_oracle as O
B = int(sys.argv[1]); out = sys.argv[2]
cfg = CONFIGS["lj13"]
oc = O.CNFConfig(n_nodes=13, dim=3, n_features=1, hidden=cfg.hidden, time_embedding_dim=cfg.time_embedding_dim,
                 mlp_width=cfg.mlp_width, mlp_depth=cfg.mlp_depth, n_blocks=cfg.n_blocks, base_scale=cfg.base_scale,
                 sigma_min=cfg.sigma_min)
params = O.stress_params(O.init_params(oc, 0), oc)
h = EcnfHandle(cfg, params, 0)
g = torch.Generator("cuda").manual_seed(7)
x = h.base_sample(torch.randn((B, cfg.event_dim), device="cuda", generator=g))
t = torch.rand(B, device="cuda", generator=g)
feat = torch.zeros((B, cfg.n_nodes), device="cuda", dtype=torch.int32)
v = h.vector_field(x, t, feat)
np.savez(out, x=x.cpu().numpy(), t=t.cpu().numpy(), v=v.cpu().numpy())
""" % (ROOT, ROOT)

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4
res = {}
for tag in ("A", "B"):
    lib = os.environ["ECNF_LIB_" + tag]
    out = f"/tmp/pair_diff_{tag}.npz"
    subprocess.run([sys.executable, "-c", CHILD, str(B), out], env=dict(os.environ, ECNF_LIB=lib), check=True)
    res[tag] = np.load(out)
assert np.array_equal(res["A"]["x"], res["B"]["x"])
va, vb = res["A"]["v"].reshape(B, 13, 3), res["B"]["v"].reshape(B, 13, 3)
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "ecnf-baseline-neurips-2023_amd"))
from oracle import ecnf_oracle as O  # noqa: E402
from ecnf_amd import CONFIGS  # noqa: E402
cfg = CONFIGS["lj13"]
oc = O.CNFConfig(n_nodes=13, dim=3, n_features=1, hidden=cfg.hidden, time_embedding_dim=cfg.time_embedding_dim,
                 mlp_width=cfg.mlp_width, mlp_depth=cfg.mlp_depth, n_blocks=cfg.n_blocks, base_scale=cfg.base_scale,
                 sigma_min=cfg.sigma_min)
params = O.stress_params(O.init_params(oc, 0), oc)
ref = O.egnn_vector_field(params, oc, res["A"]["x"].astype(np.float64), res["A"]["t"], np.zeros((B, 13), np.int64),
                          dtype=np.float64).reshape(B, 13, 3)
print(json.dumps({
    "per_atom_max_abs_diff_A_B": np.abs(va - vb).max(axis=(0, 2)).tolist(),
    "max_abs_A_vs_oracle": float(np.abs(va - ref).max()),
    "max_abs_B_vs_oracle": float(np.abs(vb - ref).max()),
    "max_abs_ref": float(np.abs(ref).max()),
}, indent=1))
