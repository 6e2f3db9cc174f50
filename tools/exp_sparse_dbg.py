"""Diagnostic for the exact trace's sparse dual tiles (blocks 1 and K): ECNF_EXACT_SPARSE=0 (every tile dual) vs the
default (1 = sparse without, 2 = with the primal-aggregate cache); LJ13, B = 3, one Euler step of dt = 1 (one evaluation) and 20 steps of 0.05."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ecnf-baseline-neurips-2023_amd"))
from oracle import ecnf_oracle as O  # noqa: E402
from ecnf_amd import CONFIGS, _lib  # noqa: E402
from ecnf_amd.engine import EcnfHandle, SolveOptions  # noqa: E402

cfg = CONFIGS["lj13"]
oc = O.CONFIGS["lj13"]
p = O.stress_params(O.init_params(oc, 0), oc)
h = EcnfHandle(cfg, p, 0)
rng = np.random.default_rng(1)
x0 = O.base_sample(rng.standard_normal((3, cfg.event_dim)).astype(np.float32), oc)
feat = np.zeros((3, cfg.n_nodes), np.int32)
g = lambda a, t=torch.float32: torch.as_tensor(a, device="cuda", dtype=t)
for dt in (1.0, 0.05):
    res = {}
    for mode, (sparse, pcache) in enumerate([("0", "1"), ("1", "0"), ("1", "1")]):
        os.environ["ECNF_EXACT_SPARSE"] = sparse
        os.environ["ECNF_EXACT_PCACHE"] = pcache
        x, dl, _, st = h.integrate(g(x0), g(feat, torch.int32), 1.0, 0.0, SolveOptions("euler", dt),
                                   divergence=_lib.DIV_EXACT)
        res[mode] = (x.cpu().numpy(), dl.cpu().numpy())
    for mode in (1, 2):
        print(f"dt {dt} form {mode}: |x - x_dense| {np.abs(res[mode][0] - res[0][0]).max():.3g}  "
              f"|dl - dl_dense| {np.abs(res[mode][1] - res[0][1]).max():.3g} (|dl| {np.abs(res[0][1]).max():.3g})",
              flush=True)
