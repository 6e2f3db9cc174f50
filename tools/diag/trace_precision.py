"""Diagnostic: where does the exact-trace error of the LJ13 kernels come from?  For a few molecules at one time t,
compare against the fp64 / fp32 oracle: (a) the exact-trace solve (one Euler step), split and strict-fp32 kernels;
(b) the full trace of the 39 unit JVPs from ecnf_vf_jvp (no translation identity); (c) the identity form
sum_{k>=D}(J_kk - J_(k mod D),k) - D from the same JVPs."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ecnf-baseline-neurips-2023_amd")]
from oracle import ecnf_oracle as O  # noqa: E402
from ecnf_amd import CONFIGS, _lib  # noqa: E402
from ecnf_amd.engine import EcnfHandle, SolveOptions  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "lj13"
cfg, oc = CONFIGS[name], O.CONFIGS[name]
p = O.stress_params(O.init_params(oc, 0), oc)
B = 3
rng = np.random.default_rng(1)
z = rng.standard_normal((B, cfg.event_dim)).astype(np.float32)
x0 = O.base_sample(z, oc)
feat = rng.integers(0, cfg.n_features, (B, cfg.n_nodes)).astype(np.int32)
t = np.ones(B, np.float32)
ND, D = cfg.event_dim, cfg.dim
eye = np.broadcast_to(np.eye(ND, dtype=np.float32), (B, ND, ND)).copy()
_, J64 = O.egnn_vector_field(p, oc, x0, t, feat, tangents=eye, dtype=np.float64)
_, J32 = O.egnn_vector_field(p, oc, x0, t, feat, tangents=eye, dtype=np.float32)
tr64 = np.einsum("bkk->b", J64)
tr32 = np.einsum("bkk->b", J32)
absum = np.einsum("bkk->b", np.abs(J64))
print(f"{name}: trace64 {tr64}, sum|J_kk| {absum}")
print(f"fp32 oracle full trace err {np.abs(tr32 - tr64).max():.3e}")
for prec in ("split_f16", "fp32"):
    h = EcnfHandle(cfg, p, 0, precision=prec)
    g = lambda a, dt=torch.float32: torch.as_tensor(np.asarray(a), device="cuda", dtype=dt)
    _, ju = h.jvp(g(x0), g(t), g(feat, torch.int32), g(eye))
    J = ju.cpu().numpy().astype(np.float64)     # [B, k, ND]: column k = J e_k
    full = np.einsum("bkk->b", J)
    ident = sum(J[:, k, k] - J[:, k, k % D] for k in range(D, ND)) - D
    print(f"[{prec}] per-entry |J - J64| max {np.abs(J - J64).max():.3e} (fp32 oracle {np.abs(J32 - J64).max():.3e})")
    print(f"[{prec}] full trace err {np.abs(full - tr64).max():.3e}   identity trace err {np.abs(ident - tr64).max():.3e}")
    diag_err = np.array([J[:, k, k] - J64[:, k, k] for k in range(ND)])
    diag_32 = np.array([J32[:, k, k] - J64[:, k, k] for k in range(ND)])
    print(f"[fp32 oracle] diag errors: sum {diag_32.sum(0)}, rms {np.sqrt((diag_32**2).mean()):.3e}")
    print(f"[{prec}] diag errors: sum {diag_err.sum(0)}, mean {diag_err.mean():.3e}, rms {np.sqrt((diag_err**2).mean()):.3e}")
    _, dl, _, _ = h.integrate(g(x0), g(feat, torch.int32), 1.0, 0.0, SolveOptions("euler", 1.0),
                              divergence=_lib.DIV_EXACT)
    print(f"[{prec}] exact solve dl err {np.abs(-dl.cpu().numpy() - tr64).max():.3e}  (dl = -1 * trace at t = 1)")
