"""Device-checked diagnostic build (a HIP debug build with bounds asserts).

tools/debug/build.sh compiles the LJ13-shape kernels with ECNF_DCHECK bounds checks (egnn_eval.hpp: LDS carve-up
against the launch's dynamic LDS, edge receiver / sender rows, edge tiles, node-GEMM row tiles, stored segment
parts, molecule slots).  A child process runs every LJ13 mode through that library at batch sizes that exercise the
batch-aware workgroup sizing (1, 5, 13, 300, 1024 molecules; the exact trace at every size, so the bounds of its
primal-aggregate cache slots are checked at 1024 molecules too, bit 6) and reads the failed-check bits with
ecnf_debug_checks(); they must be 0, and the outputs must match the product library (the checks do not touch the
arithmetic).  A 48-atom molecule with the LJ13 widths runs the receiver-tiled edge layout (N > 33) through the same
checks (field and Euler sample at 1, 7 and 300 molecules)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHECKED = os.path.join(ROOT, "tools", "debug", "libecnf_hip_checked.so")

CHILD = r"""
import ctypes, json, os, sys
import numpy as np, torch
sys.path.insert(0, os.path.join(%(root)r, "ecnf-baseline-neurips-2023_amd"))
from ecnf_amd import CONFIGS, init_params, _lib
from ecnf_amd.engine import EcnfHandle, SolveOptions
cfg = CONFIGS["lj13"]
h = EcnfHandle(cfg, init_params(cfg, 0), 0)
lib = h.lib
lib.ecnf_debug_checks.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.c_int]
flags = ctypes.c_uint32(0)
lib.ecnf_debug_checks(ctypes.byref(flags), 1)
out = {}
g = torch.Generator("cuda").manual_seed(7)
for B in (1, 5, 13, 300, 1024):
    z = torch.randn((B, cfg.event_dim), device="cuda", generator=g)
    x0 = h.base_sample(z)
    feat = torch.zeros((B, cfg.n_nodes), device="cuda", dtype=torch.int32)
    t = torch.linspace(0.05, 0.95, B, device="cuda")
    v = h.vector_field(x0, t, feat)
    u = torch.randn((B, 2, cfg.event_dim), device="cuda", generator=g)
    _, ju = h.jvp(x0, t, feat, u)
    y, _, _, _ = h.integrate(x0, feat, 0.0, 1.0, SolveOptions("euler", 0.1))
    yh, dl, _, _ = h.integrate(x0, feat, 0.0, 1.0, SolveOptions("euler", 0.25), _lib.DIV_HUTCHINSON, z)
    ya, _, nfe, _ = h.integrate(x0, feat, 0.0, 1.0, SolveOptions("dopri5", None))
    # the exact trace with its primal-aggregate cache in a caller workspace (every cache slot of the grid touched)
    ye, dle, _, _ = h.integrate(x0, feat, 1.0, 0.0, SolveOptions("euler", 0.5), _lib.DIV_EXACT)
    rec = dict(z=z, v=v, ju=ju, y=y, yh=yh, dl=dl, ya=ya, ye=ye, dle=dle)
    out[B] = {k: w.detach().cpu().numpy() for k, w in rec.items()}
# receiver-tiled edges (N = 48 > 33: every receiver's 47 edges on two whole tiles), the LJ13 widths: primal paths
from ecnf_amd.params import CNFConfig
big = CNFConfig(n_nodes=48, dim=3, n_features=1, hidden=64, mlp_width=128, mlp_depth=3, n_blocks=2, base_scale=1.0,
                sigma_min=0.01)
hb = EcnfHandle(big, init_params(big, 1), 0)
for B in (1, 7, 300):
    x0 = hb.base_sample(torch.randn((B, big.event_dim), device="cuda", generator=g))
    feat = torch.zeros((B, big.n_nodes), device="cuda", dtype=torch.int32)
    v = hb.vector_field(x0, torch.linspace(0.05, 0.95, B, device="cuda"), feat)
    y, _, _, _ = hb.integrate(x0, feat, 0.0, 1.0, SolveOptions("euler", 0.25))
    assert bool(torch.isfinite(v).all()) and bool(torch.isfinite(y).all())
lib.ecnf_debug_checks(ctypes.byref(flags), 1)
np.savez(sys.argv[1], **{f"{B}_{k}": w for B, d in out.items() for k, w in d.items()})
print(json.dumps({"flags": int(flags.value)}))
"""


def test_device_checks_pass_and_match_product(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    if not os.path.exists(CHECKED):
        pytest.fail("tools/debug/libecnf_hip_checked.so is not built: run tools/debug/build.sh")
    npz = str(tmp_path / "checked.npz")
    env = dict(os.environ, ECNF_LIB=CHECKED)
    r = subprocess.run([sys.executable, "-c", CHILD % {"root": ROOT}, npz], env=env, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    flags = json.loads(r.stdout.strip().splitlines()[-1])["flags"]
    assert flags == 0, f"device bounds checks failed: bits {flags:#x}"

    # the product library on the same inputs
    from ecnf_amd import CONFIGS, init_params, _lib
    from ecnf_amd.engine import EcnfHandle, SolveOptions
    cfg = CONFIGS["lj13"]
    h = EcnfHandle(cfg, init_params(cfg, 0), 0)
    C = np.load(npz)
    for B in (1, 5, 13, 300, 1024):
        z = torch.as_tensor(C[f"{B}_z"], device="cuda")
        x0 = h.base_sample(z)
        feat = torch.zeros((B, cfg.n_nodes), device="cuda", dtype=torch.int32)
        t = torch.linspace(0.05, 0.95, B, device="cuda")
        y, _, _, _ = h.integrate(x0, feat, 0.0, 1.0, SolveOptions("euler", 0.1))
        v = h.vector_field(x0, t, feat)
        yh, dl, _, _ = h.integrate(x0, feat, 0.0, 1.0, SolveOptions("euler", 0.25), _lib.DIV_HUTCHINSON, z)
        ye, dle, _, _ = h.integrate(x0, feat, 1.0, 0.0, SolveOptions("euler", 0.5), _lib.DIV_EXACT)
        for name, got in (("y", y), ("v", v), ("yh", yh), ("dl", dl), ("ye", ye), ("dle", dle)):
            ref = C[f"{B}_{name}"]
            err = np.abs(got.cpu().numpy() - ref).max() / max(1.0, np.abs(ref).max())
            assert err <= 1e-6, (B, name, err)
