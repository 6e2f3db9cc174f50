"""Diagnostic: per-phase shader-cycle shares of integrate_kernel (LJ13 B=1024 Euler NFE=100) from the
-DECNF_STAMPS build (tools/build_stamps.sh).  Shares are read from workgroup thread 0 at barrier boundaries."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ecnf-baseline-neurips-2023_amd"))
os.environ["ECNF_LIB"] = os.environ.get("ECNF_STAMPS_LIB", os.path.join(ROOT, "tools", "libecnf_hip_stamps.so"))

import torch  # noqa: E402
from ecnf_amd import CONFIGS, init_params, _lib  # noqa: E402
from ecnf_amd.engine import EcnfHandle, SolveOptions  # noqa: E402

NAMES = ["prologue", "node_dense", "p_gemm", "edge", "node_update", "phi_h", "epilogue", "solver",
         "edge_chain_e(w0)", "edge_shift(w0)", "edge_layer1(w0)", "edge_gate_agg(w0)", "edge_phix_in(w0)",
         "edge_phix_chain(w0)", "team_exchange"]
name = sys.argv[1] if len(sys.argv) > 1 else "lj13"
TEAM = int(os.environ.get("ECNF_PROBE_TEAM", "0"))   # ecnf_set_team mode for the probe (0 auto)
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
DIV = sys.argv[3] if len(sys.argv) > 3 else "none"   # none | hutchinson (the tangent kernel)
cfg = CONFIGS[name]
h = EcnfHandle(cfg, init_params(cfg, 0), 0)
h.set_team(TEAM)
lib = h.lib
lib.ecnf_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
z = torch.randn((B, cfg.event_dim), device="cuda")
x0 = h.base_sample(z)
feat = torch.zeros((B, cfg.n_nodes), device="cuda", dtype=torch.int32)
eps = torch.randn((B, cfg.event_dim), device="cuda") if DIV == "hutchinson" else None
div = _lib.DIV_HUTCHINSON if DIV == "hutchinson" else _lib.DIV_NONE
h.integrate(x0, feat, 0.0, 1.0, SolveOptions("euler", 0.01), div, eps)
buf = (ctypes.c_ulonglong * 32)()
lib.ecnf_debug_stamps(buf, 32, 1)
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
h.integrate(x0, feat, 0.0, 1.0, SolveOptions("euler", 0.01), div, eps)
ev1.record()
torch.cuda.synchronize()
lib.ecnf_debug_stamps(buf, 32, 1)
nwg = buf[28]
cyc = [buf[i] / nwg for i in range(len(NAMES))]
MAIN = list(range(8)) + [14]   # barrier-delimited phases (incl. the team exchange); 8..13 are edge sub-phases
tot = sum(cyc[i] for i in MAIN)
real_us = buf[29] / nwg / 100.0   # s_memrealtime is 100 MHz
out = {"config": name, "batch": B, "divergence": DIV, "workgroups": nwg, "kernel_ms": ev0.elapsed_time(ev1),
       "cycles_per_wg": tot, "wg_wall_us": real_us, "clock_GHz": tot / (real_us * 1e3),
       "shares": {NAMES[i]: cyc[i] / tot for i in MAIN},
       "edge_wave0_shares_of_edge": {NAMES[i]: cyc[i] / max(cyc[3], 1) for i in range(8, 14)}}
print(json.dumps(out, indent=1))
