"""Out-of-bounds reads of the weight buffer?  Runs every entry point of one config (field, JVP, Euler / PID solves with
no / Hutchinson / exact divergence) through the library in ECNF_LIB and saves the outputs; with REF.npz (the product
library's outputs) compares bitwise.  A build with -DECNF_DIAG_GUARD=n surrounds the packed weights with n NaN floats
on each side, so any read past either end of the buffer shows up as a NaN or a changed bit.
Usage: [ECNF_LIB=...] python tools/diag/guard_check.py CONFIG OUT.npz [REF.npz]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "ecnf-baseline-neurips-2023_amd"))
import torch  # noqa: E402

from ecnf_amd import CONFIGS, init_params, _lib  # noqa: E402
from ecnf_amd.engine import EcnfHandle, SolveOptions  # noqa: E402


def main():
    name, out = sys.argv[1], sys.argv[2]
    cfg = CONFIGS[name]
    h = EcnfHandle(cfg, init_params(cfg, 3), 0)
    res = {}
    for B in (1, 7, 300):
        g = torch.Generator("cuda").manual_seed(B)
        z = torch.randn((B, cfg.event_dim), device="cuda", generator=g)
        x0 = h.base_sample(z)
        feat = torch.randint(0, cfg.n_features, (B, cfg.n_nodes), device="cuda", generator=g, dtype=torch.int32)
        t = torch.rand(B, device="cuda", generator=g)
        u = torch.randn((B, 2, cfg.event_dim), device="cuda", generator=g)
        res[f"v_{B}"] = h.vector_field(x0, t, feat).cpu().numpy()
        v, j = h.jvp(x0, t, feat, u)
        res[f"jvp_{B}"] = j.cpu().numpy()
        cases = [("euler_none", SolveOptions("euler", 0.05), _lib.DIV_NONE, None),
                 ("euler_hutch", SolveOptions("euler", 0.05), _lib.DIV_HUTCHINSON, z),
                 ("pid_hutch", SolveOptions("dopri5", None), _lib.DIV_HUTCHINSON, z)]
        if B <= 7:
            cases.append(("euler_exact", SolveOptions("euler", 0.1), _lib.DIV_EXACT, None))
        for cname, o, div, e in cases:
            y, dl, nfe, st = h.integrate(x0, feat, 0.0, 1.0, o, div, e, check_status=False)
            res[f"{cname}_{B}_y"] = y.cpu().numpy()
            if dl is not None:
                res[f"{cname}_{B}_dl"] = dl.cpu().numpy()
            res[f"{cname}_{B}_nfe"] = nfe.cpu().numpy()
    np.savez(out, **res)
    nan = {k: int(np.isnan(v).sum()) for k, v in res.items() if np.isnan(v).any()}
    rec = {"lib": os.path.basename(os.environ.get("ECNF_LIB", "product")), "config": name, "arrays": len(res),
           "arrays_with_nan": nan}
    if len(sys.argv) > 3:
        ref = np.load(sys.argv[3])
        rec["differ_from_ref"] = [k for k in res if not np.array_equal(ref[k], res[k], equal_nan=True)]
    print(json.dumps(rec), flush=True)
    h.close()


if __name__ == "__main__":
    main()
