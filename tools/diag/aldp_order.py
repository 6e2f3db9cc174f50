"""Does the ALDP adaptive launch wait on workgroup dispatch order?  The B = 512 PID Hutchinson log_prob of
aldp_tail.py, timed with the molecules in their original order, sorted by their (measured) NFE descending and
ascending.  One molecule per workgroup and one workgroup per CU (the M = 64 tangent kernel's 8 x 256-register
waves), so the second 256 workgroups start only as earlier ones retire, in dispatch order.  Outputs must be the same
per molecule in every order (bitwise).  Usage: python tools/diag/aldp_order.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "ecnf-baseline-neurips-2023_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from ecnf_amd import CONFIGS, init_params, _lib  # noqa: E402
from ecnf_amd.engine import EcnfHandle, SolveOptions  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from aldp_tail import timed  # noqa: E402


def main():
    cfg = CONFIGS["aldp"]
    h = EcnfHandle(cfg, init_params(cfg, 0), 0)
    print(json.dumps({"mpw_tangent": h.molecules_per_workgroup(True)}))
    B = 512
    g = torch.Generator("cuda").manual_seed(1234)
    z = torch.randn((B, cfg.event_dim), device="cuda", generator=g)
    x0 = h.base_sample(z)
    feat = (torch.arange(cfg.n_nodes, device="cuda", dtype=torch.int32) % cfg.n_features).expand(B, -1).contiguous()
    eps = torch.randn((B, cfg.event_dim), device="cuda", generator=g)
    o = SolveOptions("dopri5", None)
    _, nfe0 = timed(h, x0, feat, 1.0, 0.0, o, _lib.DIV_HUTCHINSON, eps, reps=1)
    ref = h.integrate(x0, feat, 1.0, 0.0, o, _lib.DIV_HUTCHINSON, eps, check_status=False)
    for name, perm in (("original", torch.arange(B, device="cuda")),
                       ("nfe_descending", torch.argsort(nfe0, descending=True, stable=True)),
                       ("nfe_ascending", torch.argsort(nfe0, descending=False, stable=True))):
        xp, fp, ep = x0[perm].contiguous(), feat[perm].contiguous(), eps[perm].contiguous()
        ms, nfe = timed(h, xp, fp, 1.0, 0.0, o, _lib.DIV_HUTCHINSON, ep, reps=3)
        y, dl, nf, st = h.integrate(xp, fp, 1.0, 0.0, o, _lib.DIV_HUTCHINSON, ep, check_status=False)
        same = bool(torch.equal(y, ref[0][perm]) and torch.equal(dl, ref[1][perm]) and torch.equal(nf, ref[2][perm]))
        print(json.dumps({"order": name, "ms": round(ms, 3), "nfe_max": int(nfe.max()), "first8_nfe": nf[:8].tolist(),
                          "bitwise_same_per_molecule": same}), flush=True)
    h.close()


if __name__ == "__main__":
    main()
