"""ALDP B = 512 PID solves (sample and Hutchinson log_prob, aldp_tail.py's inputs) through the library in ECNF_LIB:
median launch time of 3 and the outputs saved to an .npz, so the re-dealt (chunked) solve can be compared bitwise
with a one-launch build.  Usage: ECNF_LIB=... python tools/diag/sched_check.py OUT.npz [REF.npz]"""
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
    out = sys.argv[1]
    cfg = CONFIGS["aldp"]
    h = EcnfHandle(cfg, init_params(cfg, 0), 0)
    B = 512
    g = torch.Generator("cuda").manual_seed(1234)
    z = torch.randn((B, cfg.event_dim), device="cuda", generator=g)
    x0 = h.base_sample(z)
    feat = (torch.arange(cfg.n_nodes, device="cuda", dtype=torch.int32) % cfg.n_features).expand(B, -1).contiguous()
    eps = torch.randn((B, cfg.event_dim), device="cuda", generator=g)
    o = SolveOptions("dopri5", None)
    res = {}
    for name, div, (t0, t1), e in (("sample", _lib.DIV_NONE, (0.0, 1.0), None),
                                   ("logp", _lib.DIV_HUTCHINSON, (1.0, 0.0), eps)):
        ts = []
        for _ in range(4):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            y, dl, nfe, st = h.integrate(x0, feat, t0, t1, o, div, e, check_status=False)
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        ts = sorted(ts[1:])
        res[f"{name}_y"] = y.cpu().numpy()
        res[f"{name}_nfe"] = nfe.cpu().numpy()
        res[f"{name}_status"] = st.cpu().numpy()
        if dl is not None:
            res[f"{name}_dl"] = dl.cpu().numpy()
        print(json.dumps({"lib": os.path.basename(os.environ.get("ECNF_LIB", "product")), "case": name,
                          "ms": round(ts[1], 3), "nfe_max": int(nfe.max()), "nfe_mean": round(float(nfe.float().mean()), 2),
                          "status_bad": int((st != 0).sum())}), flush=True)
    np.savez(out, **res)
    if len(sys.argv) > 2:
        ref = np.load(sys.argv[2])
        same = {k: bool(np.array_equal(ref[k], res[k])) for k in res}
        print(json.dumps({"bitwise_equal_to_ref": same}), flush=True)
    h.close()


if __name__ == "__main__":
    main()
