"""Where the ALDP adaptive launch goes (BASELINE configs[2]): per-molecule NFE distribution of the B = 512 PID solves
(sample and Hutchinson log_prob, bench_paths inputs), and the launch time of the full batch against the same solve of
the slowest molecules alone (B = 1, 2, 8 of the highest-NFE molecules), i.e. how much of the launch is the serial chain
of one molecule's evaluations on one CU.  Usage: python tools/diag/aldp_tail.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "ecnf-baseline-neurips-2023_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from ecnf_amd import CONFIGS, init_params, _lib  # noqa: E402
from ecnf_amd.engine import EcnfHandle, SolveOptions  # noqa: E402


def timed(h, x0, feat, t0, t1, o, div, eps, reps=3):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        y1, dl, nfe, st = h.integrate(x0, feat, t0, t1, o, div, eps, check_status=False)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return sorted(ts)[len(ts) // 2], nfe


def main():
    cfg = CONFIGS["aldp"]
    h = EcnfHandle(cfg, init_params(cfg, 0), 0)
    B = 512
    g = torch.Generator("cuda").manual_seed(1234)
    z = torch.randn((B, cfg.event_dim), device="cuda", generator=g)
    x0 = h.base_sample(z)
    feat = (torch.arange(cfg.n_nodes, device="cuda", dtype=torch.int32) % cfg.n_features).expand(B, -1).contiguous()
    for div, name, (t0, t1) in ((_lib.DIV_NONE, "sample", (0.0, 1.0)), (_lib.DIV_HUTCHINSON, "logp", (1.0, 0.0))):
        eps = torch.randn((B, cfg.event_dim), device="cuda", generator=g) if div else None
        o = SolveOptions("dopri5", None)
        ms, nfe = timed(h, x0, feat, t0, t1, o, div, eps)
        n = nfe.float()
        q = torch.quantile(n, torch.tensor([0.5, 0.9, 0.99], device="cuda")).tolist()
        order = torch.argsort(nfe, descending=True)
        rec = {"case": name, "B": B, "ms": round(ms, 3), "nfe_mean": round(float(n.mean()), 1),
               "nfe_p50_p90_p99": [round(v, 1) for v in q], "nfe_max": int(nfe.max()),
               "us_per_max_nfe": round(1e3 * ms / int(nfe.max()), 1)}
        for k in (1, 2, 8):
            idx = order[:k]
            ms_k, nfe_k = timed(h, x0[idx].contiguous(), feat[idx].contiguous(), t0, t1, o, div,
                                eps[idx].contiguous() if eps is not None else None)
            rec[f"slowest_{k}_ms"] = round(ms_k, 3)
            rec[f"slowest_{k}_nfe_max"] = int(nfe_k.max())
        print(json.dumps(rec), flush=True)
    h.close()


if __name__ == "__main__":
    main()
