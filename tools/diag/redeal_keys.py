"""Which remaining-work estimate should the re-deal sort by?  ALDP B = 512 PID Hutchinson log_prob through a chunked
build (ECNF_LIB): the solver state each molecule stored at the end of the first chunk (read from the workspace) beside
its final NFE, and the list-scheduling makespan (in evaluations, 256 CUs, one molecule per CU) of the second launch
when the unfinished molecules are dealt in the order of each candidate key, against the order of the true remaining
NFE.  Usage: ECNF_LIB=tools/libt_ach4.so python tools/diag/redeal_keys.py"""
import ctypes
import heapq
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "ecnf-baseline-neurips-2023_amd"))
import torch  # noqa: E402

from ecnf_amd import CONFIGS, init_params, _lib  # noqa: E402
from ecnf_amd.engine import EcnfHandle, SolveOptions, _ptr, _stream  # noqa: E402


def makespan(work, order, ncu=256):
    """list scheduling in dispatch order: each job starts on the first free CU"""
    free = [0.0] * ncu
    heapq.heapify(free)
    end = 0.0
    for j in order:
        t = heapq.heappop(free)
        t += work[j]
        end = max(end, t)
        heapq.heappush(free, t)
    return end


def main():
    cfg = CONFIGS["aldp"]
    h = EcnfHandle(cfg, init_params(cfg, 0), 0)
    B, ND = 512, cfg.event_dim
    g = torch.Generator("cuda").manual_seed(1234)
    z = torch.randn((B, ND), device="cuda", generator=g)
    x0 = h.base_sample(z)
    feat = (torch.arange(cfg.n_nodes, device="cuda", dtype=torch.int32) % cfg.n_features).expand(B, -1).contiguous()
    eps = torch.randn((B, ND), device="cuda", generator=g)
    o = SolveOptions("dopri5", None).to_c(1.0, 0.0, _lib.DIV_HUTCHINSON)
    nbytes = ctypes.c_size_t(0)
    _lib.check(h.lib.ecnf_integrate_workspace_size(h._h, ctypes.byref(o), B, ctypes.byref(nbytes)))
    ws = torch.zeros(nbytes.value // 4, device="cuda", dtype=torch.float32)
    y1 = torch.empty_like(x0)
    dl = torch.empty(B, device="cuda")
    nfe = torch.empty(B, device="cuda", dtype=torch.int32)
    st = torch.empty(B, device="cuda", dtype=torch.int32)
    _lib.check(h.lib.ecnf_integrate_ws(h._h, ctypes.byref(o), _ptr(x0), _ptr(feat), _ptr(eps), _ptr(y1), _ptr(dl),
                                       _ptr(nfe), _ptr(st), B, _ptr(ws), nbytes.value, _stream(h.device)))
    torch.cuda.synchronize()
    stride = (2 * ND + 10 + 3) // 4 * 4
    S = ws[:B * stride].reshape(B, stride).cpu().numpy()
    sc = S[:, 2 * ND:]
    tau, dt = sc[:, 2], sc[:, 3]
    ints = sc.view(np.int32)
    nfe1, steps1, active = ints[:, 6], ints[:, 7], ints[:, 9]
    final = nfe.cpu().numpy()
    tau0, tau1 = -1.0, 0.0   # reverse time: tau = -t from -1 to 0
    rem_true = (final - nfe1).astype(np.float64)
    act = np.nonzero(active)[0]
    keys = {
        "remaining_over_dt": (tau1 - tau) / dt,
        "nfe_rate_extrapolated": nfe1 * (tau1 - tau) / np.maximum(tau - tau0, 1e-12),
        "true_remaining": rem_true,
    }
    chunk_evals = float(np.max(nfe1))   # the first launch (2 rounds at B = 512) ~ 2 x its per-molecule evaluations
    out = {"chunk1_nfe_max": int(nfe1.max()), "chunk1_steps": int(steps1.max()), "unfinished": int(len(act)),
           "final_nfe_max": int(final.max())}
    for name, k in keys.items():
        order = act[np.lexsort((act, -k[act]))]
        r = np.corrcoef(np.argsort(np.argsort(-k[act])), np.argsort(np.argsort(-rem_true[act])))[0, 1]
        out[name] = {"spearman_vs_true": round(float(r), 3), "makespan_evals": round(makespan(rem_true, order), 1)}
    out["batch_order_makespan_evals"] = round(makespan(rem_true, act), 1)
    print(json.dumps(out), flush=True)
    h.close()


if __name__ == "__main__":
    main()
