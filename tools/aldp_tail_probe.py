"""Diagnostic: ALDP B = 512 PID Hutchinson log_prob (BASELINE configs[2], t = 1 -> 0 on real frames) through the
re-dealt solve with and without its tail teams (ecnf_hip.hip redeal_kernel, kTailG), and the one-launch solve
(no workspace): kernel time (HIP events, median of 5) and bitwise equality of y(0), the divergence integral, NFE and
status with the one-launch solve.  Usage: python tools/aldp_tail_probe.py [B]"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ecnf-baseline-neurips-2023_amd"))

import torch  # noqa: E402
from ecnf_amd import CONFIGS, init_params, _lib  # noqa: E402
from ecnf_amd.engine import EcnfHandle, SolveOptions, _ptr, _stream  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
cfg = CONFIGS["aldp"]
h = EcnfHandle(cfg, init_params(cfg, 0), 0)
if os.environ.get("TP_INPUT", "frames") == "frames":   # real frames of the reference's data file
    fr = np.load(os.path.join(ROOT, "tests", "golden", "aldp_frames.npy")).reshape(-1, cfg.event_dim)
    x = torch.tensor(fr[np.arange(B) % fr.shape[0]], device="cuda")
    x = x - x.reshape(B, cfg.n_nodes, 3).mean(1, keepdim=True).repeat(1, cfg.n_nodes, 1).reshape(B, -1)
    eps = torch.randn((B, cfg.event_dim), generator=torch.Generator("cuda").manual_seed(4321), device="cuda")
else:   # base draws, as tools/bench_paths.py's ALDP log_prob case (the per-config profiles)
    gb = torch.Generator("cuda").manual_seed(1234)
    x = h.base_sample(torch.randn((B, cfg.event_dim), device="cuda", generator=gb))
    eps = torch.randn((B, cfg.event_dim), device="cuda", generator=gb)
feat = torch.arange(cfg.n_nodes, device="cuda", dtype=torch.int32).expand(B, -1).contiguous()
o = SolveOptions("dopri5", None).to_c(1.0, 0.0, _lib.DIV_HUTCHINSON)


def solve(workspace):
    nb = ctypes.c_size_t(0)
    _lib.check(h.lib.ecnf_integrate_workspace_size(h._h, ctypes.byref(o), B, ctypes.byref(nb)))
    ws = torch.empty(nb.value, device="cuda", dtype=torch.uint8) if workspace else None
    y = torch.empty_like(x)
    dl = torch.empty(B, device="cuda")
    nfe = torch.empty(B, device="cuda", dtype=torch.int32)
    st = torch.empty(B, device="cuda", dtype=torch.int32)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    _lib.check(h.lib.ecnf_integrate_ws(h._h, ctypes.byref(o), _ptr(x), _ptr(feat), _ptr(eps), _ptr(y), _ptr(dl),
                                       _ptr(nfe), _ptr(st), B, _ptr(ws), nb.value if workspace else 0,
                                       _stream(h.device)))
    b.record()
    torch.cuda.synchronize()
    global last_ws
    last_ws = ws
    return a.elapsed_time(b), (y, dl, nfe, st)


last_ws = None


def redeal_info(nfe):
    """the re-deal scratch of the last solve (ecnf_hip.hip sched_floats: [B][stride] states, order, nslots, nteam)"""
    ND = cfg.event_dim
    stride = (2 * ND + 10 + 3) & ~3
    f = last_ws.view(torch.float32)
    i = last_ws.view(torch.int32)
    st = f[:B * stride].reshape(B, stride)
    tau, dt, active = st[:, 2 * ND + 2], st[:, 2 * ND + 3], st[:, 2 * ND + 9].view(torch.int32)
    key = torch.where(active != 0, (0.0 - tau) / dt, torch.full_like(tau, -1.0))
    if os.environ.get("TP_DUMP"):   # per molecule: re-deal key, NFE at the first launch's end, final NFE
        np.savez(os.environ["TP_DUMP"], key=key.cpu().numpy(), nfe1=st[:, 2 * ND + 6].view(torch.int32).cpu().numpy(),
                 steps1=st[:, 2 * ND + 7].view(torch.int32).cpu().numpy(), nfe=nfe.cpu().numpy())
    o0 = B * stride
    order = i[o0:o0 + B]
    nb = o0 + ((B + 3) & ~3)
    nslots, nteam = int(i[nb]), int(i[nb + 1])
    nfe_c = nfe.cpu().numpy()
    rank_true = np.argsort(-nfe_c)
    ordv = order[:nslots].cpu().numpy()
    pos = {int(m): k for k, m in enumerate(ordv)}
    return {"nslots": nslots, "nteam": nteam,
            "slowest": [{"mol": int(m), "nfe": int(nfe_c[m]), "slot": pos.get(int(m), -1),
                         "key": float(key[m])} for m in rank_true[:12]],
            "key_top": [round(float(v), 1) for v in torch.sort(key, descending=True).values[:12].cpu()],
            "key_sum": float(key.clamp(min=0).sum())}


res = {}
ref = None
for tag, mode, ws in (("one_launch", 0, False), ("redeal_no_tail", 1, True), ("redeal_tail", 0, True)):
    h.set_team(mode)
    solve(ws)
    ts, out = [], None
    for _ in range(5):
        t, out = solve(ws)
        ts.append(t)
    ref = out if ref is None else ref
    res[tag] = {"ms": sorted(ts)[2], "all_ms": [round(t, 2) for t in ts],
                "bitwise_vs_one_launch": all(bool(torch.equal(p, q)) for p, q in zip(out, ref)),
                "nfe_max": int(out[2].max()), "status_ok": int(out[3].abs().sum()) == 0}
    if ws:
        res[tag]["redeal"] = redeal_info(out[2])
    print(tag, json.dumps(res[tag]), flush=True)
h.set_team(0)
print(json.dumps({"B": B, **res}))
