"""Diagnostic (CPU, numpy): which weights' split residual biases the exact trace?  The oracle's Dense layers are
patched to use the two-piece fp16 weights (h0 + h1 of the per-matrix scaled weight, as the host packs them) in the
primal product, the tangent product, or both, and the exact trace of the LJ13 field is compared with fp64 at three
times, beside the fp32 oracle's own error.  Usage: python tools/diag/weight_split_trace.py
[config] [--groups]"""
import sys, numpy as np
sys.path[:0] = [__import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))]
from oracle import ecnf_oracle as O
name = sys.argv[1] if len(sys.argv) > 1 else "lj13"
oc = O.CONFIGS[name]
p = O.stress_params(O.init_params(oc, 0), oc)
def split2(W):
    W = W.astype(np.float64)
    s = 2.0 ** (12 - np.floor(np.log2(np.abs(W).max())))  # per-matrix scale like the host
    Ws = W * s
    h0 = Ws.astype(np.float16).astype(np.float64)
    h1 = (Ws - h0).astype(np.float16).astype(np.float64)
    return (h0 + h1) / s
MODE = {"prim": "exact", "tan": "exact"}
orig = O._dense
def dense(x, dx, params, prefix, dtype):
    W = params[prefix + "/kernel"].astype(np.float64); b = params[prefix + "/bias"].astype(np.float64)
    Wp = split2(W) if MODE["prim"] == "split" else W
    Wt = split2(W) if MODE["tan"] == "split" else W
    y = x @ Wp + b
    dy = None if dx is None else dx @ Wt
    return y, dy
B = 6
rng = np.random.default_rng(1)
N, D = oc.n_nodes, oc.dim; ND = N * D
z = rng.standard_normal((B, ND)).astype(np.float32)
x0 = O.base_sample(z, oc)
feat = rng.integers(0, oc.n_features, (B, N)).astype(np.int32)
for t0 in (1.0, 0.5, 0.1):
    t = np.full(B, t0, np.float32)
    eye = np.broadcast_to(np.eye(ND), (B, ND, ND)).copy()
    _, J64 = O.egnn_vector_field(p, oc, x0, t, feat, tangents=eye, dtype=np.float64)
    _, J32 = O.egnn_vector_field(p, oc, x0, t, feat, tangents=eye.astype(np.float32), dtype=np.float32)
    tr64 = np.einsum("bkk->b", J64); tr32 = np.einsum("bkk->b", J32.astype(np.float64))
    print(f"t={t0} fp32 oracle trace err {np.abs(tr32-tr64).max():.3e}  signed {np.mean(tr32-tr64):+.3e}")
    O._dense = dense
    for mp, mt in (("split", "split"), ("split", "exact"), ("exact", "split")):
        MODE["prim"], MODE["tan"] = mp, mt
        _, J = O.egnn_vector_field(p, oc, x0, t, feat, tangents=eye, dtype=np.float64)
        tr = np.einsum("bkk->b", J)
        print(f"   prim={mp} tan={mt}: trace err {np.abs(tr-tr64).max():.3e} signed mean {np.mean(tr-tr64):+.3e}")
    O._dense = orig

# Per layer group (round 5): the tangent kernels' chain MFMAs carry the exact 3-piece weights on the primal product (the
# fourth term w2 x0).  Dropping it on one group of chain layers = two-piece weights on that group's PRIMAL product
# only; the signed trace bias of each group alone shows whether the fourth term could be kept on a few layers.
if len(sys.argv) > 2 and sys.argv[2] == "--groups":
    import re
    blocks = sorted({k[:k.index("/phi_e/")] for k in p if "/phi_e/" in k})
    L = oc.mlp_depth
    groups = [(f"{b} phi_e 2..L", rf"^{re.escape(b)}/phi_e/Dense_[1-9]") for b in blocks] + \
             [(f"{b} phi_x torso", rf"^{re.escape(b)}/phi_x_torso/Dense_") for b in blocks]
    def dense_g(x, dx, params, prefix, dtype):
        W = params[prefix + "/kernel"].astype(np.float64); b = params[prefix + "/bias"].astype(np.float64)
        Wp = split2(W) if re.search(MODE["group"], prefix) else W
        return x @ Wp + b, None if dx is None else dx @ W
    for t0 in (1.0, 0.5, 0.1):
        t = np.full(B, t0, np.float32)
        eye = np.broadcast_to(np.eye(ND), (B, ND, ND)).copy()
        _, J64 = O.egnn_vector_field(p, oc, x0, t, feat, tangents=eye, dtype=np.float64)
        _, J32 = O.egnn_vector_field(p, oc, x0, t, feat, tangents=eye.astype(np.float32), dtype=np.float32)
        tr64 = np.einsum("bkk->b", J64)
        e32 = np.einsum("bkk->b", J32.astype(np.float64)) - tr64
        print(f"t={t0} fp32 oracle: |err| {np.abs(e32).max():.3e} signed mean {e32.mean():+.3e}")
        O._dense = dense_g
        for name_g, pat in groups + [("all chain layers", r"/(phi_e/Dense_[1-9]|phi_x_torso/Dense_)")]:
            MODE["group"] = pat
            _, J = O.egnn_vector_field(p, oc, x0, t, feat, tangents=eye, dtype=np.float64)
            e = np.einsum("bkk->b", J) - tr64
            print(f"   two-piece primal on {name_g:24s}: |err| {np.abs(e).max():.3e} signed mean {e.mean():+.3e}")
        O._dense = orig
