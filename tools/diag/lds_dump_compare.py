"""Compare two LDS images of tools/diag/lds_dump_run.py (flat vs ds form) region by region (the carve-up of
egnn_eval.hpp carve_lds for the padded (128, 2, 3) test network at one molecule per workgroup).
Usage: python tools/diag/lds_dump_compare.py A.npz B.npz [stage]"""
import sys

import numpy as np


def align4(n):
    return (n + 3) & ~3


def ld_node(k, vec=True):
    a = align4(k)
    return a if (a >> 2) & 1 else a + 4


def regions(N=7, D=3, H=64, T=8, M=128, L=2, MPW=1, NT=1):
    RP = 32 * ((MPW * N + 31) // 32)
    R = RP * (1 + NT)
    out, p = [], 0
    for name, size, ld in (("hin", align4(R * ld_node(H + T)), ld_node(H + T)), ("hb", align4(R * ld_node(H)), ld_node(H)),
                           ("P", align4(R * ld_node(2 * M)), ld_node(2 * M)), ("macc", align4(R * ld_node(M)), ld_node(M)),
                           ("xc", align4(R * D), D), ("dxacc", align4(R * D), D), ("mean", align4(2 * MPW * D), D),
                           ("temb", align4(MPW * T), T), ("vecs", align4((2 * L + 2) * M), M), ("feat", align4(MPW * N), N)):
        out.append((name, p, p + size, ld))
        p += size
    out.append(("solver", p, p + 13 * align4(MPW * N * D) + 32 + 12, N * D))
    return out


def main():
    a, b = np.load(sys.argv[1]), np.load(sys.argv[2])
    st = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    A, B = a["dump"][st], b["dump"][st]
    for k in ("v", "ju"):
        print(k, "max |a - ref|", float(np.abs(a[k] - (a["vr"] if k == "v" else a["jr"])).max()),
              "max |b - ref|", float(np.nan_to_num(np.abs(b[k] - (b["vr"] if k == "v" else b["jr"])), nan=-1).max()))
    for name, lo, hi, ld in regions():
        x, y = A[lo:hi], B[lo:hi]
        bad = np.nonzero(~((x == y) | (np.isnan(x) & np.isnan(y))))[0]
        if len(bad) == 0:
            print(f"{name:7s} [{lo},{hi}) identical")
            continue
        rows = sorted(set((bad // ld).tolist()))
        print(f"{name:7s} [{lo},{hi}) {len(bad)} differ; rows {rows[:20]}{'...' if len(rows) > 20 else ''}; "
              f"first {[(int(i), float(x[i]), float(y[i])) for i in bad[:4]]}")


if __name__ == "__main__":
    main()
