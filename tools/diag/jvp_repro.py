"""Diagnostic: the tangent vf_kernel (ecnf_vf_jvp) of the (128, 2, 3) shape against the fp64 oracle, per molecule, over
batch sizes, tangent counts, padded (units (48, 80), H = 40) and unpadded (units (128, 128), H = 64) networks, with
repeats to expose run-to-run differences.  Library: ECNF_LIB (default: the product).  Prints one line per case.
--poison HEX[:MODE]: before every launch, fill every VGPR / AGPR and the LDS of every SIMD with the 32-bit pattern HEX
(tools/diag/poison.hip, built as tools/diag/libpoison.so) to expose reads of never-written registers or LDS (MODE 1: LDS only, 2: registers only, 3: both, the default)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "ecnf-baseline-neurips-2023_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
from ecnf_amd import cnf as C  # noqa: E402
from oracle import ecnf_oracle as O  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
first = "--first" in sys.argv   # one launch (padded network, B = 1, one tangent), then exit: 1 if it is wrong
poison = None
if "--poison" in sys.argv:
    spec = sys.argv[sys.argv.index("--poison") + 1].split(":")
    bits, pmode = int(spec[0], 16), int(spec[1]) if len(spec) > 1 else 3
    plib = ctypes.CDLL(os.path.join(ROOT, "tools", "diag", "libpoison.so"))
    poison = lambda: plib.poison_launch(ctypes.c_uint(bits), 4096, pmode)  # noqa: E731
for units, H in (((48, 80), 40), ((128, 128), 64)):
    cnf = C.build_cnf(n_frames=7, dim=3, sigma_min=0.01, base_scale=1.0, n_blocks_egnn=2, mlp_units=units,
                      n_invariant_feat_hidden=H, time_embedding_dim=8, n_features=3, device=0)
    oc = O.CNFConfig(n_nodes=7, dim=3, n_features=3, hidden=H, time_embedding_dim=8, mlp_units=units, n_blocks=2)
    p = O.stress_params(O.init_params(oc, 1), oc)
    h = cnf.to_device(p)
    chk = getattr(h.lib, "ecnf_debug_checks", None)
    for B in (1, 2, 6):
        for ntan in (1, 2):
            rng = np.random.default_rng(3)
            x0 = O.base_sample(rng.standard_normal((B, 21)).astype(np.float32), oc)
            feat = rng.integers(0, 3, (B, 7)).astype(np.int32)
            t = np.linspace(0.0, 1.0, B).astype(np.float32)
            u = rng.standard_normal((B, ntan, 21)).astype(np.float32)
            vr, jr = O.egnn_vector_field(p, oc, x0, t, feat, tangents=u, dtype=np.float64)
            outs = []
            for r in range(1 if first else reps):
                if poison is not None:
                    torch.cuda.synchronize()
                    assert poison() == 0
                v, ju = h.jvp(torch.from_numpy(x0).cuda(), torch.from_numpy(t).cuda(), torch.from_numpy(feat).cuda(),
                              torch.from_numpy(u).cuda())
                torch.cuda.synchronize()
                outs.append((v.cpu().numpy(), ju.cpu().numpy()))
            ev = [np.abs(o[0] - vr).max(axis=1).round(7).tolist() for o in outs]
            ej = [np.nan_to_num(np.abs(o[1] - jr).reshape(B, -1).max(axis=1), nan=-1.0).round(7).tolist() for o in outs]
            same = all(np.array_equal(outs[0][1], o[1], equal_nan=True) for o in outs[1:])
            flags = ""
            if chk is not None:
                f = ctypes.c_uint32(0)
                chk(ctypes.byref(f), 1)
                flags = f" checks 0x{f.value:x}"
            print(f"units {units} B {B} ntan {ntan} repeatable {same} err_v {ev[0]} err_jvp(rep0) {ej[0]} "
                  f"err_jvp(rep1) {ej[1] if len(ej) > 1 else ''}{flags}", flush=True)
            if first:
                sys.exit(0 if max(ev[0]) < 1e-5 and 0 <= max(ej[0]) < 1e-5 else 1)
