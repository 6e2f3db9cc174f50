"""Generate tests/golden/golden_v1.npz: inputs and fp64 oracle outputs for small cases of every config.

The reference cannot run in this container (JAX absent) and ships no golden vectors, so these
fixtures are the oracle's fp64 outputs (and, for the log-densities, its fp32 outputs: the fp32-class bound of
tests/tolerance.py) (pinned by the KATs in tests/test_oracle.py).  They let the GPU parity tests
check the kernels without re-running the slow oracle, and let the CPU suite detect oracle drift.

Params are NOT stored (LJ13 is 2 MB): they are regenerated from (config, seed) by oracle.init_params +
stress_params (numpy PCG64, deterministic); a float64 checksum of the flat blob is stored to catch generator drift.

ALDP log-prob inputs are real frames of the reference's data fixture (tests/golden/aldp_frames.npy, extracted
from ecnf/targets/data/aldp_500K_train_mini.h5 by extract_aldp_frames.py), zero-CoM centred as
setup_training.py:91-94 does.

Usage: python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import ecnf_oracle as O  # noqa: E402

OUT = os.path.join(HERE, "golden_v1.npz")
CASES = ("dw4", "lj13", "aldp", "qm9")


def params_for(name):
    oc = O.CONFIGS[name]
    return oc, O.stress_params(O.init_params(oc, 0), oc)


def main():
    out = {}
    for name in CASES:
        oc, p = params_for(name)
        B = 3
        rng = np.random.default_rng(100 + CASES.index(name))
        z = rng.standard_normal((B, oc.n_nodes * oc.dim)).astype(np.float32)
        if name == "aldp":
            frames = np.load(os.path.join(HERE, "aldp_frames.npy"))[:B].astype(np.float32)
            frames = frames - frames.mean(axis=1, keepdims=True)
            x0 = frames.reshape(B, -1)
            feat = np.tile(np.arange(oc.n_nodes, dtype=np.int32), (B, 1))   # data.py:146 features = arange(22)
        else:
            x0 = O.base_sample(z, oc)
            feat = np.zeros((B, oc.n_nodes), np.int32)
        t = np.array([0.0, 0.4, 1.0], np.float32)
        u = rng.standard_normal((B, 2, oc.n_nodes * oc.dim)).astype(np.float32)
        pre = f"{name}/"
        out[pre + "param_checksum"] = np.array(O.flatten_params(p, oc).astype(np.float64).sum())
        out[pre + "z"], out[pre + "x0"], out[pre + "feat"], out[pre + "t"], out[pre + "u"] = z, x0, feat, t, u
        out[pre + "v"] = O.egnn_vector_field(p, oc, x0, t, feat, dtype=np.float64)
        if name != "qm9":
            out[pre + "v_jvp"], out[pre + "ju"] = O.egnn_vector_field(p, oc, x0, t, feat, tangents=u, dtype=np.float64)
        out[pre + "euler10_x1"], _ = O.sample_cnf(p, oc, x0, feat, solver="euler", dt0=0.1, dtype=np.float64)
        if name in ("dw4", "lj13"):
            out[pre + "dopri_x1"], _ = O.sample_cnf(p, oc, x0, feat, solver="dopri5", dt0=0.1, dtype=np.float64)
            x1, lq, _ = O.sample_and_log_prob(p, oc, x0, feat, eps=z, approx=True, solver="dopri5", dt0=0.1,
                                              dtype=np.float64)
            out[pre + "hutch_x1"], out[pre + "hutch_logq"] = x1, lq
            x1, lq, _ = O.sample_and_log_prob(p, oc, x0, feat, eps=z, approx=True, solver="dopri5", dt0=0.1,
                                              dtype=np.float32)
            out[pre + "hutch_x1_f32"], out[pre + "hutch_logq_f32"] = x1, lq
        if name == "aldp":
            eps = rng.standard_normal(x0.shape).astype(np.float32)
            out[pre + "eps"] = eps
            lp, lp0, dl, _, xb = O.get_log_prob(p, oc, x0, feat, eps=eps, approx=True, solver="dopri5", dt0=0.1,
                                               dtype=np.float64)
            out[pre + "logp_hutch"], out[pre + "logp_hutch_dl"], out[pre + "logp_hutch_x0"] = lp, dl, xb
            lp, lp0, dl, _, xb = O.get_log_prob(p, oc, x0, feat, eps=eps, approx=True, solver="dopri5", dt0=0.1,
                                               dtype=np.float32)
            out[pre + "logp_hutch_f32"], out[pre + "logp_hutch_dl_f32"] = lp, dl
        if name == "dw4":
            lp, lp0, dl, _, xb = O.get_log_prob(p, oc, x0, feat, approx=False, solver="dopri5", dt0=0.1,
                                               dtype=np.float64)
            out[pre + "logp_exact"], out[pre + "logp_exact_dl"], out[pre + "logp_exact_x0"] = lp, dl, xb
            lp, lp0, dl, _, xb = O.get_log_prob(p, oc, x0, feat, approx=False, solver="dopri5", dt0=0.1,
                                               dtype=np.float32)
            out[pre + "logp_exact_f32"], out[pre + "logp_exact_dl_f32"] = lp, dl
    np.savez_compressed(OUT, **out)
    print(OUT, os.path.getsize(OUT), "bytes,", len(out), "arrays")


if __name__ == "__main__":
    main()
