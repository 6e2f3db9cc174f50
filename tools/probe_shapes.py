import sys, numpy as np, torch
sys.path.insert(0, "ecnf-baseline-neurips-2023_amd")
from ecnf_amd import cnf as C
for N in (34, 48, 64):
    for units, H in (((64, 64), 32), ((128, 128, 128), 64), ((256,) * 4, 128)):
        cnf = C.build_cnf(n_frames=N, dim=3, sigma_min=0.01, base_scale=1.0, n_blocks_egnn=2, mlp_units=units,
                          n_invariant_feat_hidden=H, time_embedding_dim=8, n_features=2, device=0)
        p = cnf.init(0)
        x0 = np.random.default_rng(0).standard_normal((2, N * 3)).astype(np.float32)
        x0 = (x0.reshape(2, N, 3) - x0.reshape(2, N, 3).mean(1, keepdims=True)).reshape(2, -1)
        f = np.zeros((2, N), np.int32)
        res = []
        for name, fn in (("field", lambda: cnf.apply(p, x0, np.zeros(2, np.float32), f)),
                         ("hutch", lambda: C.get_log_prob(cnf, p, x0, None, features=f, approx=True, use_fixed_step_size=True, step_size=0.5, solver="euler", eps=x0)),
                         ("exact", lambda: C.get_log_prob(cnf, p, x0, None, features=f, approx=False, use_fixed_step_size=True, step_size=0.5, solver="euler"))):
            try:
                fn(); res.append(name + ":ok")
            except Exception as e:
                res.append(name + ":" + str(e)[:70])
        print(N, units[0], len(units), H, res, flush=True)
