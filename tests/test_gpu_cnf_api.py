"""The reference-named surface (ecnf_amd.cnf, mirroring ecnf/cnf/core.py:7-49, build_cnf.py:34-102 and
sample_and_log_prob.py:11-149) end to end on the GPU: build_cnf -> init / a flax-path .npz loaded through dataio ->
apply / sample_cnf / get_log_prob / sample_and_log_prob_cnf, against the fp64 golden fixtures (tolerances as in
test_gpu_parity.py: eval 2e-5 relative, trajectories 1e-4, log-densities fp32-class against the fixtures' fp64 and
fp32 oracle values, tests/tolerance.py)."""
import os

import numpy as np
import pytest
import torch

from oracle import ecnf_oracle as O
from tolerance import fp32_class

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs a ROCm GPU", allow_module_level=True)

from ecnf_amd import cnf as C  # noqa: E402
from ecnf_amd import dataio  # noqa: E402
from ecnf_amd import CONFIGS  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
G = np.load(os.path.join(HERE, "golden", "golden_v1.npz"))


def _build(name):
    c = CONFIGS[name]
    return C.build_cnf(n_frames=c.n_nodes, dim=c.dim, sigma_min=c.sigma_min, base_scale=c.base_scale,
                       n_blocks_egnn=c.n_blocks, mlp_units=(c.mlp_width,) * c.mlp_depth,
                       n_invariant_feat_hidden=c.hidden, time_embedding_dim=c.time_embedding_dim,
                       n_features=c.n_features, device=0)


def _params_via_npz(name, tmp_path):
    """The fixture weights written as a flax-path .npz and read back through dataio (row f4)."""
    oc = O.CONFIGS[name]
    p = O.stress_params(O.init_params(oc, 0), oc)
    path = tmp_path / f"{name}.npz"
    dataio.save_params_npz(path, p, CONFIGS[name])
    q = dataio.load_params_npz(path, CONFIGS[name])
    assert abs(float(O.flatten_params(q, oc).astype(np.float64).sum()) - float(G[name + "/param_checksum"])) < 1e-6
    return q


def _err(a, b):
    a = a.detach().cpu().numpy() if torch.is_tensor(a) else np.asarray(a)
    return float(np.abs(a - b).max())


@pytest.mark.parametrize("name", ["dw4", "lj13", "aldp", "qm9"])
def test_apply_and_sample_cnf(name, tmp_path):
    cnf = _build(name)
    params = _params_via_npz(name, tmp_path)
    pre = name + "/"
    v = cnf.apply(params, G[pre + "x0"], G[pre + "t"], G[pre + "feat"])
    assert _err(v, G[pre + "v"]) <= 2e-5 * max(1.0, np.abs(G[pre + "v"]).max())
    x1 = C.sample_cnf(cnf, params, None, features=G[pre + "feat"], use_fixed_step_size=True, step_size=0.1,
                      x0=G[pre + "x0"], solver="euler")
    assert _err(x1, G[pre + "euler10_x1"]) <= 1e-4 * max(1.0, np.abs(G[pre + "euler10_x1"]).max())
    if pre + "dopri_x1" in G:
        x1 = C.sample_cnf(cnf, params, None, features=G[pre + "feat"], use_fixed_step_size=True, step_size=0.1,
                          x0=G[pre + "x0"])
        assert _err(x1, G[pre + "dopri_x1"]) <= 1e-4
        # one molecule, features [N] (the reference's per-molecule call): a flat [N*D] result
        x1_0 = C.sample_cnf(cnf, params, None, features=G[pre + "feat"][0], use_fixed_step_size=True,
                            step_size=0.1, x0=G[pre + "x0"][0])
        assert x1_0.shape == (CONFIGS[name].event_dim,) and _err(x1_0, G[pre + "dopri_x1"][0]) <= 1e-4


@pytest.mark.parametrize("name", ["dw4", "lj13"])
def test_sample_and_log_prob_cnf(name, tmp_path):
    cnf = _build(name)
    params = _params_via_npz(name, tmp_path)
    pre = name + "/"
    x1, log_q = C.sample_and_log_prob_cnf(cnf, params, None, features=G[pre + "feat"], approx=True,
                                          use_fixed_step_size=True, step_size=0.1, z=G[pre + "z"])
    fp32_class(f"{name} hutch x1", x1, G[pre + "hutch_x1"], G[pre + "hutch_x1_f32"])
    fp32_class(f"{name} hutch log_q", log_q, G[pre + "hutch_logq"], G[pre + "hutch_logq_f32"])


def test_get_log_prob_hutchinson_aldp(tmp_path):
    cnf = _build("aldp")
    params = _params_via_npz("aldp", tmp_path)
    lp, lp0, dl = C.get_log_prob(cnf, params, G["aldp/x0"], None, features=G["aldp/feat"], approx=True,
                                 use_fixed_step_size=True, step_size=0.1, eps=G["aldp/eps"])
    fp32_class("aldp hutch log_p", lp, G["aldp/logp_hutch"], G["aldp/logp_hutch_f32"])
    fp32_class("aldp hutch dl", dl, G["aldp/logp_hutch_dl"], G["aldp/logp_hutch_dl_f32"])
    assert _err(lp - dl - lp0, 0.0) <= 1e-4


def test_get_log_prob_exact_dw4(tmp_path):
    cnf = _build("dw4")
    params = _params_via_npz("dw4", tmp_path)
    lp, lp0, dl = C.get_log_prob(cnf, params, G["dw4/x0"], None, features=G["dw4/feat"], approx=False,
                                 use_fixed_step_size=True, step_size=0.1)
    fp32_class("dw4 exact log_p", lp, G["dw4/logp_exact"], G["dw4/logp_exact_f32"])
    fp32_class("dw4 exact dl", dl, G["dw4/logp_exact_dl"], G["dw4/logp_exact_dl_f32"])


def test_base_and_ot_path():
    cnf = _build("lj13")
    x, lp = cnf.sample_and_log_prob_base(3, (4,))
    assert x.shape == (4, 39) and lp.shape == (4,)
    xr = x.reshape(4, 13, 3)
    assert float(xr.mean(1).abs().max()) <= 1e-6                        # zero CoM
    oc = O.CONFIGS["lj13"]
    assert _err(lp, O.base_log_prob(x.cpu().numpy(), oc)) <= 1e-4
    x1 = torch.randn(4, 39, device="cuda")
    t = torch.rand(4, device="cuda")
    xt, ut = cnf.get_x_t_and_conditional_u_t(x, x1, t)
    xt_r, ut_r = O.ot_conditional_vf(x.cpu().numpy(), x1.cpu().numpy(), t.cpu().numpy(), oc.sigma_min)
    assert _err(xt, xt_r) <= 1e-6 and _err(ut, ut_r) <= 1e-6


def test_params_updated_in_place_are_not_stale():
    """The handle cache is keyed by the CONTENT of the params (id(params) served stale weights)."""
    cnf = _build("lj13")
    oc = O.CONFIGS["lj13"]
    params = O.stress_params(O.init_params(oc, 0), oc)
    pre = "lj13/"
    v1 = cnf.apply(params, G[pre + "x0"], G[pre + "t"], G[pre + "feat"])
    params["EGNN_0/2/Dense_0/kernel"] *= 2.0                         # in place, same dict object
    v2 = cnf.apply(params, G[pre + "x0"], G[pre + "t"], G[pre + "feat"])
    ref2 = O.egnn_vector_field(params, oc, G[pre + "x0"], G[pre + "t"], G[pre + "feat"], dtype=np.float64)
    assert _err(v2, ref2) <= 2e-5 * max(1.0, np.abs(ref2).max())
    assert _err(v1, ref2) > 1e-3
    h = cnf.to_device(params)                                        # explicit handle: no per-call hashing
    assert cnf.to_device(dict(params)) is h
    v3 = cnf.apply(h, G[pre + "x0"], G[pre + "t"], G[pre + "feat"])
    assert torch.equal(v3, v2)


def test_mutated_cached_handle_is_evicted():
    """the content-hash cache must not serve a handle whose weights were changed after it was cached:
    apply(p0) after to_device(p0).update_params(p1) still uses p0's weights (and precision changes evict too)."""
    cnf = _build("lj13")
    oc = O.CONFIGS["lj13"]
    p0 = O.stress_params(O.init_params(oc, 0), oc)
    p1 = O.stress_params(O.init_params(oc, 1), oc)
    pre = "lj13/"
    args = (G[pre + "x0"], G[pre + "t"], G[pre + "feat"])
    v0 = cnf.apply(p0, *args)
    h = cnf.to_device(p0)
    h.update_params(p1)
    v1 = cnf.apply(h, *args)
    ref1 = O.egnn_vector_field(p1, oc, *args, dtype=np.float64)
    assert _err(v1, ref1) <= 2e-5 * max(1.0, np.abs(ref1).max())
    v0b = cnf.apply(p0, *args)                       # a fresh upload of p0, not the mutated handle
    assert torch.equal(v0b, v0)
    h2 = cnf.to_device(p0)
    assert h2 is not h
    h2.set_precision("fp32")
    assert cnf.to_device(p0) is not h2 and cnf.to_device(p0).precision == "split_f16"
