"""GPU parity of the target densities and eval reductions through the C-ABI,
against the oracle restatements of leonard_jones.py:10-27, double_well.py:9-19, evaluation.py:10-22 and
setup_training.py:182.

Tolerances: log p |err| <= 1e-5 x max(1, |ref|) (fp32 pair sums vs fp64); ESS |err| <= 1e-5 relative."""
import numpy as np
import pytest
import torch

from oracle import ecnf_oracle as O

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs a ROCm GPU", allow_module_level=True)

from ecnf_amd import targets as T  # noqa: E402
from ecnf_amd import distributed as D  # noqa: E402


def _cfgs(rng, B, N, D_, scale):
    x = (rng.standard_normal((B, N, D_)) * scale).astype(np.float32)
    x[0, 1] = x[0, 0]          # coincident atoms: safe_norm returns 1
    return x


@pytest.mark.parametrize("kw", [{}, {"epsilon": 2.0, "tau": 0.5, "r": 1.1, "harmonic_potential_coef": 0.25}])
def test_lj13_log_prob(kw):
    rng = np.random.default_rng(0)
    x = _cfgs(rng, 513, 13, 3, 1.2)
    got = T.lj_log_prob(torch.from_numpy(x).cuda().reshape(513, -1), 13, 3, **kw).cpu().numpy()
    ref = -O.lj_energy(x, 13, 3, **kw)
    err = np.abs(got - ref) / np.maximum(1.0, np.abs(ref))
    assert err.max() <= 1e-5, err.max()


@pytest.mark.parametrize("kw", [{}, {"temperature": 2.0, "a": 0.1, "b": -3.0, "c": 1.0, "d0": 3.5}])
def test_dw4_log_prob(kw):
    rng = np.random.default_rng(1)
    x = _cfgs(rng, 300, 4, 2, 2.0)
    got = T.dw_log_prob(torch.from_numpy(x).cuda(), 4, 2, **kw).cpu().numpy()
    okw = dict(kw)
    if "temperature" in okw:
        okw["tau"] = okw.pop("temperature")
    ref = -O.dw_energy(x, 4, 2, **okw)
    err = np.abs(got - ref) / np.maximum(1.0, np.abs(ref))
    assert err.max() <= 1e-5, err.max()


@pytest.mark.parametrize("n", [1, 37, 65536])
def test_ess_from_device_partials(n):
    rng = np.random.default_rng(n)
    lw = (rng.standard_normal(n) * 3.0).astype(np.float32)
    mask = (rng.random(n) > 0.2).astype(np.float32)
    mask[0] = 1.0
    fwd, rev = D.ess_from_device(torch.from_numpy(lw).cuda(), torch.from_numpy(mask).cuda())
    assert abs(float(fwd) - O.forward_ess(lw, mask)) <= 1e-5 * max(1e-3, O.forward_ess(lw, mask)) + 1e-7
    # reverse ESS over the unmasked entries (the device reduction skips masked ones)
    assert abs(float(rev) - O.reverse_ess(lw[mask > 0])) <= 1e-5 * O.reverse_ess(lw[mask > 0]) + 1e-7


def test_lse_partials_contract_and_errors():
    v = torch.tensor([0.5, -2.0, 3.0], device="cuda")
    p = T.lse_partials(v).cpu().numpy()
    assert p[0] == 3.0 and p[2] == 2.0 and p[4] == 6.0 and p[6] == 3.0
    np.testing.assert_allclose(p[1], np.exp([0.5 - 3, -2 - 3, 0]).sum(), rtol=1e-6)
    empty = T.lse_partials(torch.zeros(0, device="cuda")).cpu().numpy()
    assert np.isneginf(empty[0]) and empty[1] == 0.0 and empty[6] == 0.0
    with pytest.raises(ValueError):
        T.lj_log_prob(torch.zeros(3, 39), 13, 3)      # host tensor


def test_lj13_per_node_r():
    """leonard_jones.py:10-20 with the array form of r: pair (receiver i, sender j) uses r[i]."""
    rng = np.random.default_rng(5)
    x = _cfgs(rng, 257, 13, 3, 1.2)
    r = (1.0 + 0.1 * rng.standard_normal(13)).astype(np.float32)
    got = T.lj_log_prob(torch.from_numpy(x).cuda().reshape(257, -1), 13, 3, r=torch.from_numpy(r).cuda()).cpu().numpy()
    ref = -O.lj_energy(x, 13, 3, r=r)
    err = np.abs(got - ref) / np.maximum(1.0, np.abs(ref))
    assert err.max() <= 1e-5, err.max()
    with pytest.raises(ValueError):
        T.lj_log_prob(torch.from_numpy(x).cuda(), 13, 3, r=torch.ones(12, device="cuda"))
    # scalar r given as a numpy scalar or a 0-d tensor: the scalar form, not a per-node array
    xd = torch.from_numpy(x).cuda().reshape(257, -1)
    ref = T.lj_log_prob(xd, 13, 3, r=1.1)
    for r0 in (np.float32(1.1), np.array(1.1, np.float32), torch.tensor(1.1), torch.tensor(1.1, device="cuda")):
        assert torch.equal(T.lj_log_prob(xd, 13, 3, r=r0), ref), type(r0)


@pytest.mark.parametrize("n", [5, 3000])
def test_ess_with_infinite_log_weights(n):
    """-inf log_w (a target energy that overflowed to +inf) has zero weight in the log-sum-exps, as
    jax.nn.logsumexp gives it: no NaN in either ESS (lse_push started from -inf)."""
    rng = np.random.default_rng(n)
    lw = (rng.standard_normal(n) * 2.0).astype(np.float32)
    lw[[0, n // 2, n - 1]] = -np.inf
    fwd, rev = D.ess_from_device(torch.from_numpy(lw).cuda())
    rev_ref, fwd_ref = O.reverse_ess(lw), O.forward_ess(lw)
    assert np.isfinite(float(rev)) and abs(float(rev) - rev_ref) <= 1e-5 * rev_ref
    assert float(fwd) == fwd_ref == 0.0                     # LSE(-log_w) = +inf
    p = T.lse_partials(torch.from_numpy(lw).cuda()).cpu().numpy()
    assert np.isfinite(p[:2]).all() and np.isposinf(p[2]) and p[3] == 3.0 and p[6] == n
    # an all -inf input: an empty log-sum-exp, not NaN
    q = T.lse_partials(torch.full((7,), -np.inf, device="cuda")).cpu().numpy()
    assert np.isneginf(q[0]) and q[1] == 0.0 and np.isposinf(q[2]) and q[3] == 7.0
