"""CPU tests of running any mlp_units / hidden width on the compiled kernel shapes (ecnf_amd.params.kernel_config,
pad_params): the zero-padded network computes the SAME function as the reference-shaped one (checked bitwise in the
fp64 oracle, field and JVP, to fp64 rounding), the reference tree matches the oracle's param_spec for unequal widths, and shapes without
a compiled kernel are refused."""
import numpy as np
import pytest

from ecnf_amd import params as P
from oracle import ecnf_oracle as O


@pytest.mark.parametrize("n,units,H,T,K", [(5, (16, 16), 32, 10, 2), (7, (48, 80), 40, 8, 2), (4, (30, 60, 100), 20, 6, 3),
                                           (6, (200, 256, 120, 90), 36, 8, 2)])
def test_padded_network_is_the_same_function(n, units, H, T, K):
    oc = O.CNFConfig(n_nodes=n, dim=3, n_features=2, hidden=H, time_embedding_dim=T, mlp_units=units, n_blocks=K)
    assert P.ref_param_spec(2, H, T, units, K) == O.param_spec(oc)
    kc = P.kernel_config(n, 3, 2, H, T, units, K)
    assert kc.mlp_width >= max(units) and kc.hidden % 32 == 0 and kc.hidden >= H
    assert (kc.mlp_width, kc.mlp_depth, 3) in P.COMPILED_SHAPES
    p = O.stress_params(O.init_params(oc, 0), oc)
    pp = P.pad_params(p, H, T, units, kc)
    assert P.flatten_params(pp, kc).size == P.param_count(kc)
    okc = O.CNFConfig(n_nodes=n, dim=3, n_features=2, hidden=kc.hidden, time_embedding_dim=T, mlp_width=kc.mlp_width,
                      mlp_depth=kc.mlp_depth, n_blocks=K)
    rng = np.random.default_rng(1)
    x = rng.standard_normal((3, 3 * n)).astype(np.float32)
    t = np.array([0.0, 0.5, 1.0], np.float32)
    f = rng.integers(0, 2, (3, n))
    u = rng.standard_normal((3, 2, 3 * n)).astype(np.float32)
    v1, j1 = O.egnn_vector_field(p, oc, x, t, f, tangents=u)
    v2, j2 = O.egnn_vector_field(pp, okc, x, t, f, tangents=u)
    # the padded terms are exact zeros; only the BLAS blocking of the longer fp64 dot products may differ
    np.testing.assert_allclose(v2, v1, rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(j2, j1, rtol=1e-12, atol=1e-14)


def test_unsupported_shapes_are_refused():
    with pytest.raises(ValueError):
        P.kernel_config(5, 3, 1, 32, 8, (300, 16), 2)       # wider than every compiled kernel
    with pytest.raises(ValueError):
        P.kernel_config(5, 3, 1, 32, 8, (16,), 2)           # depth 1 is not compiled
    with pytest.raises(ValueError):
        P.kernel_config(5, 2, 1, 32, 8, (64, 64, 64, 64), 2)   # depth 4 is compiled for dim 3 only
    with pytest.raises(ValueError):
        oc = O.CNFConfig(n_nodes=5, dim=3, hidden=32, mlp_units=(16, 16), n_blocks=2)
        p = O.init_params(oc, 0)
        del p["EGNN_0/0/phi_e/Dense_1/kernel"]
        P.pad_params(p, 32, 8, (16, 16), P.kernel_config(5, 3, 1, 32, 8, (16, 16), 2))


def test_padded_config_entry_points_take_reference_params(tmp_path):
    """a padded kernel config carries the reference widths (ref_mlp_units / ref_hidden), so every entry
    point that flattens params (EcnfHandle, update_params, the Trainer, dataio) takes reference-shaped params, and
    crop_params / unflatten_params(reference_shapes=True) give them back."""
    from ecnf_amd import dataio
    units, H, T, K, n = (48, 80), 40, 8, 2, 7
    oc = O.CNFConfig(n_nodes=n, dim=3, n_features=2, hidden=H, time_embedding_dim=T, mlp_units=units, n_blocks=K)
    kc = P.kernel_config(n, 3, 2, H, T, units, K)
    assert kc.ref_mlp_units == units and kc.ref_hidden == H
    assert P.kernel_config(5, 3, 1, 64, 8, (128, 128, 128), 3).ref_mlp_units == ()   # unpadded: no reference widths
    p = O.stress_params(O.init_params(oc, 0), oc)
    blob = P.flatten_params(p, kc)
    assert np.array_equal(blob, P.flatten_params(P.pad_params(p, H, T, units, kc), kc))
    back = P.unflatten_params(blob, kc, reference_shapes=True)
    assert set(back) == set(p) and all(np.array_equal(back[k], p[k]) for k in p)
    f = tmp_path / "w.npz"
    dataio.save_params_npz(f, P.pad_params(p, H, T, units, kc), kc)
    loaded = dataio.load_params_npz(f, kc)
    assert all(loaded[k].shape == np.asarray(p[k]).shape and np.array_equal(loaded[k], p[k]) for k in p)
