"""CPU tests of the weights / dataset I/O (ecnf_amd.dataio; reference ecnf/targets/data.py:14-154)."""
import os

import numpy as np
import pytest

from ecnf_amd import CONFIGS, flatten_params, init_params, param_spec
from ecnf_amd import dataio as io

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.mark.parametrize("name", ["dw4", "lj13", "aldp", "qm9"])
def test_params_npz_round_trip(tmp_path, name):
    cfg = CONFIGS[name]
    p = init_params(cfg, 3)
    f = tmp_path / "w.npz"
    io.save_params_npz(f, p, cfg)
    q = io.load_params_npz(f, cfg)
    assert sorted(q) == sorted(path for path, _ in param_spec(cfg))
    np.testing.assert_array_equal(flatten_params(q, cfg), flatten_params(p, cfg))


def test_params_npz_nested_tree_and_errors(tmp_path):
    cfg = CONFIGS["dw4"]
    p = init_params(cfg, 0)
    nested: dict = {}
    for path, a in p.items():
        d = nested
        parts = path.split("/")
        for k in parts[:-1]:
            d = d.setdefault(k, {})
        d[parts[-1]] = a
    f = tmp_path / "w.npz"
    io.save_params_npz(f, {"params": nested}, cfg)
    np.testing.assert_array_equal(flatten_params(io.load_params_npz(f, cfg), cfg), flatten_params(p, cfg))
    # a missing key, an extra key and a wrong shape are all refused
    bad = dict(p)
    bad.pop("EGNN_0/final_scaling")
    np.savez(tmp_path / "missing.npz", **bad)
    with pytest.raises(ValueError, match="missing"):
        io.load_params_npz(tmp_path / "missing.npz", cfg)
    np.savez(tmp_path / "extra.npz", **p, **{"EGNN_0/bogus": np.zeros(3, np.float32)})
    with pytest.raises(ValueError, match="unexpected"):
        io.load_params_npz(tmp_path / "extra.npz", cfg)
    wrong = dict(p)
    wrong["Embed_0/embedding"] = np.zeros((2, 2), np.float32)
    np.savez(tmp_path / "shape.npz", **wrong)
    with pytest.raises(ValueError, match="shape"):
        io.load_params_npz(tmp_path / "shape.npz", cfg)


def test_lj13_dw4_qm9_loaders_follow_reference_splits(tmp_path):
    rng = np.random.default_rng(0)
    # LJ13 (data.py:58-92): holdout[idx[:n]], val = all[1000:2000], test = all[:1000]
    holdout = rng.standard_normal((50, 39)).astype(np.float32)
    idx = rng.permutation(50)
    alld = rng.standard_normal((2100, 39)).astype(np.float32)
    np.save(tmp_path / "holdout_data_LJ13.npy", holdout)
    np.save(tmp_path / "idx_LJ13.npy", idx)
    np.save(tmp_path / "all_data_LJ13.npy", alld)
    tr, va, te = io.load_lj13(20, tmp_path)
    np.testing.assert_array_equal(tr.positions, holdout[idx[:20]].reshape(-1, 13, 3))
    np.testing.assert_array_equal(va.positions, alld[1000:2000].reshape(-1, 13, 3))
    np.testing.assert_array_equal(te.positions, alld[:1000].reshape(-1, 13, 3))
    assert tr.features.shape == (20, 13, 1) and not tr.features.any()
    with pytest.raises(ValueError):
        io.load_lj13(51, tmp_path)
    # DW4 (data.py:31-56)
    d = rng.standard_normal((3500, 8)).astype(np.float32)
    np.save(tmp_path / "dw4-data.npy", d)
    tr, va, te = io.load_dw4(100, 1000, 1000, tmp_path)
    d = d.reshape(-1, 4, 2)
    np.testing.assert_array_equal(tr.positions, d[:100])
    np.testing.assert_array_equal(va.positions, d[-2000:-1000])
    np.testing.assert_array_equal(te.positions, d[-1000:])
    # QM9 (data.py:94-121): no download
    with pytest.raises(FileNotFoundError):
        io.load_qm9(path=tmp_path)
    for split, n in (("train", 7), ("valid", 3), ("test", 4)):
        np.save(tmp_path / f"qm9pos_{split}.npy", rng.standard_normal((n, 19, 3)).astype(np.float32))
    tr, va, te = io.load_qm9(5, tmp_path)
    assert tr.positions.shape == (5, 19, 3) and va.positions.shape == (3, 19, 3) and te.positions.shape == (4, 19, 3)
    # a pickled object array is refused (never unpickled)
    np.save(tmp_path / "obj.npy", np.array([d, None], dtype=object), allow_pickle=True)
    os.replace(tmp_path / "obj.npy", tmp_path / "dw4-data.npy")
    with pytest.raises(ValueError):
        io.load_dw4(path=tmp_path)


def test_aldp_frames_features():
    frames = np.load(os.path.join(GOLDEN, "aldp_frames.npy"), allow_pickle=False)
    s = io.aldp_sample(frames[:5])
    assert s.positions.shape == (5, 22, 3)
    f = io.features_for_kernel(s)
    assert f.shape == (5, 22) and f.dtype == np.int32
    np.testing.assert_array_equal(f, np.tile(np.arange(22, dtype=np.int32), (5, 1)))
    with pytest.raises(ValueError):
        io.positional_dataset_only_to_full_graph(np.zeros((3, 4)))
