"""Weights and dataset I/O around the sampling path.

* Weights: a flax-path ``.npz`` (keys = the ``params/...`` paths of ``params.param_spec``, e.g.
  ``EGNN_0/0/phi_e/Dense_0/kernel``) round-trips to the flat blob ``ecnf_create`` takes.  A reference checkpoint's
  ``params["params"]`` tree exported with ``flax.traverse_util.flatten_dict(..., sep="/")`` and ``np.savez`` loads
  directly.  Loading never unpickles (``allow_pickle=False``).
* Datasets: the reference's ``ecnf/targets/data.py`` loaders (``load_dw4:31-56``, ``load_lj13:58-92``,
  ``load_qm9:94-121``) restated over numpy arrays: same files, same splits, same reshapes, zero integer features
  (``positional_dataset_only_to_full_graph:23-28``).  Differences: no download (``load_qm9`` raises instead of
  fetching from figshare) and no pickled object arrays — the reference's ``dw4-dataidx.npy`` is a pickled object
  array (``np.load(..., allow_pickle=True)[0]``), so ``load_dw4`` takes the plain float array saved from it.
"""
from __future__ import annotations

import os
from typing import Mapping, NamedTuple, Optional, Tuple, Union

import numpy as np

from .params import CNFConfig, _flat_lookup, flatten_params, param_spec, unflatten_params

PathLike = Union[str, os.PathLike]


# ---------------------------------------------------------------------------------------------------------------
# weights
# ---------------------------------------------------------------------------------------------------------------
def save_params_npz(path: PathLike, params: Mapping, cfg: CNFConfig) -> None:
    """Write ``params`` (flat flax-path dict or nested flax tree) as an ``.npz`` keyed by flax path (fp32).  For a
    padded kernel config (params.kernel_config) the file holds the reference network's shapes, whether ``params`` are
    reference-shaped or padded."""
    blob = flatten_params(params, cfg)   # validates names and shapes (pads reference-shaped params)
    np.savez(path, **unflatten_params(blob, cfg, reference_shapes=True))


def load_params_npz(path: PathLike, cfg: CNFConfig) -> dict:
    """Read a flax-path ``.npz`` into a flat dict; raises ValueError on a missing / extra key or a wrong shape."""
    with np.load(path, allow_pickle=False) as f:
        flat = {k: np.asarray(f[k], np.float32) for k in f.files}
    flat = _flat_lookup(flat)
    expected = {p for p, _ in param_spec(cfg)}
    extra = sorted(set(flat) - expected)
    if extra:
        raise ValueError(f"unexpected parameters {extra[:4]}{'...' if len(extra) > 4 else ''}")
    flatten_params(flat, cfg)   # missing keys / shapes
    return flat


# ---------------------------------------------------------------------------------------------------------------
# datasets (ecnf/targets/data.py)
# ---------------------------------------------------------------------------------------------------------------
class FullGraphSample(NamedTuple):
    """positions [n, N, D] float32, features [n, N, 1] int32 (data.py:14-21)."""
    positions: np.ndarray
    features: np.ndarray

    def __getitem__(self, i):
        return FullGraphSample(self.positions[i], self.features[i])


def positional_dataset_only_to_full_graph(positions: np.ndarray) -> FullGraphSample:
    """Zero integer features beside the positions (data.py:23-28)."""
    positions = np.asarray(positions, np.float32)
    if positions.ndim != 3:
        raise ValueError(f"positions must be [n_data_points, n_nodes, dim], got shape {positions.shape}")
    return FullGraphSample(positions, np.zeros((*positions.shape[:-1], 1), np.int32))


def _load(path: PathLike) -> np.ndarray:
    if not os.path.exists(path):
        raise FileNotFoundError(f"{path} not found (the build does not download datasets)")
    return np.load(path, allow_pickle=False)


def load_dw4(train_set_size: int = 1000, val_set_size: int = 1000, test_set_size: int = 1000,
             path: Optional[PathLike] = None, fname: str = "dw4-data.npy"
             ) -> Tuple[FullGraphSample, FullGraphSample, FullGraphSample]:
    """data.py:31-56: reshape to [-1, 4, 2]; train = first, val = before test, test = last."""
    data = np.asarray(_load(os.path.join(path or ".", fname)), np.float32).reshape(-1, 4, 2)
    train = data[:train_set_size]
    val = data[-test_set_size - val_set_size:-test_set_size]
    test = data[-test_set_size:]
    return tuple(positional_dataset_only_to_full_graph(a) for a in (train, val, test))


def load_lj13(train_set_size: int = 1000, path: Optional[PathLike] = None
              ) -> Tuple[FullGraphSample, FullGraphSample, FullGraphSample]:
    """data.py:58-92: train = holdout[idx[:train_set_size]], val = all[1000:2000], test = all[:1000]."""
    base = path or "."
    train = np.asarray(_load(os.path.join(base, "holdout_data_LJ13.npy")), np.float32)
    idx = np.asarray(_load(os.path.join(base, "idx_LJ13.npy")), np.int64)
    val_test = np.asarray(_load(os.path.join(base, "all_data_LJ13.npy")), np.float32)
    if train_set_size > len(idx):
        raise ValueError(f"train_set_size {train_set_size} > {len(idx)} indices")
    train = train[idx[:train_set_size]].reshape(-1, 13, 3)
    val = val_test[1000:2000].reshape(-1, 13, 3)
    test = val_test[:1000].reshape(-1, 13, 3)
    return tuple(positional_dataset_only_to_full_graph(a) for a in (train, val, test))


def load_qm9(train_set_size: Optional[int] = None, path: Optional[PathLike] = None
             ) -> Tuple[FullGraphSample, FullGraphSample, FullGraphSample]:
    """data.py:94-121 (train, valid, test) from qm9pos_{train,valid,test}.npy; no download."""
    base = path or "."
    train = np.asarray(_load(os.path.join(base, "qm9pos_train.npy")), np.float32)
    if train_set_size is not None:
        if train_set_size > len(train):
            raise ValueError(f"train_set_size {train_set_size} > {len(train)} molecules")
        train = train[:train_set_size]
    valid = np.asarray(_load(os.path.join(base, "qm9pos_valid.npy")), np.float32)
    test = np.asarray(_load(os.path.join(base, "qm9pos_test.npy")), np.float32)
    return tuple(positional_dataset_only_to_full_graph(a) for a in (train, valid, test))


def aldp_sample(positions: np.ndarray) -> FullGraphSample:
    """data.py:124-154 for already-extracted coordinates (mdtraj is absent here): features = atom index
    (``arange(n_atoms)``, data.py:146), repeated per frame."""
    positions = np.asarray(positions, np.float32)
    if positions.ndim != 3:
        raise ValueError(f"positions must be [n_frames, n_atoms, 3], got shape {positions.shape}")
    feat = np.broadcast_to(np.arange(positions.shape[1], dtype=np.int32)[None, :, None],
                           (*positions.shape[:2], 1)).copy()
    return FullGraphSample(positions, feat)


def features_for_kernel(sample: FullGraphSample) -> np.ndarray:
    """[n, N, 1] dataset features -> the [n, N] int32 rows ``ecnf_integrate`` takes."""
    f = np.asarray(sample.features)
    return np.ascontiguousarray(f.reshape(f.shape[0], -1).astype(np.int32))
