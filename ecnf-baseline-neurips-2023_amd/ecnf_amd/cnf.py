"""The reference's ``ecnf.cnf`` surface on the MI355X engine.

Mirrors (names, argument meaning, error behaviour):
  * ``FlowMatchingCNF`` / ``VectorFieldApply``            ecnf/cnf/core.py:7-49
  * ``optimal_transport_conditional_vf``                   ecnf/cnf/core.py:35-39
  * ``build_cnf``                                          ecnf/cnf/build_cnf.py:34-102
  * ``sample_cnf`` / ``get_log_prob`` / ``sample_and_log_prob_cnf``   ecnf/cnf/sample_and_log_prob.py:11-149

Differences, all deliberate and documented in DESIGN.md:
  * calls are batched natively: ``features`` may be [N] (one molecule, like the reference) or [B, N]; the
    reference's callers vmap (setup_training.py:47,197) — here the batch goes to one kernel launch;
  * ``key`` is an int seed or a ``torch.Generator`` on the device (JAX threefry is not reproduced); the noise can
    instead be passed explicitly (``x0=``, ``z=``, ``eps=``) for bit-reproducible comparisons;
  * the fixed-step branch of sample_and_log_prob_cnf integrates (x0, 0) — the reference passes ``y0=x0``
    (sample_and_log_prob.py:139-140) and cannot run;
  * ``solver="euler"`` is available besides the reference's Dopri5 (fixed step only).
"""
from __future__ import annotations

import hashlib
import weakref
from functools import partial
from typing import Callable, Mapping, NamedTuple, Optional, Sequence, Tuple, Union

import numpy as np
import torch

from . import _lib
from .engine import EcnfHandle, SolveOptions
from .params import CNFConfig, flatten_params, init_from_spec, init_params, kernel_config, ref_param_spec

Params = Union[Mapping, np.ndarray, EcnfHandle]


class FlowMatchingCNF(NamedTuple):
    """core.py:42-49 (+ ``cfg``, ``device`` and ``to_device``: params -> an explicit EcnfHandle)."""
    init: Callable
    apply: Callable
    sample_base: Callable
    get_x_t_and_conditional_u_t: Callable
    log_prob_base: Callable
    sample_and_log_prob_base: Callable
    cfg: CNFConfig
    device: torch.device
    to_device: Callable


def optimal_transport_conditional_vf(x0, x1, t, sigma_min: float):
    """core.py:35-39."""
    t = torch.as_tensor(t, device=x0.device, dtype=x0.dtype)
    if t.dim() == x0.dim() - 1:
        t = t[..., None]
    x_t = (1 - (1 - sigma_min) * t) * x0 + t * x1
    u_t = x1 - (1 - sigma_min) * x0
    return x_t, u_t


# --------------------------------------------------------------------------------------------------
# params -> device handle (uploaded once per distinct CONTENT)
# --------------------------------------------------------------------------------------------------
_HANDLE_CACHE: "dict[tuple, EcnfHandle]" = {}
_CACHE_MAX = 8


def params_digest(params: Union[Mapping, np.ndarray], cfg: CNFConfig) -> str:
    """Content hash of the flat (ravel_pytree-ordered) params blob: a dict updated in place, or a new dict with
    the same values, maps to the handle holding exactly these weights."""
    blob = params if isinstance(params, np.ndarray) else flatten_params(params, cfg)
    blob = np.ascontiguousarray(blob, dtype=np.float32)
    return hashlib.blake2b(blob.view(np.uint8), digest_size=16).hexdigest()


def device_params(params: Params, cfg: CNFConfig, device: torch.device) -> EcnfHandle:
    """Upload ``params`` (flax-path dict, nested flax dict or flat blob) to a handle, reusing the handle of an
    earlier upload with identical content (blake2b of the flat blob; the hash costs ~1 ms per MB of weights per
    call -- pass an :class:`EcnfHandle` (``to_device``) to skip it).  An EcnfHandle is used as is."""
    if isinstance(params, EcnfHandle):
        return params
    key = (params_digest(params, cfg), cfg, str(device))
    hit = _HANDLE_CACHE.get(key)
    if hit is not None:
        return hit
    h = EcnfHandle(cfg, params, device)
    if len(_HANDLE_CACHE) >= _CACHE_MAX:
        _HANDLE_CACHE.pop(next(iter(_HANDLE_CACHE)))   # freed by its __del__ once no caller holds it
    _HANDLE_CACHE[key] = h
    # a caller that changes this handle (update_params / set_precision, e.g. on the handle of cnf.to_device(p) in a
    # training loop) takes it out of the cache: a later apply(p, ...) uploads p again instead of using other weights
    # (a weak reference: a callback holding h would keep every cached handle in a reference cycle, so an evicted
    # handle's device memory would wait for the cyclic GC instead of being freed when its last caller drops it)
    ref = weakref.ref(h)
    h._on_mutate.append(lambda: _HANDLE_CACHE.pop(key, None) if _HANDLE_CACHE.get(key) is ref() else None)
    return h


def _generator(key, device) -> torch.Generator:
    if isinstance(key, torch.Generator):
        return key
    g = torch.Generator(device=device)
    g.manual_seed(int(key) if key is not None else 0)
    return g


def _batched(features, cfg: CNFConfig, n: Optional[int]):
    """Returns (features [B, N] or None, B, squeeze)."""
    if features is None:
        return None, (1 if n is None else int(n)), n is None
    f = torch.as_tensor(features)
    if f.dim() == 1:
        if n is None:
            return f.reshape(1, -1), 1, True
        return f.reshape(1, -1).expand(int(n), -1), int(n), False
    return f, f.shape[0], False


# --------------------------------------------------------------------------------------------------
# build_cnf
# --------------------------------------------------------------------------------------------------
def build_cnf(n_frames: int, dim: int, sigma_min: float, base_scale: float, n_blocks_egnn: int,
              mlp_units: Sequence[int], n_invariant_feat_hidden: int, time_embedding_dim: int, n_features: int,
              device: Union[int, str, torch.device] = 0) -> FlowMatchingCNF:
    """build_cnf.py:34-102: zero-CoM scaled Gaussian base + FlatEgnn vector field (on the HIP engine).

    Any mlp_units (each <= 256, a compiled depth) and n_invariant_feat_hidden run on the compiled kernel shape
    params.kernel_config picks: the reference-shaped params are zero-padded on upload (params.pad_params), which
    leaves the function unchanged.  ``cfg`` is that kernel shape (with the reference widths in ``cfg.ref_mlp_units`` /
    ``cfg.ref_hidden``, so EcnfHandle.update_params, the Trainer and dataio pad reference-shaped params too);
    ``init`` returns reference-shaped params."""
    units = tuple(int(u) for u in mlp_units)
    H = int(n_invariant_feat_hidden)
    cfg = kernel_config(int(n_frames), int(dim), int(n_features), H, int(time_embedding_dim), units,
                        int(n_blocks_egnn), float(base_scale), float(sigma_min))
    padded = units != cfg.mlp_units or H != cfg.hidden
    dev = torch.device(device) if not isinstance(device, int) else torch.device("cuda", device)

    def init(key, x=None, t=None, features=None):
        seed = key if isinstance(key, (int, np.integer)) else 0
        if not padded:
            return init_params(cfg, int(seed))
        return init_from_spec(ref_param_spec(cfg.n_features, H, cfg.time_embedding_dim, units, cfg.n_blocks),
                              int(seed))

    def to_device(params):
        # reference-shaped params of a padded config are zero-padded by flatten_params (cfg.ref_mlp_units)
        return device_params(params, cfg, dev)

    def apply(params, x, t, features=None):
        h = to_device(params)
        x = torch.as_tensor(x, device=dev, dtype=torch.float32)
        if x.dim() != 2:
            raise ValueError("positions must be rank 2 [batch, n_frames*dim] (build_cnf.py:73)")
        t = torch.as_tensor(t, device=dev, dtype=torch.float32)
        if t.dim() != 1:
            raise ValueError("time must be rank 1 (build_cnf.py:75)")
        return h.vector_field(x, t, features)

    def sample_base(key, n: int):
        g = _generator(key, dev)
        z = torch.randn((int(n), cfg.event_dim), generator=g, device=dev, dtype=torch.float32)
        return _base_handle().base_sample(z)

    def log_prob_base(x):
        x = torch.as_tensor(x, device=dev, dtype=torch.float32)
        squeeze = x.dim() == 1
        out = _base_handle().base_log_prob(x.reshape(-1, cfg.event_dim))
        return out[0] if squeeze else out

    def sample_and_log_prob_base(seed, sample_shape=()):
        n = int(np.prod(sample_shape)) if sample_shape else 1
        x = sample_base(seed, n)
        lp = log_prob_base(x)
        if not sample_shape:
            return x[0], lp[0]
        return x.reshape(*sample_shape, cfg.event_dim), lp.reshape(sample_shape)

    # the base kernels only need the config; keep a zero-params handle for them
    _base = {}

    def _base_handle():
        if "h" not in _base:
            _base["h"] = EcnfHandle(cfg, np.zeros(_param_count(cfg), np.float32), dev)
        return _base["h"]

    return FlowMatchingCNF(init=init, apply=apply, sample_base=sample_base,
                           get_x_t_and_conditional_u_t=partial(optimal_transport_conditional_vf, sigma_min=sigma_min),
                           log_prob_base=log_prob_base, sample_and_log_prob_base=sample_and_log_prob_base,
                           cfg=cfg, device=dev, to_device=to_device)


def _param_count(cfg):
    from .params import param_count
    return param_count(cfg)


def _opts(use_fixed_step_size, rtol, atol, step_size, solver, max_steps):
    if solver == "euler" and not use_fixed_step_size:
        raise ValueError("solver='euler' needs use_fixed_step_size=True")
    return SolveOptions(solver=solver, step_size=step_size if use_fixed_step_size else None, rtol=rtol, atol=atol,
                        dtmin=1e-5, max_steps=max_steps)


# --------------------------------------------------------------------------------------------------
# sample_and_log_prob.py
# --------------------------------------------------------------------------------------------------
def sample_cnf(cnf: FlowMatchingCNF, params: Params, key, features=None, use_fixed_step_size: bool = False,
               rtol: float = 1e-5, atol: float = 1e-5, step_size: float = 0.05, *, n_samples: Optional[int] = None,
               x0=None, solver: str = "dopri5", max_steps: int = 4096):
    """sample_and_log_prob.py:11-38: x0 ~ base, ODE 0 -> 1; returns x1 ([N*D] for one molecule, else [B, N*D])."""
    cfg = cnf.cfg
    h = cnf.to_device(params)
    if x0 is not None:
        x0 = torch.as_tensor(x0, device=cnf.device, dtype=torch.float32)
        squeeze = x0.dim() == 1
        x0 = x0.reshape(-1, cfg.event_dim)
        feats, B, _ = _batched(features, cfg, x0.shape[0])
    else:
        feats, B, squeeze = _batched(features, cfg, n_samples)
        x0 = cnf.sample_base(key, B)
    y1, _, _, _ = h.integrate(x0, feats, 0.0, 1.0, _opts(use_fixed_step_size, rtol, atol, step_size, solver, max_steps))
    return y1[0] if squeeze else y1


def get_log_prob(cnf: FlowMatchingCNF, params: Params, x, key, features=None, approx: bool = False,
                 use_fixed_step_size: bool = False, rtol: float = 1e-5, atol: float = 1e-5, step_size: float = 0.05,
                 *, eps=None, solver: str = "dopri5", max_steps: int = 4096):
    """sample_and_log_prob.py:41-94: ODE 1 -> 0 on (x, 0); returns (log_p, log_prob_base, delta_log_likelihood).

    approx=False: exact trace of the full N*D Jacobian; approx=True: Hutchinson with eps ~ N(0, I) drawn once."""
    cfg = cnf.cfg
    h = cnf.to_device(params)
    x = torch.as_tensor(x, device=cnf.device, dtype=torch.float32)
    squeeze = x.dim() == 1
    x = x.reshape(-1, cfg.event_dim)
    feats, B, _ = _batched(features, cfg, x.shape[0])
    div = _lib.DIV_HUTCHINSON if approx else _lib.DIV_EXACT
    if approx and eps is None:
        g = _generator(key, cnf.device)
        eps = torch.randn(x.shape, generator=g, device=cnf.device, dtype=torch.float32)
    x0, dl, _, _ = h.integrate(x, feats, 1.0, 0.0, _opts(use_fixed_step_size, rtol, atol, step_size, solver,
                                                          max_steps), divergence=div, eps=eps)
    lpb = h.base_log_prob(x0)
    log_p = lpb + dl
    if squeeze:
        return log_p[0], lpb[0], dl[0]
    return log_p, lpb, dl


def sample_and_log_prob_cnf(cnf: FlowMatchingCNF, params: Params, key, features=None, approx: bool = False,
                            use_fixed_step_size: bool = False, rtol: float = 1e-5, atol: float = 1e-5,
                            step_size: float = 0.05, *, n_samples: Optional[int] = None, z=None,
                            solver: str = "dopri5", max_steps: int = 4096):
    """sample_and_log_prob.py:97-149: x0 ~ base, ODE 0 -> 1 on (x0, 0); returns (x1, log p0(x0) - l(1)).

    As in the reference, the Hutchinson probe is the same standard-normal draw z that produced x0
    (sample_and_log_prob.py:130 vs :137)."""
    cfg = cnf.cfg
    h = cnf.to_device(params)
    if z is not None:
        z = torch.as_tensor(z, device=cnf.device, dtype=torch.float32)
        squeeze = z.dim() == 1
        z = z.reshape(-1, cfg.event_dim)
        feats, B, _ = _batched(features, cfg, z.shape[0])
    else:
        feats, B, squeeze = _batched(features, cfg, n_samples)
        g = _generator(key, cnf.device)
        z = torch.randn((B, cfg.event_dim), generator=g, device=cnf.device, dtype=torch.float32)
    x0 = h.base_sample(z)
    div = _lib.DIV_HUTCHINSON if approx else _lib.DIV_EXACT
    x1, dl, _, _ = h.integrate(x0, feats, 0.0, 1.0, _opts(use_fixed_step_size, rtol, atol, step_size, solver,
                                                           max_steps), divergence=div, eps=z)
    log_p = h.base_log_prob(x0) - dl
    if squeeze:
        return x1[0], log_p[0]
    return x1, log_p
