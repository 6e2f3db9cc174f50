"""Flow-matching training on the MI355X engine.

Mirrors, by name and argument meaning:
  * ``flow_matching_loss_fn``        ecnf/cnf/loss.py:10-32
  * ``TrainingState`` / ``flow_matching_update_fn``   ecnf/cnf/gradient_step.py:13-53 (Adam + EMA)
  * ``adam`` / ``warmup_cosine_decay_schedule``      the optax pieces setup_training.py:96-109 builds

The loss, its gradient (hand-written reverse mode through the EGNN, strict-fp32 GEMMs on the matrix cores) and the
Adam / EMA update run in libecnf_hip.so (ecnf_fm_loss_grad, ecnf_adam_update); parameters, gradients and moments
are flat device blobs in the reference's ravel_pytree order, so ``unflatten_params(blob.cpu().numpy(), cfg)`` is the
flax-path params dict.  Differences: JAX keys are int seeds / torch Generators (threefry is not reproduced), and the
noise can be passed explicitly (``x0=``, ``t=``) for bit-reproducible comparisons.
"""
from __future__ import annotations

import ctypes
import math
from typing import Callable, Mapping, NamedTuple, Optional, Union

import numpy as np
import torch

from . import _lib
from .params import CNFConfig, flatten_params, param_count


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


class Trainer:
    """Workspace for the training step of one config on one device (ecnf_trainer_create)."""

    def __init__(self, cfg: CNFConfig, max_batch: int, device: Union[int, torch.device] = 0):
        if not torch.cuda.is_available():
            raise RuntimeError("ecnf_amd needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.lib = _lib.load()
        self.cfg = cfg
        self.max_batch = int(max_batch)
        self.device = torch.device("cuda", device if isinstance(device, int) else device.index or 0)
        self._c = _lib.EcnfCfg(cfg.n_nodes, cfg.dim, cfg.n_features, cfg.hidden, cfg.time_embedding_dim,
                               cfg.mlp_width, cfg.mlp_depth, cfg.n_blocks, cfg.base_scale,
                               cfg.normalization_constant)
        h = ctypes.c_void_p()
        _lib.check(self.lib.ecnf_trainer_create(ctypes.byref(self._c), self.max_batch, self.device.index,
                                                ctypes.byref(h)))
        self._h = h
        self.n_params = param_count(cfg)

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            _lib.check(self.lib.ecnf_trainer_destroy(self._h))
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _stream(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream

    def set_reduction_arena(self, floats: int = 0) -> int:
        """Diagnostic (ecnf_trainer_set_reduction_arena): shrink the split-reduction partial arena (0 restores it);
        returns the size in floats now in use."""
        used = ctypes.c_size_t()
        _lib.check(self.lib.ecnf_trainer_set_reduction_arena(self._h, int(floats), ctypes.byref(used)))
        return used.value

    def device_params(self, params) -> torch.Tensor:
        """A flax-path dict, nested flax tree, host blob or device tensor -> the flat fp32 device blob."""
        if torch.is_tensor(params):
            p = params.to(self.device, torch.float32).contiguous()
        else:
            blob = params if isinstance(params, np.ndarray) else flatten_params(params, self.cfg)
            p = torch.as_tensor(np.ascontiguousarray(blob, np.float32), device=self.device)
        if p.numel() != self.n_params:
            raise ValueError(f"params blob has {p.numel()} floats, expected {self.n_params}")
        return p.reshape(-1)

    def loss_and_grad(self, params: torch.Tensor, x1, x0, t, features, sigma_min: Optional[float] = None):
        """(loss [scalar device tensor], grad [n_params device tensor]) of loss.py:10-32 for the given noise."""
        cfg = self.cfg
        p = self.device_params(params)
        x1 = torch.as_tensor(x1, device=self.device, dtype=torch.float32).reshape(-1, cfg.event_dim).contiguous()
        B = x1.shape[0]
        if B < 1 or B > self.max_batch:
            raise ValueError(f"batch must lie in [1, {self.max_batch}]")
        x0 = torch.as_tensor(x0, device=self.device, dtype=torch.float32).reshape(B, cfg.event_dim).contiguous()
        t = torch.as_tensor(t, device=self.device, dtype=torch.float32).reshape(B).contiguous()
        f = torch.as_tensor(features)
        if f.dtype.is_floating_point:
            raise ValueError("features are integer embedding ids")
        if f.dim() == 1:
            f = f.reshape(1, -1).expand(B, -1)
        if not f.is_cuda and f.numel() and (int(f.min()) < 0 or int(f.max()) >= cfg.n_features):
            raise ValueError(f"feature ids must lie in [0, {cfg.n_features})")
        f = f.to(self.device, torch.int32).reshape(B, cfg.n_nodes).contiguous()
        loss = torch.empty(1, device=self.device, dtype=torch.float32)
        grad = torch.empty(self.n_params, device=self.device, dtype=torch.float32)
        sm = cfg.sigma_min if sigma_min is None else float(sigma_min)
        _lib.check(self.lib.ecnf_fm_loss_grad(self._h, _ptr(p), _ptr(x1), _ptr(x0), _ptr(t), _ptr(f), sm, B,
                                              _ptr(loss), _ptr(grad), self._stream()))
        return loss[0], grad

    def adam_update(self, grad, params, mu, nu, ema, lr: float, count: int, b1: float = 0.9, b2: float = 0.999,
                    eps: float = 1e-8, eps_root: float = 0.0, ema_beta: float = 0.999):
        """In place: params, mu, nu (and ema when given).  Returns the device float[2] (|grad|, |update|)."""
        o = _lib.EcnfAdamOpts(float(lr), float(b1), float(b2), float(eps), float(eps_root), int(count),
                              float(ema_beta))
        norms = torch.empty(2, device=self.device, dtype=torch.float32)
        _lib.check(self.lib.ecnf_adam_update(self._h, _ptr(grad), _ptr(params), _ptr(mu), _ptr(nu), _ptr(ema),
                                             self.n_params, ctypes.byref(o), _ptr(norms), self._stream()))
        return norms


# ------------------------------------------------------------------------------------------------------------
# optax pieces used by setup_training.py:96-109
# ------------------------------------------------------------------------------------------------------------
def warmup_cosine_decay_schedule(init_value: float, peak_value: float, warmup_steps: int, decay_steps: int,
                                 end_value: float = 0.0, exponent: float = 1.0) -> Callable[[int], float]:
    """optax.warmup_cosine_decay_schedule: linear init -> peak over warmup_steps, then cosine decay to end_value
    at decay_steps (join_schedules of linear_schedule and cosine_decay_schedule(peak, decay_steps - warmup))."""
    alpha = 0.0 if peak_value == 0 else end_value / peak_value

    def schedule(count: int) -> float:
        count = int(count)
        if count < warmup_steps:
            if warmup_steps <= 0:
                return peak_value
            frac = 1.0 - min(max(count, 0), warmup_steps) / warmup_steps
            return (init_value - peak_value) * frac + peak_value
        c = count - warmup_steps
        ds = decay_steps - warmup_steps
        if ds <= 0:
            return peak_value * alpha if ds < 0 else peak_value
        c = min(c, ds)
        cosine = 0.5 * (1.0 + math.cos(math.pi * c / ds))
        return peak_value * ((1.0 - alpha) * cosine ** exponent + alpha)

    return schedule


class AdamState(NamedTuple):
    count: int
    mu: torch.Tensor
    nu: torch.Tensor


class Adam(NamedTuple):
    """optax.adam(learning_rate, b1, b2, eps, eps_root): ``init(params) -> AdamState``; the update itself runs in
    :func:`flow_matching_update_fn` (ecnf_adam_update, fused with apply_updates and the EMA)."""
    learning_rate: Union[float, Callable[[int], float]]
    b1: float = 0.9
    b2: float = 0.999
    eps: float = 1e-8
    eps_root: float = 0.0

    def init(self, params: torch.Tensor) -> AdamState:
        return AdamState(0, torch.zeros_like(params), torch.zeros_like(params))

    def lr(self, count: int) -> float:
        return float(self.learning_rate(count)) if callable(self.learning_rate) else float(self.learning_rate)


def adam(learning_rate, b1: float = 0.9, b2: float = 0.999, eps: float = 1e-8, eps_root: float = 0.0) -> Adam:
    return Adam(learning_rate, b1, b2, eps, eps_root)


# ------------------------------------------------------------------------------------------------------------
# loss.py / gradient_step.py
# ------------------------------------------------------------------------------------------------------------
class TrainingState(NamedTuple):
    """gradient_step.py:13-17: params (flat device blob), opt_state (AdamState), key (int seed or torch.Generator),
    ema_params (flat device blob, or None when EMA is off)."""
    params: torch.Tensor
    opt_state: AdamState
    key: Union[int, torch.Generator]
    ema_params: Optional[torch.Tensor] = None


_TRAINERS: "dict[tuple, Trainer]" = {}


def trainer_for(cfg: CNFConfig, batch: int, device: torch.device) -> Trainer:
    """A cached Trainer whose workspace holds `batch` molecules (grown by powers of two)."""
    key = (cfg, str(device))
    tr = _TRAINERS.get(key)
    if tr is None or tr.max_batch < batch:
        cap = 1 << max(6, (int(batch) - 1).bit_length())
        tr = Trainer(cfg, cap, device)
        _TRAINERS[key] = tr
    return tr


def _generator(key, device) -> torch.Generator:
    if isinstance(key, torch.Generator):
        return key
    g = torch.Generator(device=device)
    g.manual_seed(int(key) if key is not None else 0)
    return g


def _noise(cnf, key, batch: int):
    """loss.py:22-25: key1 -> x0 = cnf.sample_base(key1, batch), key2 -> t ~ U(0, 1)."""
    g = _generator(key, cnf.device)
    x0 = cnf.sample_base(g, batch)
    t = torch.rand((batch,), generator=g, device=cnf.device, dtype=torch.float32)
    return x0, t


def flow_matching_loss_fn(cnf, params, x_data, key, features=None, *, x0=None, t=None, with_grad: bool = False):
    """loss.py:10-32: (loss, info).  with_grad=True returns (loss, info, grad) -- jax.grad's companion here."""
    if features is None:
        raise ValueError("features must be given for the EGNN vector field (build_cnf.py:73-75)")
    x_data = torch.as_tensor(x_data, device=cnf.device, dtype=torch.float32)
    if x_data.dim() != 2:
        raise ValueError("x_data must be rank 2 [batch, n_frames*dim] (loss.py:17)")
    B = x_data.shape[0]
    if x0 is None or t is None:
        nx0, nt = _noise(cnf, key, B)
        x0 = nx0 if x0 is None else x0
        t = nt if t is None else t
    tr = trainer_for(cnf.cfg, B, cnf.device)
    loss, grad = tr.loss_and_grad(params, x_data, x0, t, features)
    info = {"loss": loss}
    return (loss, info, grad) if with_grad else (loss, info)


def flow_matching_update_fn(cnf, opt: Adam, state: TrainingState, x_data, features=None, ema_beta: float = 0.999,
                            *, x0=None, t=None):
    """gradient_step.py:21-53: grads of the flow-matching loss, one Adam step, optional EMA; returns
    (new TrainingState, info{loss, grad_norm, update_norm})."""
    g = _generator(state.key, cnf.device)
    loss, info, grad = flow_matching_loss_fn(cnf, state.params, x_data, g, features, x0=x0, t=t, with_grad=True)
    tr = trainer_for(cnf.cfg, int(torch.as_tensor(x_data).shape[0]), cnf.device)
    params = state.params.clone()
    mu, nu = state.opt_state.mu.clone(), state.opt_state.nu.clone()
    ema = None if state.ema_params is None else state.ema_params.clone()
    count = state.opt_state.count + 1
    norms = tr.adam_update(grad, params, mu, nu, ema, lr=opt.lr(state.opt_state.count), count=count, b1=opt.b1,
                           b2=opt.b2, eps=opt.eps, eps_root=opt.eps_root, ema_beta=ema_beta)
    info.update(grad_norm=norms[0], update_norm=norms[1])
    return TrainingState(params=params, opt_state=AdamState(count, mu, nu), key=g, ema_params=ema), info


def init_training_state(cnf, params: Mapping, opt: Adam, key=0, use_ema: bool = False) -> TrainingState:
    """setup_training.py:132-139."""
    tr = trainer_for(cnf.cfg, 1, cnf.device)
    p = tr.device_params(params)
    return TrainingState(params=p, opt_state=opt.init(p), key=key, ema_params=p.clone() if use_ema else None)
