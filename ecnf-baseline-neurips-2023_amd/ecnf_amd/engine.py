"""Device engine: one handle per (params, device) over the C-ABI, torch tensors as device memory.

Everything here runs on the HIP library; torch only allocates device memory and supplies the stream.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Mapping, Optional, Tuple, Union

import numpy as np
import torch

from . import _lib
from .params import CNFConfig, flatten_params, param_count


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _stream(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


@dataclass
class SolveOptions:
    """diffeqsolve arguments (sample_and_log_prob.py:32-37,84-89,139-144).

    step_size > 0 selects ConstantStepSize(dt0=step_size); step_size None selects PIDController(rtol, atol,
    dtmin) with dt0=None (Hairer initial step)."""
    solver: str = "dopri5"          # "dopri5" (the reference's) or "euler" (fixed-step NFE = 1/step_size)
    step_size: Optional[float] = 0.05
    rtol: float = 1e-5
    atol: float = 1e-5
    dtmin: float = 1e-5
    max_steps: int = 4096

    def to_c(self, t0: float, t1: float, divergence: int) -> _lib.EcnfSolveOpts:
        o = _lib.EcnfSolveOpts()
        o.solver = {"euler": _lib.SOLVER_EULER, "dopri5": _lib.SOLVER_DOPRI5}[self.solver]
        o.divergence = divergence
        o.t0, o.t1 = float(t0), float(t1)
        o.dt0 = float(self.step_size) if self.step_size else 0.0
        o.rtol, o.atol, o.dtmin = float(self.rtol), float(self.atol), float(self.dtmin)
        o.max_steps = int(self.max_steps)
        return o


class EcnfHandle:
    """Owns the device copy of the params (repacked into MFMA fragment order by ecnf_create)."""

    def __init__(self, cfg: CNFConfig, params: Union[Mapping, np.ndarray], device: Union[int, torch.device] = 0):
        if not torch.cuda.is_available():
            raise RuntimeError("ecnf_amd needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.lib = _lib.load()
        self.cfg = cfg
        self.device = torch.device("cuda", device if isinstance(device, int) else device.index or 0)
        blob = params if isinstance(params, np.ndarray) else flatten_params(params, cfg)
        blob = np.ascontiguousarray(blob, dtype=np.float32)
        if blob.size != param_count(cfg):
            raise ValueError(f"params blob has {blob.size} floats, expected {param_count(cfg)}")
        self._c = _lib.EcnfCfg(cfg.n_nodes, cfg.dim, cfg.n_features, cfg.hidden, cfg.time_embedding_dim,
                               cfg.mlp_width, cfg.mlp_depth, cfg.n_blocks, cfg.base_scale,
                               cfg.normalization_constant)
        n = ctypes.c_size_t()
        _lib.check(self.lib.ecnf_param_count(ctypes.byref(self._c), ctypes.byref(n)))
        assert n.value == blob.size
        h = ctypes.c_void_p()
        _lib.check(self.lib.ecnf_create(ctypes.byref(self._c), blob.ctypes.data, blob.size, self.device.index,
                                        ctypes.byref(h)))
        self._h = h

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            _lib.check(self.lib.ecnf_destroy(self._h))
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---------------------------------------------------------------------------------- helpers
    def _f32(self, x, shape_tail, name) -> torch.Tensor:
        x = torch.as_tensor(x, device=self.device)
        if x.dtype != torch.float32:
            x = x.float()
        x = x.contiguous()
        if tuple(x.shape[1:]) != tuple(shape_tail):
            raise ValueError(f"{name} must have shape [batch, {', '.join(map(str, shape_tail))}], got {tuple(x.shape)}")
        return x

    def _feat(self, feat, batch) -> torch.Tensor:
        N = self.cfg.n_nodes
        if feat is None:
            # build_cnf.py:74 asserts rank 2 on node_features: the EGNN field has no features=None path
            raise ValueError("features must be given for the EGNN vector field (build_cnf.py:73-75)")
        f = torch.as_tensor(feat, device=self.device)
        if f.dim() == 1:
            f = f.reshape(1, -1).expand(batch, -1)
        if f.numel() != batch * N:
            raise ValueError(f"features must have {N} entries per molecule")
        f = f.reshape(batch, N)
        if f.shape[1] != N:
            raise ValueError(f"features must have {N} entries per molecule, got {f.shape[1]}")
        if f.dtype.is_floating_point:
            raise ValueError("features are integer embedding ids")
        f = f.to(torch.int32).contiguous()
        if f.numel() and (int(f.min()) < 0 or int(f.max()) >= self.cfg.n_features):
            raise ValueError(f"feature ids must lie in [0, {self.cfg.n_features})")
        return f

    def molecules_per_workgroup(self, with_tangent: bool = False) -> int:
        v = ctypes.c_int32()
        _lib.check(self.lib.ecnf_molecules_per_workgroup(self._h, int(with_tangent), ctypes.byref(v)))
        return v.value

    def chain_arithmetic(self, with_tangent: bool = False) -> str:
        """'split_f16' (2-piece fp16 split, 3 cross terms), 'split_bf16' (3-piece bf16 split, 6 cross terms; both
        chain_split.hpp) or 'fp32_mfma'."""
        v = ctypes.c_int32()
        _lib.check(self.lib.ecnf_chain_arithmetic(self._h, int(with_tangent), ctypes.byref(v)))
        return {_lib.CHAIN_SPLIT_BF16: "split_bf16", _lib.CHAIN_SPLIT_F16: "split_f16"}.get(v.value, "fp32_mfma")

    # ---------------------------------------------------------------------------------- C-ABI calls
    def vector_field(self, x, t, feat) -> torch.Tensor:
        """cnf.apply(params, x[B, N*D], t[B], features[B, N]) (core.py:7-19)."""
        x = self._f32(x, (self.cfg.event_dim,), "x")
        B = x.shape[0]
        t = torch.as_tensor(t, device=self.device, dtype=torch.float32).reshape(-1).expand(B).contiguous()
        f = self._feat(feat, B)
        v = torch.empty_like(x)
        _lib.check(self.lib.ecnf_vector_field(self._h, _ptr(x), _ptr(t), _ptr(f), _ptr(v), B, _stream(self.device)))
        return v

    def jvp(self, x, t, feat, tangents) -> Tuple[torch.Tensor, torch.Tensor]:
        """(v, J @ u) for tangents u [B, K, N*D]: forward-mode counterpart of jax.vjp (sample_and_log_prob.py:64)."""
        x = self._f32(x, (self.cfg.event_dim,), "x")
        B = x.shape[0]
        u = torch.as_tensor(tangents, device=self.device, dtype=torch.float32)
        if u.dim() == 2:
            u = u[:, None]
        u = u.contiguous()
        if u.shape[0] != B or u.shape[2] != self.cfg.event_dim:
            raise ValueError(f"tangents must be [batch, K, {self.cfg.event_dim}]")
        t = torch.as_tensor(t, device=self.device, dtype=torch.float32).reshape(-1).expand(B).contiguous()
        f = self._feat(feat, B)
        v = torch.empty_like(x)
        ju = torch.empty_like(u)
        _lib.check(self.lib.ecnf_vf_jvp(self._h, _ptr(x), _ptr(t), _ptr(f), _ptr(u), u.shape[1], _ptr(v), _ptr(ju), B,
                                        _stream(self.device)))
        return v, ju

    def integrate(self, y0, feat, t0: float, t1: float, opts: SolveOptions, divergence: int = _lib.DIV_NONE,
                  eps=None, check_status: bool = True):
        """One-launch ODE solve for the whole batch.  Returns (y1, dlogp or None, nfe, status)."""
        y0 = self._f32(y0, (self.cfg.event_dim,), "y0")
        B = y0.shape[0]
        f = self._feat(feat, B)
        e = None
        if divergence == _lib.DIV_HUTCHINSON:
            if eps is None:
                raise ValueError("Hutchinson divergence needs eps")
            e = self._f32(eps, (self.cfg.event_dim,), "eps")
            if e.shape[0] != B:
                raise ValueError("eps batch mismatch")
        y1 = torch.empty_like(y0)
        dl = torch.empty(B, device=self.device, dtype=torch.float32) if divergence != _lib.DIV_NONE else None
        nfe = torch.empty(B, device=self.device, dtype=torch.int32)
        status = torch.empty(B, device=self.device, dtype=torch.int32)
        o = opts.to_c(t0, t1, divergence)
        _lib.check(self.lib.ecnf_integrate(self._h, ctypes.byref(o), _ptr(y0), _ptr(f), _ptr(e), _ptr(y1), _ptr(dl),
                                           _ptr(nfe), _ptr(status), B, _stream(self.device)))
        if check_status and B:
            bad = int((status != 0).sum())
            if bad:
                # diffrax raises when max_steps is exceeded
                raise RuntimeError(f"{bad} molecule(s) exceeded max_steps={opts.max_steps}")
        return y1, dl, nfe, status

    def base_sample(self, z) -> torch.Tensor:
        z = self._f32(z, (self.cfg.event_dim,), "z")
        x0 = torch.empty_like(z)
        _lib.check(self.lib.ecnf_base_sample(self._h, _ptr(z), _ptr(x0), z.shape[0], _stream(self.device)))
        return x0

    def base_log_prob(self, y) -> torch.Tensor:
        y = self._f32(y, (self.cfg.event_dim,), "y")
        out = torch.empty(y.shape[0], device=self.device, dtype=torch.float32)
        _lib.check(self.lib.ecnf_base_log_prob(self._h, _ptr(y), _ptr(out), y.shape[0], _stream(self.device)))
        return out
