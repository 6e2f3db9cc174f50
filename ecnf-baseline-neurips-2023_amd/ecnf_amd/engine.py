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


PRECISIONS = {"split_f16": _lib.PREC_SPLIT_F16, "fp32": _lib.PREC_FP32}


class EcnfHandle:
    """Owns the device copy of the params (repacked into MFMA fragment order by ecnf_create).

    precision: "split_f16" (default; fp32 operands split into fp16 pieces on the 16-bit matrix cores) or "fp32"
    (every GEMM on the fp32 matrix cores) -- include/ecnf.h ecnf_precision."""

    def __init__(self, cfg: CNFConfig, params: Union[Mapping, np.ndarray], device: Union[int, torch.device] = 0,
                 precision: str = "split_f16"):
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
        # callbacks run when this handle's weights or precision change (ecnf_amd.cnf evicts its content-hash cache
        # entry, so a params dict never maps to a handle holding other weights)
        self._on_mutate = []
        cur = ctypes.c_int32()
        _lib.check(self.lib.ecnf_get_precision(self._h, ctypes.byref(cur)))
        if precision == "split_f16" and cur.value == _lib.PREC_FP32:
            # edge-MLP weights >= 2^15 do not fit the fp16 split: ecnf_create made this a strict-fp32 handle
            self.precision = "fp32"
        else:
            self._set_precision(precision)

    def _mutated(self) -> None:
        for cb in self._on_mutate:
            cb()
        self._on_mutate = []

    def update_params(self, params) -> None:
        """Re-pack new weights into this handle (ecnf_update_params): a flax-path dict / flat host blob, or the flat
        device tensor of a TrainingState."""
        self._mutated()
        if torch.is_tensor(params) and params.is_cuda:
            p = params.to(self.device, torch.float32).contiguous().reshape(-1)
            if p.numel() != param_count(self.cfg):
                raise ValueError(f"params blob has {p.numel()} floats, expected {param_count(self.cfg)}")
            _lib.check(self.lib.ecnf_update_params(self._h, p.data_ptr(), 1))
            self._sync_precision()
            return
        blob = params if isinstance(params, np.ndarray) else flatten_params(params, self.cfg)
        blob = np.ascontiguousarray(blob, dtype=np.float32)
        if blob.size != param_count(self.cfg):
            raise ValueError(f"params blob has {blob.size} floats, expected {param_count(self.cfg)}")
        _lib.check(self.lib.ecnf_update_params(self._h, blob.ctypes.data, 0))
        self._sync_precision()

    def _sync_precision(self) -> None:
        cur = ctypes.c_int32()
        _lib.check(self.lib.ecnf_get_precision(self._h, ctypes.byref(cur)))
        self.precision = "fp32" if cur.value == _lib.PREC_FP32 else "split_f16"

    def set_precision(self, precision: str) -> None:
        self._mutated()
        self._set_precision(precision)

    def _set_precision(self, precision: str) -> None:
        if precision not in PRECISIONS:
            raise ValueError(f"precision must be one of {sorted(PRECISIONS)}")
        _lib.check(self.lib.ecnf_set_precision(self._h, PRECISIONS[precision]))
        self.precision = precision

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
        on_device = torch.is_tensor(feat) and feat.is_cuda
        f = torch.as_tensor(feat)
        if f.dtype.is_floating_point:
            raise ValueError("features are integer embedding ids")
        if not on_device and f.numel() and (int(f.min()) < 0 or int(f.max()) >= self.cfg.n_features):
            # host input: validated here, before the upload.  Device inputs are checked by the kernels (status
            # ECNF_E_INVALID per molecule from integrate, NaN rows from vector_field / jvp): no device-to-host
            # sync on the call path
            raise ValueError(f"feature ids must lie in [0, {self.cfg.n_features})")
        f = f.to(self.device)
        if f.dim() == 1:
            f = f.reshape(1, -1).expand(batch, -1)
        if f.numel() != batch * N:
            raise ValueError(f"features must have {N} entries per molecule")
        return f.reshape(batch, N).to(torch.int32).contiguous()

    def molecules_per_workgroup(self, with_tangent: bool = False) -> int:
        v = ctypes.c_int32()
        _lib.check(self.lib.ecnf_molecules_per_workgroup(self._h, int(with_tangent), ctypes.byref(v)))
        return v.value

    def _fp32_available(self, with_tangent: bool) -> bool:
        """Whether the strict-fp32 kernels exist for this shape and fit the LDS (every compiled shape has them, the
        M = 256 tangent kernels included since round 3; a tangent kernel can still miss the LDS at large N)."""
        prev = self.precision
        self._set_precision("fp32")
        try:
            return self.molecules_per_workgroup(with_tangent) > 0
        finally:
            self._set_precision(prev)

    def chain_arithmetic(self, with_tangent: bool = False) -> str:
        """Edge-chain arithmetic at the current precision: 'split_f16' (2-piece fp16 split, 3 cross terms),
        'split_bf16' (3-piece bf16 split, 6 cross terms; both chain_split.hpp) or 'fp32_mfma'."""
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
                  eps=None, check_status: bool = True, fallback: bool = True):
        """ODE solve of the whole batch in one launch (adaptive solves with more workgroups than CUs: two launches,
        the unfinished molecules re-dealt longest first; bitwise the same results).  Returns (y1, dlogp or None, nfe,
        status).

        check_status: read the per-molecule status back (one sync) and raise like diffrax / chex would:
        ECNF_E_MAX_STEPS -> RuntimeError, ECNF_E_INVALID (embedding ids out of range) -> ValueError.
        fallback (with check_status, split_f16 precision): molecules that report ECNF_E_NONFINITE (an activation
        beyond the fp16 range of the split GEMMs) are solved again on the strict-fp32 kernels and replaced; a
        molecule that is still non-finite raises."""
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
        y1, dl, nfe, status = self._integrate(y0, f, e, t0, t1, opts, divergence)
        if check_status and B:
            bad = status != _lib.ECNF_OK
            if bool(bad.any()):
                st = status.cpu()
                if fallback and self.precision == "split_f16" and bool((st == _lib.ECNF_E_NONFINITE).any()) and \
                        self._fp32_available(divergence != _lib.DIV_NONE):
                    idx = torch.nonzero(status == _lib.ECNF_E_NONFINITE).reshape(-1)
                    self._set_precision("fp32")
                    try:
                        r = self._integrate(y0[idx].contiguous(), f[idx].contiguous(),
                                            None if e is None else e[idx].contiguous(), t0, t1, opts, divergence)
                    finally:
                        self._set_precision("split_f16")
                    y1[idx], nfe[idx], status[idx] = r[0], r[2], r[3]
                    if dl is not None:
                        dl[idx] = r[1]
                    st = status.cpu()
                if bool((st == _lib.ECNF_E_INVALID).any()):
                    raise ValueError(f"feature ids must lie in [0, {self.cfg.n_features})")
                n_ms = int((st == _lib.ECNF_E_MAX_STEPS).sum())
                if n_ms:
                    # diffrax raises when max_steps is exceeded
                    raise RuntimeError(f"{n_ms} molecule(s) exceeded max_steps={opts.max_steps}")
                n_nf = int((st == _lib.ECNF_E_NONFINITE).sum())
                if n_nf:
                    raise RuntimeError(f"{n_nf} molecule(s) ended with a non-finite state")
                n_hip = int((st == _lib.ECNF_E_HIP).sum())
                if n_hip:
                    raise RuntimeError(f"{n_hip} molecule(s) failed on the device (a team exchange timed out)")
        return y1, dl, nfe, status

    def _integrate(self, y0, f, e, t0, t1, opts: SolveOptions, divergence: int):
        B = y0.shape[0]
        y1 = torch.empty_like(y0)
        dl = torch.empty(B, device=self.device, dtype=torch.float32) if divergence != _lib.DIV_NONE else None
        nfe = torch.empty(B, device=self.device, dtype=torch.int32)
        status = torch.empty(B, device=self.device, dtype=torch.int32)
        o = opts.to_c(t0, t1, divergence)
        # the exact trace's primal-aggregate cache and the adaptive solves' re-deal scratch: a caller-owned workspace
        # from torch's stream-ordered caching allocator (ecnf_integrate_ws), so concurrent solves on one handle never
        # share it and the call allocates nothing itself
        nbytes = ctypes.c_size_t(0)
        _lib.check(self.lib.ecnf_integrate_workspace_size(self._h, ctypes.byref(o), B, ctypes.byref(nbytes)))
        ws = torch.empty(nbytes.value, device=self.device, dtype=torch.uint8) if nbytes.value else None
        _lib.check(self.lib.ecnf_integrate_ws(self._h, ctypes.byref(o), _ptr(y0), _ptr(f), _ptr(e), _ptr(y1), _ptr(dl),
                                              _ptr(nfe), _ptr(status), B, _ptr(ws), nbytes.value,
                                              _stream(self.device)))
        return y1, dl, nfe, status

    def set_exact_form(self, form: str) -> None:
        """A/B diagnostic of the exact trace (ecnf_set_exact_form): 'default' (sparse blocks 1 and K with the cached
        primal aggregates), 'all_dual' (every edge tile carries a tangent) or 'sparse' (no cache)."""
        forms = {"default": _lib.EXACT_FORM_DEFAULT, "all_dual": _lib.EXACT_FORM_ALL_DUAL,
                 "sparse": _lib.EXACT_FORM_SPARSE}
        _lib.check(self.lib.ecnf_set_exact_form(self._h, forms[form]))

    def set_team(self, mode: int = 0) -> None:
        """Team (latency) mode of the primal solves (ecnf_set_team): 0 auto, 1 off, G >= 2 workgroups per molecule."""
        _lib.check(self.lib.ecnf_set_team(self._h, int(mode)))

    def team_workgroups(self, batch: int, with_tangent: bool = False) -> int:
        """Workgroups per molecule a solve of `batch` molecules would use (1: the batch path)."""
        g = ctypes.c_int32()
        _lib.check(self.lib.ecnf_team_workgroups(self._h, int(with_tangent), int(batch), ctypes.byref(g)))
        return g.value

    def integrate_plan(self, batch: int, t0: float, t1: float, opts: "SolveOptions",
                       divergence: int = _lib.DIV_NONE) -> Tuple[int, int]:
        """(workgroups of the first launch, launches) of a solve given a workspace of ecnf_integrate_workspace_size
        bytes (ecnf_integrate_plan; 2 launches: the chunked, re-dealt adaptive solve)."""
        o = opts.to_c(t0, t1, divergence)
        wg, nl = ctypes.c_int32(), ctypes.c_int32()
        _lib.check(self.lib.ecnf_integrate_plan(self._h, ctypes.byref(o), int(batch), ctypes.byref(wg), ctypes.byref(nl)))
        return wg.value, nl.value

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
