"""ctypes binding of libecnf_hip.so (C-ABI declared in include/ecnf.h).

The library is built in-tree by ``__graft_entry__.build()`` (hipcc --offload-arch=gfx950) next to this file.
There is no fallback: if the library is missing or fails to load, every entry point raises.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

LIB_NAME = "libecnf_hip.so"
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)

ECNF_OK, ECNF_E_INVALID, ECNF_E_UNSUPPORTED, ECNF_E_HIP, ECNF_E_MAX_STEPS, ECNF_E_NONFINITE = 0, 1, 2, 3, 4, 5
PREC_SPLIT_F16, PREC_FP32 = 0, 1
SOLVER_EULER, SOLVER_DOPRI5 = 0, 1
DIV_NONE, DIV_HUTCHINSON, DIV_EXACT = 0, 1, 2
CHAIN_FP32_MFMA, CHAIN_SPLIT_BF16, CHAIN_SPLIT_F16 = 0, 1, 2
EXACT_FORM_DEFAULT, EXACT_FORM_ALL_DUAL, EXACT_FORM_SPARSE = 0, 1, 2

# every symbol include/ecnf.h declares
EXPORTED_SYMBOLS = (
    "ecnf_abi_version", "ecnf_last_error", "ecnf_param_count", "ecnf_create", "ecnf_destroy",
    "ecnf_vector_field", "ecnf_vf_jvp", "ecnf_integrate", "ecnf_base_sample", "ecnf_base_log_prob",
    "ecnf_molecules_per_workgroup", "ecnf_chain_arithmetic", "ecnf_target_log_prob", "ecnf_lse_partials",
    "ecnf_set_precision", "ecnf_get_precision", "ecnf_trainer_create", "ecnf_trainer_destroy", "ecnf_fm_loss_grad",
    "ecnf_adam_update", "ecnf_update_params", "ecnf_integrate_workspace_size", "ecnf_integrate_ws",
    "ecnf_reserve_workspace", "ecnf_set_exact_form", "ecnf_struct_layout", "ecnf_trainer_set_reduction_arena",
    "ecnf_set_team", "ecnf_team_workgroups", "ecnf_integrate_plan",
)

TARGET_LJ, TARGET_DW = 0, 1


class EcnfCfg(ctypes.Structure):
    _fields_ = [
        ("n_nodes", ctypes.c_int32),
        ("dim", ctypes.c_int32),
        ("n_features", ctypes.c_int32),
        ("hidden", ctypes.c_int32),
        ("time_embedding_dim", ctypes.c_int32),
        ("mlp_width", ctypes.c_int32),
        ("mlp_depth", ctypes.c_int32),
        ("n_blocks", ctypes.c_int32),
        ("base_scale", ctypes.c_float),
        ("normalization_constant", ctypes.c_float),
    ]


class EcnfSolveOpts(ctypes.Structure):
    _fields_ = [
        ("solver", ctypes.c_int32),
        ("divergence", ctypes.c_int32),
        ("t0", ctypes.c_float),
        ("t1", ctypes.c_float),
        ("dt0", ctypes.c_float),
        ("rtol", ctypes.c_float),
        ("atol", ctypes.c_float),
        ("dtmin", ctypes.c_float),
        ("max_steps", ctypes.c_int32),
    ]


class EcnfTarget(ctypes.Structure):
    _fields_ = [
        ("kind", ctypes.c_int32),
        ("n_nodes", ctypes.c_int32),
        ("dim", ctypes.c_int32),
        ("epsilon", ctypes.c_float),
        ("tau", ctypes.c_float),
        ("r", ctypes.c_float),
        ("harmonic_coef", ctypes.c_float),
        ("a", ctypes.c_float),
        ("b", ctypes.c_float),
        ("c", ctypes.c_float),
        ("d0", ctypes.c_float),
        ("r_nodes", ctypes.c_void_p),
    ]


class EcnfAdamOpts(ctypes.Structure):
    _fields_ = [
        ("lr", ctypes.c_float),
        ("b1", ctypes.c_float),
        ("b2", ctypes.c_float),
        ("eps", ctypes.c_float),
        ("eps_root", ctypes.c_float),
        ("count", ctypes.c_int32),
        ("ema_beta", ctypes.c_float),
    ]


# the ABI structs in ecnf_struct_layout's `which` order
ABI_STRUCTS = (EcnfCfg, EcnfSolveOpts, EcnfTarget, EcnfAdamOpts)


def struct_layout(which: int):
    """(sizeof, [field offsets]) of ABI struct `which` as the compiled library lays it out."""
    buf = (ctypes.c_size_t * 16)()
    n = load().ecnf_struct_layout(which, buf, 16)
    if n < 0:
        raise ValueError(f"unknown struct {which}")
    return buf[0], list(buf[1:1 + n])


class EcnfError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"ecnf error {code}: {msg}")
        self.code = code


class EcnfInvalid(EcnfError, ValueError):
    pass


_lib: Optional[ctypes.CDLL] = None


def load(path: Optional[str] = None) -> ctypes.CDLL:
    """Load (once) and type the C-ABI.  Raises FileNotFoundError / OSError when the HIP library is absent."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("ECNF_LIB", LIB_PATH)
    if not os.path.exists(path):
        raise FileNotFoundError(
            f"{path} not found: build the HIP library first (python -c 'import __graft_entry__ as g; g.build()')")
    lib = ctypes.CDLL(path)
    P, I32, SZ = ctypes.c_void_p, ctypes.c_int32, ctypes.c_size_t
    sig = {
        "ecnf_abi_version": ([], ctypes.c_int),
        "ecnf_last_error": ([], ctypes.c_char_p),
        "ecnf_param_count": ([ctypes.POINTER(EcnfCfg), ctypes.POINTER(SZ)], ctypes.c_int),
        "ecnf_create": ([ctypes.POINTER(EcnfCfg), P, SZ, ctypes.c_int, ctypes.POINTER(P)], ctypes.c_int),
        "ecnf_destroy": ([P], ctypes.c_int),
        "ecnf_vector_field": ([P, P, P, P, P, I32, P], ctypes.c_int),
        "ecnf_vf_jvp": ([P, P, P, P, P, I32, P, P, I32, P], ctypes.c_int),
        "ecnf_integrate": ([P, ctypes.POINTER(EcnfSolveOpts), P, P, P, P, P, P, P, I32, P], ctypes.c_int),
        "ecnf_base_sample": ([P, P, P, I32, P], ctypes.c_int),
        "ecnf_base_log_prob": ([P, P, P, I32, P], ctypes.c_int),
        "ecnf_molecules_per_workgroup": ([P, I32, ctypes.POINTER(I32)], ctypes.c_int),
        "ecnf_chain_arithmetic": ([P, I32, ctypes.POINTER(I32)], ctypes.c_int),
        "ecnf_target_log_prob": ([ctypes.POINTER(EcnfTarget), P, P, I32, P], ctypes.c_int),
        "ecnf_lse_partials": ([P, P, I32, P, P], ctypes.c_int),
        "ecnf_set_precision": ([P, I32], ctypes.c_int),
        "ecnf_get_precision": ([P, ctypes.POINTER(I32)], ctypes.c_int),
        "ecnf_trainer_create": ([ctypes.POINTER(EcnfCfg), I32, ctypes.c_int, ctypes.POINTER(P)], ctypes.c_int),
        "ecnf_trainer_destroy": ([P], ctypes.c_int),
        "ecnf_trainer_set_reduction_arena": ([P, SZ, ctypes.POINTER(SZ)], ctypes.c_int),
        "ecnf_fm_loss_grad": ([P, P, P, P, P, P, ctypes.c_float, I32, P, P, P], ctypes.c_int),
        "ecnf_adam_update": ([P, P, P, P, P, P, SZ, ctypes.POINTER(EcnfAdamOpts), P, P], ctypes.c_int),
        "ecnf_update_params": ([P, P, I32], ctypes.c_int),
        "ecnf_integrate_workspace_size": ([P, ctypes.POINTER(EcnfSolveOpts), I32, ctypes.POINTER(SZ)], ctypes.c_int),
        "ecnf_integrate_ws": ([P, ctypes.POINTER(EcnfSolveOpts), P, P, P, P, P, P, P, I32, P, SZ, P], ctypes.c_int),
        "ecnf_reserve_workspace": ([P, SZ], ctypes.c_int),
        "ecnf_set_exact_form": ([P, I32], ctypes.c_int),
        "ecnf_set_team": ([P, I32], ctypes.c_int),
        "ecnf_team_workgroups": ([P, I32, I32, ctypes.POINTER(I32)], ctypes.c_int),
        "ecnf_integrate_plan": ([P, ctypes.POINTER(EcnfSolveOpts), I32, ctypes.POINTER(I32), ctypes.POINTER(I32)],
                                ctypes.c_int),
        "ecnf_struct_layout": ([I32, ctypes.POINTER(SZ), I32], ctypes.c_int),
    }
    for name, (argtypes, restype) in sig.items():
        if path != LIB_PATH and not hasattr(lib, name):
            continue   # an older A/B timing build (ECNF_LIB, tools/build_timing.sh) may predate an entry point
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = restype
    _lib = lib
    return lib


def check(rc: int) -> None:
    if rc == ECNF_OK:
        return
    msg = load().ecnf_last_error().decode(errors="replace")
    if rc in (ECNF_E_INVALID, ECNF_E_UNSUPPORTED):
        raise EcnfInvalid(rc, msg)
    raise EcnfError(rc, msg)
