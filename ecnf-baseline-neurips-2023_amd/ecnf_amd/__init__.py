"""ecnf_amd — MI355X-native equivariant-CNF sample / log_prob path (reference: Kalyan0821/ecnf-baseline-neurips-2023).

The compute path is libecnf_hip.so (hand-written CDNA4 kernels, include/ecnf.h) driven through ctypes; torch
supplies device memory, streams and torch.distributed (RCCL) only.
"""
from .params import CONFIGS, CNFConfig, flatten_params, init_params, param_count, param_spec, unflatten_params

__all__ = [
    "CONFIGS", "CNFConfig", "flatten_params", "init_params", "param_count", "param_spec", "unflatten_params",
]


def __getattr__(name):
    # torch-dependent modules load lazily so that the layout helpers import without a GPU stack
    if name in ("cnf", "engine", "distributed", "targets", "dataio", "train"):
        import importlib
        return importlib.import_module(f".{name}", __name__)
    raise AttributeError(name)
