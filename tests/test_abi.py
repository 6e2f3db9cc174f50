"""CPU tests of the C-ABI boundary (include/ecnf.h): the library loads, exports every declared symbol, agrees with
the Python/oracle parameter layout, and rejects bad arguments with status codes (no GPU compute here)."""
import ctypes
import os
import re
import subprocess
import sys

import numpy as np
import pytest

from ecnf_amd import CONFIGS, CNFConfig, _lib, param_count, param_spec
from oracle import ecnf_oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "ecnf.h")


def _c(cfg: CNFConfig, **over):
    d = dict(n_nodes=cfg.n_nodes, dim=cfg.dim, n_features=cfg.n_features, hidden=cfg.hidden,
             time_embedding_dim=cfg.time_embedding_dim, mlp_width=cfg.mlp_width, mlp_depth=cfg.mlp_depth,
             n_blocks=cfg.n_blocks, base_scale=cfg.base_scale, normalization_constant=1.0)
    d.update(over)
    return _lib.EcnfCfg(**d)


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(_lib.LIB_PATH):
        pytest.fail("libecnf_hip.so is not built: run __graft_entry__.build()")
    return _lib.load()


def test_exports_every_declared_symbol(lib):
    text = open(HEADER).read()
    declared = set(re.findall(r"^\s*(?:int|const char\*)\s+(ecnf_\w+)\s*\(", text, re.M))
    assert declared == set(_lib.EXPORTED_SYMBOLS)
    nm = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (ecnf_\w+)", nm))
    assert declared <= exported, declared - exported
    assert lib.ecnf_abi_version() == 3


def _ctypes_layout(cls):
    return ctypes.sizeof(cls), [getattr(cls, f).offset for f, _ in cls._fields_]


def test_struct_layouts_match_the_library(lib):
    """The ctypes mirrors in ecnf_amd/_lib.py have the compiled library's sizeof and field offsets."""
    for which, cls in enumerate(_lib.ABI_STRUCTS):
        assert _ctypes_layout(cls) == _lib.struct_layout(which), cls.__name__
    assert lib.ecnf_struct_layout(7, None, 0) == -1


def test_integration_md_stub_matches_the_library(lib):
    """Every ctypes.Structure in INTEGRATION.md's code blocks (the reference-side binding a maintainer would paste)
    is executed and compared with the library's layout of the struct it mirrors (matched by its `# ecnf_*` comment)."""
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    blocks = re.findall(r"```python\n(.*?)```", text, re.S)
    src = "\n".join(blocks)
    structs = re.findall(r"^(class (\w+)\(ctypes\.Structure\):\s*# (ecnf_\w+)\n(?:[ \t]+.*\n)+)", src, re.M)
    names = {c_name: (py_name, body) for body, py_name, c_name in structs}
    which = {"ecnf_cfg": 0, "ecnf_solve_opts": 1, "ecnf_target": 2, "ecnf_adam_opts": 3}
    assert set(names) == set(which), sorted(names)
    for c_name, (py_name, body) in names.items():
        ns = {"ctypes": ctypes}
        exec(body, ns)
        assert _ctypes_layout(ns[py_name]) == _lib.struct_layout(which[c_name]), c_name
        # field names as in include/ecnf.h (and _lib.py)
        assert [f for f, _ in ns[py_name]._fields_] == [f for f, _ in _lib.ABI_STRUCTS[which[c_name]]._fields_]


@pytest.mark.parametrize("name", list(CONFIGS))
def test_param_count_agrees(lib, name):
    cfg = CONFIGS[name]
    n = ctypes.c_size_t()
    assert lib.ecnf_param_count(ctypes.byref(_c(cfg)), ctypes.byref(n)) == _lib.ECNF_OK
    assert n.value == param_count(cfg) == O.param_count(O.CONFIGS[name])
    assert [p for p, _ in param_spec(cfg)] == [p for p, _ in O.param_spec(O.CONFIGS[name])]


@pytest.mark.parametrize("over,code", [
    (dict(mlp_width=96), _lib.ECNF_E_UNSUPPORTED),
    (dict(n_nodes=1), _lib.ECNF_E_UNSUPPORTED),
    (dict(n_nodes=65), _lib.ECNF_E_UNSUPPORTED),
    (dict(dim=4), _lib.ECNF_E_UNSUPPORTED),
    (dict(hidden=48), _lib.ECNF_E_UNSUPPORTED),
    (dict(time_embedding_dim=7), _lib.ECNF_E_UNSUPPORTED),
    (dict(mlp_depth=5), _lib.ECNF_E_UNSUPPORTED),
    (dict(n_blocks=11), _lib.ECNF_E_UNSUPPORTED),
    (dict(n_features=0), _lib.ECNF_E_INVALID),
    (dict(base_scale=0.0), _lib.ECNF_E_INVALID),
])
def test_rejects_bad_config(lib, over, code):
    n = ctypes.c_size_t()
    assert lib.ecnf_param_count(ctypes.byref(_c(CONFIGS["lj13"], **over)), ctypes.byref(n)) == code
    assert lib.ecnf_last_error()


def test_create_checks_blob_size_before_touching_the_device(lib):
    cfg = CONFIGS["lj13"]
    blob = np.zeros(param_count(cfg) - 1, np.float32)
    h = ctypes.c_void_p()
    rc = lib.ecnf_create(ctypes.byref(_c(cfg)), blob.ctypes.data, blob.size, 0, ctypes.byref(h))
    assert rc == _lib.ECNF_E_INVALID and b"expected" in lib.ecnf_last_error()


def test_create_without_gpu_fails_cleanly(lib):
    """No GPU here: ecnf_create must return ECNF_E_HIP (or succeed on a GPU host), never crash."""
    cfg = CONFIGS["dw4"]
    blob = np.zeros(param_count(cfg), np.float32)
    h = ctypes.c_void_p()
    rc = lib.ecnf_create(ctypes.byref(_c(cfg)), blob.ctypes.data, blob.size, 0, ctypes.byref(h))
    assert rc in (_lib.ECNF_OK, _lib.ECNF_E_HIP, _lib.ECNF_E_INVALID)
    if rc == _lib.ECNF_OK:
        assert lib.ecnf_destroy(h) == _lib.ECNF_OK


def test_null_handle_rejected(lib):
    assert lib.ecnf_vector_field(None, None, None, None, None, 1, None) == _lib.ECNF_E_INVALID
    assert lib.ecnf_integrate(None, None, None, None, None, None, None, None, None, 1, None) == _lib.ECNF_E_INVALID
    assert lib.ecnf_integrate_ws(None, None, None, None, None, None, None, None, None, 1, None, 0,
                                 None) == _lib.ECNF_E_INVALID
    n = ctypes.c_size_t()
    assert lib.ecnf_integrate_workspace_size(None, None, 1, ctypes.byref(n)) == _lib.ECNF_E_INVALID
    assert lib.ecnf_reserve_workspace(None, 16) == _lib.ECNF_E_INVALID
    assert lib.ecnf_set_exact_form(None, 0) == _lib.ECNF_E_INVALID


def test_product_path_has_no_fallback():
    """With the HIP library missing the engine raises instead of computing anything on the CPU."""
    code = ("import sys; sys.path.insert(0, %r); import os; os.environ['ECNF_LIB'] = '/nonexistent/libecnf_hip.so'\n"
            "from ecnf_amd import _lib\n"
            "try:\n    _lib.load()\nexcept FileNotFoundError:\n    print('RAISED')\n") % os.path.join(
        ROOT, "ecnf-baseline-neurips-2023_amd")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert "RAISED" in out.stdout, out.stderr
    pkg = os.path.join(ROOT, "ecnf-baseline-neurips-2023_amd", "ecnf_amd")
    for f in sorted(os.listdir(pkg)):
        if f.endswith(".py"):
            src = open(os.path.join(pkg, f)).read()
            assert "import oracle" not in src and "from oracle" not in src, f"{f} imports the oracle"


def test_flatten_roundtrip_and_shape_errors():
    cfg = CONFIGS["aldp"]
    from ecnf_amd import flatten_params, init_params, unflatten_params
    p = init_params(cfg, 3)
    blob = flatten_params(p, cfg)
    assert blob.size == param_count(cfg)
    np.testing.assert_array_equal(flatten_params(unflatten_params(blob, cfg), cfg), blob)
    nested = {"params": {"EGNN_0": {}, "Embed_0": {}}}
    for path, arr in p.items():
        d = nested["params"]
        parts = path.split("/")
        for q in parts[:-1]:
            d = d.setdefault(q, {})
        d[parts[-1]] = arr
    np.testing.assert_array_equal(flatten_params(nested, cfg), blob)
    bad = dict(p)
    bad["EGNN_0/final_scaling"] = np.ones(2, np.float32)
    with pytest.raises(ValueError):
        flatten_params(bad, cfg)
    del bad["EGNN_0/final_scaling"]
    with pytest.raises(ValueError):
        flatten_params(bad, cfg)
