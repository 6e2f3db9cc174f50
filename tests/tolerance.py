"""The fp32-class bound every GPU parity test applies to positions AND log-densities.

The reference runs in fp32 (x64 off, ecnf/utils/loop.py:62-63), so "parity" means: the HIP result is as close to the
exact (fp64) answer as an fp32 evaluation of the same math is.  A GPU result `got` passes when

    max |got - ref64| <= C * max |ref32 - ref64| + FLOOR * max(1, max |ref64|)

with ref64 / ref32 the numpy oracle (oracle/ecnf_oracle.py) at float64 / float32 on the same inputs.  C = 4 covers
the different summation orders of the kernels (fused MFMA accumulation, segmented DPP scans, the exact trace's sum
over N*D - D JVP columns); FLOOR covers cases where the fp32 oracle happens to land almost exactly.
"""
import numpy as np

C = 4.0
FLOOR = 2e-7


def _np(a):
    try:
        import torch
        if torch.is_tensor(a):
            return a.detach().cpu().numpy()
    except ImportError:   # pragma: no cover
        pass
    return np.asarray(a)


def fp32_class(name, got, ref64, ref32, c=C, floor=FLOOR):
    """Assert the fp32-class bound (module docstring); returns (err_hip, err_fp32) for logging."""
    got, ref64, ref32 = _np(got).astype(np.float64), _np(ref64).astype(np.float64), _np(ref32).astype(np.float64)
    assert got.shape == ref64.shape == ref32.shape, (name, got.shape, ref64.shape, ref32.shape)
    scale = max(1.0, float(np.abs(ref64).max()))
    e_hip = float(np.abs(got - ref64).max())
    e_32 = float(np.abs(ref32 - ref64).max())
    print(f"{name}: |hip - fp64| = {e_hip:.3e}, |fp32 oracle - fp64| = {e_32:.3e}, "
          f"ratio {e_hip / max(e_32, 1e-30):.2f}, bound {c * e_32 + floor * scale:.3e}")
    assert e_hip <= c * e_32 + floor * scale, (name, e_hip, e_32, scale)
    return e_hip, e_32
