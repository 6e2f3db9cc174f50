"""Sanitizer runs of the host side of the C-ABI ("-fsanitize=address host build of the C++
stepper").  tools/asan/build.sh instruments the host translation units of libecnf_hip.so with AddressSanitizer
(host pass only; device code is not instrumented) and builds tools/asan/abi_asan.cpp, which drives every entry point
of include/ecnf.h: argument checks, the ravel_pytree param walk and the split-fragment repacking of ecnf_create on
the CPU; on a GPU also one small call of each compute entry point and the error paths behind a valid handle.

ASan aborts the process with a report on any heap / stack / use-after-scope error.  LeakSanitizer runs in both tests
as a scoped check at the end of the driver's main (__lsan_do_recoverable_leak_check, with the ROCm runtime's own
allocations suppressed by tools/asan/lsan.supp) instead of at process exit (leak_check_at_exit=0): the exit-time scan
of a GPU process also walks the HIP runtime's teardown, and the driver reports how long the scoped scan took."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASAN_DIR = os.path.join(ROOT, "tools", "asan")
EXE = os.path.join(ASAN_DIR, "abi_asan")
OBJ_DIR = os.path.join(ROOT, "ecnf-baseline-neurips-2023_amd", "build")


def _env():
    supp = os.path.join(ASAN_DIR, "lsan.supp")
    return dict(os.environ, ABI_ASAN_TRACE="1",
                ASAN_OPTIONS="detect_leaks=1:leak_check_at_exit=0:abort_on_error=0:halt_on_error=1:"
                             "detect_stack_use_after_return=1",
                LSAN_OPTIONS=f"suppressions={supp}:print_suppressions=0")


def _ensure_built():
    srcs = [os.path.join(ASAN_DIR, "abi_asan.cpp"), os.path.join(ASAN_DIR, "build.sh")]
    fresh = os.path.exists(EXE) and all(os.path.getmtime(EXE) >= os.path.getmtime(s) for s in srcs)
    if fresh:
        return
    if not os.path.isdir(OBJ_DIR) or not any(f.startswith("ecnf_part_") for f in os.listdir(OBJ_DIR)):
        pytest.skip("kernel objects not built (run __graft_entry__.build() first)")
    r = subprocess.run(["bash", os.path.join(ASAN_DIR, "build.sh")], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]


def _run(timeout=300):
    try:
        r = subprocess.run([EXE], capture_output=True, text=True, timeout=timeout, env=_env())
    except subprocess.TimeoutExpired as e:   # ABI_ASAN_TRACE names the last check that started
        err = e.stderr.decode() if isinstance(e.stderr, bytes) else (e.stderr or "")
        pytest.fail(f"abi_asan did not finish in {timeout} s; stderr tail:\n{err[-3000:]}")
    out = r.stdout + r.stderr
    assert "ERROR: AddressSanitizer" not in out and "ERROR: LeakSanitizer" not in out, out[-4000:]
    assert r.returncode == 0, out[-4000:]
    return out


def test_asan_host_paths():
    """CPU: argument validation, param walk and repacking under ASan (ecnf_create stops at the first device call)."""
    _ensure_built()
    out = _run()
    assert "0 failure(s)" in out and "leak check clean" in out, out[-2000:]


@pytest.mark.gpu
def test_asan_device_paths():
    """GPU box: the prebuilt ASan driver (host code instrumented) runs every entry point on the device."""
    if not os.path.exists(EXE):
        pytest.fail("tools/asan/abi_asan is not built: run tools/asan/build.sh")
    out = _run(timeout=150)
    print([ln for ln in out.splitlines() if "leak check" in ln])
    assert "host + device paths" in out and "0 failure(s)" in out and "leak check clean" in out, out[-2000:]
