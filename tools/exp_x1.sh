# exact-trace block-1 sparse dual tiles: parity, then the A/B timing of the LJ13 exact log_prob (B = 1024, Euler-100)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "exact_sparse" -v -s --timeout 200 --timeout-method thread > gpurun_out/pytest_x1a.log 2>&1
rc=$?; grep -E "sparse vs|oracle|passed|failed|Error" gpurun_out/pytest_x1a.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_device_checks.py tests/test_gpu_invariance_jacobian.py tests/test_gpu_cnf_api.py tests/test_gpu_qm9_divergence.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_x1.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_x1.log | tail -8; [ $rc -eq 0 ] || exit $rc
ECNF_PATHS_ONLY=lj13 ECNF_PATHS_DIV=exact ECNF_EXACT_SPARSE=0 timeout -k 10 120 python -u tools/bench_paths.py gpurun_out/px_dense.json &&
ECNF_PATHS_ONLY=lj13 ECNF_PATHS_DIV=exact timeout -k 10 120 python -u tools/bench_paths.py gpurun_out/px_sparse.json &&
ECNF_PATHS_ONLY=lj13 ECNF_PATHS_DIV=exact ECNF_EXACT_SPARSE=0 timeout -k 10 120 python -u tools/bench_paths.py gpurun_out/px_dense2.json &&
ECNF_PATHS_ONLY=lj13 ECNF_PATHS_DIV=exact timeout -k 10 120 python -u tools/bench_paths.py gpurun_out/px_sparse2.json
