# full GPU suite on the current build, then the exact-trace A/B (tools/exp_x2.sh)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "exact" -v -s --timeout 200 --timeout-method thread > gpurun_out/pytest_x3a.log 2>&1
rc=$?; grep -E "sparse vs|passed|failed|rror" gpurun_out/pytest_x3a.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_x3.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|rror" gpurun_out/pytest_x3.log | tail -5; [ $rc -eq 0 ] || exit $rc
bash tools/exp_x2.sh
