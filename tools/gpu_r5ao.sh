# round 5: the poisoned-register GPU test (tests/test_gpu_uninit.py) on the product
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5ao && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_uninit.py -x -v --timeout 240 --timeout-method thread > gpurun_out/r5ao/pytest_uninit.log 2>&1; rc=$?
grep -E "PASS|FAIL|passed|failed|Error" gpurun_out/r5ao/pytest_uninit.log | head -20; exit $rc
