# round 5: the re-dealt adaptive solves at the product build: the new test first, then the whole GPU suite, then the
# ALDP cases of bench_paths and the sched_check timing
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5s && export TMPDIR=/tmp && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_redeal.py -x -v -s --timeout 240 --timeout-method thread > gpurun_out/r5s/redeal.log 2>&1; rc=$?
grep -E "PASS|FAIL|B=|passed|failed" gpurun_out/r5s/redeal.log | head -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r5s/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/r5s/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/bench_paths.py --only aldp --reps 3 > gpurun_out/r5s/paths_aldp.log 2>&1 && grep "^{" gpurun_out/r5s/paths_aldp.log | cut -c1-300
