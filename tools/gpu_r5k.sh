# round 5: validation of the pipelined-dot build: full GPU suite, smoke, bench, rocprof evidence of the bench workload
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_r5k.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_r5k.log; [ $rc -eq 0 ] || exit $rc
bash tools/evidence.sh r5k
