# round 5: ALDP phase stamps, then the large-N tests (M = 128 wide tangent kernels at 40 / 64 atoms)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5g gpurun_out/r5h && export TMPDIR=/tmp && \
bash tools/gpu_r5g.sh && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_large_n.py -x -v --timeout 280 --timeout-method thread > gpurun_out/r5h/large_n.log 2>&1; rc=$?; tail -15 gpurun_out/r5h/large_n.log; exit $rc
