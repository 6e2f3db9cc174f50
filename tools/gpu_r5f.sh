# round 5: interleaved A/B of the round-4 source vs HEAD (LJ13-only timing builds), the RCCL test, the ALDP tail study
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5f && export TMPDIR=/tmp && \
timeout -k 10 300 python -u tools/time_variants.py 3 > gpurun_out/r5f/ab_lj13.log 2>&1; rc=$?; tail -3 gpurun_out/r5f/ab_lj13.log; [ $rc -eq 0 ] || exit $rc; \
timeout -k 10 300 python -u -m pytest tests/test_gpu_rccl.py -x -v --timeout 280 --timeout-method thread > gpurun_out/r5f/rccl.log 2>&1; rc=$?; tail -3 gpurun_out/r5f/rccl.log; [ $rc -eq 0 ] || exit $rc; \
timeout -k 10 300 python -u tools/diag/aldp_tail.py > gpurun_out/r5f/aldp_tail.log 2>&1; rc=$?; cat gpurun_out/r5f/aldp_tail.log | grep -v amdgpu.ids; exit $rc
