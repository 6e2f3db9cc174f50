# round 5: A/B of the pipelined edge-tail dots / layer-1 reads / shift reciprocal (LJ13 and ALDP timing builds)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5i && export TMPDIR=/tmp && \
TV_GLOB='libt_[hn]e*.so' timeout -k 10 240 python -u tools/time_variants.py 3 > gpurun_out/r5i/lj13.log 2>&1 && \
TV_CASE=lj13_hutch TV_GLOB='libt_[hn]e*.so' timeout -k 10 240 python -u tools/time_variants.py 3 > gpurun_out/r5i/lj13_hutch.log 2>&1 && \
TV_CASE=aldp_hutch TV_GLOB='libt_[ar][ne]*.so' timeout -k 10 240 python -u tools/time_variants.py 3 > gpurun_out/r5i/aldp_hutch.log 2>&1 && \
TV_CASE=aldp_sample TV_GLOB='libt_[ar][ne]*.so' timeout -k 10 240 python -u tools/time_variants.py 3 > gpurun_out/r5i/aldp_sample.log 2>&1
rc=$?; tail -n 3 gpurun_out/r5i/*.log; exit $rc
