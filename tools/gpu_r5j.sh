# round 5: packed vs scalar fp32 activation arithmetic in the split chains (LJ13 and ALDP timing builds)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5j && export TMPDIR=/tmp && \
TV_GLOB='libt_[ns][ec]*.so' timeout -k 10 240 python -u tools/time_variants.py 3 > gpurun_out/r5j/lj13.log 2>&1 && \
TV_CASE=lj13_hutch TV_GLOB='libt_[ns][ec]*.so' timeout -k 10 240 python -u tools/time_variants.py 3 > gpurun_out/r5j/lj13_hutch.log 2>&1 && \
TV_CASE=aldp_hutch TV_GLOB='libt_a[ns][ec]*.so' timeout -k 10 240 python -u tools/time_variants.py 3 > gpurun_out/r5j/aldp_hutch.log 2>&1 && \
TV_CASE=aldp_sample TV_GLOB='libt_a[ns][ec]*.so' timeout -k 10 240 python -u tools/time_variants.py 3 > gpurun_out/r5j/aldp_sample.log 2>&1
rc=$?; tail -n 3 gpurun_out/r5j/*.log; exit $rc
