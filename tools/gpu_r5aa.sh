# round 5: aggregation atomics as ds_add_f32 (opaque integer row offset) vs the flat form: first the (128, 2, 3) JVP
# reproducer on the ds form (one launch), then interleaved timing of the tangent kernels (LJ13 Hutchinson, ALDP)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5aa && export TMPDIR=/tmp && \
ECNF_LIB=tools/libt_ds1283.so timeout -k 10 120 python -u tools/diag/jvp_repro.py 1 --first > gpurun_out/r5aa/ds1283_first.log 2>&1; rc=$?
echo "== ds1283 --first rc $rc"; grep units gpurun_out/r5aa/ds1283_first.log | cut -c1-200; [ $rc -le 1 ] || exit $rc
[ $rc -eq 0 ] && { ECNF_LIB=tools/libt_ds1283.so timeout -k 10 120 python -u tools/diag/jvp_repro.py 2 > gpurun_out/r5aa/ds1283.log 2>&1; rc=$?; echo "== ds1283 full rc $rc"; grep units gpurun_out/r5aa/ds1283.log | cut -c1-120; [ $rc -eq 0 ] || exit $rc; }
TV_CASE=lj13_hutch TV_GLOB='libt_[fd][ls]*.so' timeout -k 10 240 python -u tools/time_variants.py 3 > gpurun_out/r5aa/lj13_hutch.log 2>&1 && tail -2 gpurun_out/r5aa/lj13_hutch.log && \
TV_CASE=aldp_hutch TV_GLOB='libt_a[fd][ls]*.so' timeout -k 10 240 python -u tools/time_variants.py 3 > gpurun_out/r5aa/aldp_hutch.log 2>&1 && tail -2 gpurun_out/r5aa/aldp_hutch.log && \
TV_GLOB='libt_[fd][ls]*.so' timeout -k 10 240 python -u tools/time_variants.py 2 > gpurun_out/r5aa/lj13.log 2>&1 && tail -2 gpurun_out/r5aa/lj13.log
