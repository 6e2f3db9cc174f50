# round 5: flat vs ds_add_f32 aggregation atomics in the product source (tools/diag/ds_agg_variants.py form, both
# sites), LJ13-only and ALDP-shape builds, interleaved A/B (tools/time_variants.py)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5am && export TMPDIR=/tmp
TV_GLOB='libt_ab_*_lj.so' TV_CASE=lj13_hutch timeout -k 10 240 python -u tools/time_variants.py 4 > gpurun_out/r5am/ab_lj13_hutch.log 2>&1 && tail -2 gpurun_out/r5am/ab_lj13_hutch.log &&
TV_GLOB='libt_ab_*_lj.so' TV_CASE=lj13 timeout -k 10 240 python -u tools/time_variants.py 3 > gpurun_out/r5am/ab_lj13.log 2>&1 && tail -2 gpurun_out/r5am/ab_lj13.log &&
TV_GLOB='libt_ab_*_aldp.so' TV_CASE=aldp_hutch timeout -k 10 240 python -u tools/time_variants.py 4 > gpurun_out/r5am/ab_aldp_hutch.log 2>&1 && tail -2 gpurun_out/r5am/ab_aldp_hutch.log &&
TV_GLOB='libt_ab_*_aldp.so' TV_CASE=aldp_sample timeout -k 10 240 python -u tools/time_variants.py 3 > gpurun_out/r5am/ab_aldp_sample.log 2>&1 && tail -2 gpurun_out/r5am/ab_aldp_sample.log
