# round 5: flat vs ds_add_f32 aggregation at the QM9 shape (M = 256, L = 4), interleaved A/B
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5ap && export TMPDIR=/tmp
TV_GLOB='libt_q_*.so' TV_CASE=qm9_hutch timeout -k 10 400 python -u tools/time_variants.py 3 > gpurun_out/r5ap/ab_qm9_hutch.log 2>&1 && tail -2 gpurun_out/r5ap/ab_qm9_hutch.log &&
TV_GLOB='libt_q_*.so' TV_CASE=qm9 timeout -k 10 400 python -u tools/time_variants.py 2 > gpurun_out/r5ap/ab_qm9.log 2>&1 && tail -2 gpurun_out/r5ap/ab_qm9.log
