# round-4: tile-deal rotation for co-resident batch workgroups (tools/libt_rot0.so vs libt_rot1.so, LJ13 only):
# LJ13 B=1024 Euler-100 Hutchinson (the 10-tile, 4-wave tangent kernel at 2 workgroups per CU) and primal
# (gpurun_out/r4u/)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4u && export TMPDIR=/tmp && \
ECNF_LIB=tools/libt_rot1.so timeout -k 5 150 python -u tools/diag_small.py lj13 > gpurun_out/r4u/diag_rot1.log 2>&1 && grep -c " ok " gpurun_out/r4u/diag_rot1.log && \
TV_CASE=lj13_hutch TV_GLOB='libt_rot*.so' timeout -k 10 300 python -u tools/time_variants.py 3 > gpurun_out/r4u/ab_hutch.log 2>&1 && cat gpurun_out/r4u/ab_hutch.log && \
TV_GLOB='libt_rot*.so' timeout -k 10 200 python -u tools/time_variants.py 3 > gpurun_out/r4u/ab_primal.log 2>&1 && tail -2 gpurun_out/r4u/ab_primal.log
