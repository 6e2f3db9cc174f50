# round-4: A/B of halves mode on / off (LJ13 B=1024 Euler-100 primal, ALDP B=512 PID sample), then the default
# bench line and the rocprof evidence of the bench workload (gpurun_out/r4d/, gpurun_out/prof_r4d/)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4d && export TMPDIR=/tmp && \
TV_GLOB='libt_h*.so' timeout -k 10 300 python -u tools/time_variants.py 5 > gpurun_out/r4d/ab_lj13.log 2>&1 && tail -2 gpurun_out/r4d/ab_lj13.log && \
TV_CASE=aldp_sample TV_GLOB='libt_a*.so' timeout -k 10 300 python -u tools/time_variants.py 5 > gpurun_out/r4d/ab_aldps.log 2>&1 && tail -2 gpurun_out/r4d/ab_aldps.log && \
timeout -k 10 600 python -u bench.py > gpurun_out/r4d/bench.json 2> gpurun_out/r4d/bench.err && cat gpurun_out/r4d/bench.json && \
bash tools/profile_round.sh r4d && python tools/pmc_summary.py gpurun_out/prof_r4d gpurun_out/r4d/pmc.json && cat gpurun_out/r4d/pmc.json
