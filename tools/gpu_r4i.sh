# round-4 perf evidence with the column-split team mode: small solves of every config (a fault stops the call), the
# halves-mode A/B (LJ13 primal, ALDP PID sample), the default bench line, the rocprof evidence of the bench workload,
# then the team-mode tests (gpurun_out/r4i/, gpurun_out/prof_r4i/)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4i && export TMPDIR=/tmp && \
timeout -k 5 150 python -u tools/diag_small.py dw4 lj13 aldp qm9 > gpurun_out/r4i/diag.log 2>&1; rc=$?; grep -c " ok " gpurun_out/r4i/diag.log; \
[ $rc -eq 0 ] || { cat gpurun_out/r4i/diag.log; exit $rc; }; \
TV_GLOB='libt_h*.so' timeout -k 10 200 python -u tools/time_variants.py 4 > gpurun_out/r4i/ab_lj13.log 2>&1 && tail -2 gpurun_out/r4i/ab_lj13.log && \
TV_CASE=aldp_sample TV_GLOB='libt_a*.so' timeout -k 10 200 python -u tools/time_variants.py 4 > gpurun_out/r4i/ab_aldps.log 2>&1 && tail -2 gpurun_out/r4i/ab_aldps.log && \
timeout -k 10 420 python -u bench.py > gpurun_out/r4i/bench.json 2> gpurun_out/r4i/bench.err && cat gpurun_out/r4i/bench.json && \
bash tools/profile_round.sh r4i && python tools/pmc_summary.py gpurun_out/prof_r4i gpurun_out/r4i/pmc.json && cat gpurun_out/r4i/pmc.json && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_team.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r4i/pytest_team.log 2>&1; rc=$?; tail -3 gpurun_out/r4i/pytest_team.log; exit $rc
