# round-4 validation after the LDS-pointer fix and the monotonic halves barrier: small solves of every config first (a fault stops the call), then the
# whole GPU suite, smoke, the halves-mode A/B (LJ13 primal, ALDP PID sample), the default bench line and the rocprof
# evidence of the bench workload (gpurun_out/r4h/, gpurun_out/prof_r4h/)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4h && export TMPDIR=/tmp && \
timeout -k 5 150 python -u tools/diag_small.py dw4 lj13 aldp qm9 > gpurun_out/r4h/diag.log 2>&1; rc=$?; cat gpurun_out/r4h/diag.log | grep -v amdgpu.ids; \
[ $rc -eq 0 ] || exit $rc; \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4h/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r4h/pytest.log; \
[ $rc -eq 0 ] || exit $rc; \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4h/smoke.log 2>&1 && cat gpurun_out/r4h/smoke.log && \
TV_GLOB='libt_h*.so' timeout -k 10 200 python -u tools/time_variants.py 4 > gpurun_out/r4h/ab_lj13.log 2>&1 && tail -2 gpurun_out/r4h/ab_lj13.log && \
TV_CASE=aldp_sample TV_GLOB='libt_a*.so' timeout -k 10 200 python -u tools/time_variants.py 4 > gpurun_out/r4h/ab_aldps.log 2>&1 && tail -2 gpurun_out/r4h/ab_aldps.log && \
timeout -k 10 420 python -u bench.py > gpurun_out/r4h/bench.json 2> gpurun_out/r4h/bench.err && cat gpurun_out/r4h/bench.json && \
bash tools/profile_round.sh r4h && python tools/pmc_summary.py gpurun_out/prof_r4h gpurun_out/r4h/pmc.json && cat gpurun_out/r4h/pmc.json
