# round-4 combined validation at HEAD: the whole GPU suite and smoke, the halves-mode A/B (LJ13 primal, ALDP PID
# sample), the default bench line and the rocprof evidence of the bench workload (gpurun_out/r4e/, prof_r4e/)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4e && export TMPDIR=/tmp && \
timeout -k 10 240 python -u -c "import torch; print('torch', torch.__version__, flush=True); torch.zeros(1, device='cuda'); print('gpu ok', flush=True)" && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4e/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r4e/pytest.log; \
[ $rc -eq 0 ] || exit $rc; \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4e/smoke.log 2>&1 && cat gpurun_out/r4e/smoke.log && \
TV_GLOB='libt_h*.so' timeout -k 10 200 python -u tools/time_variants.py 4 > gpurun_out/r4e/ab_lj13.log 2>&1 && tail -2 gpurun_out/r4e/ab_lj13.log && \
TV_CASE=aldp_sample TV_GLOB='libt_a*.so' timeout -k 10 200 python -u tools/time_variants.py 4 > gpurun_out/r4e/ab_aldps.log 2>&1 && tail -2 gpurun_out/r4e/ab_aldps.log && \
timeout -k 10 420 python -u bench.py > gpurun_out/r4e/bench.json 2> gpurun_out/r4e/bench.err && cat gpurun_out/r4e/bench.json && \
bash tools/profile_round.sh r4e && python tools/pmc_summary.py gpurun_out/prof_r4e gpurun_out/r4e/pmc.json && cat gpurun_out/r4e/pmc.json
