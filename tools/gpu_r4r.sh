# round-4 final: the product build with the 8-wave column-split kernel (ECNF_COLS_NW = 8).  Small solves of every
# config (a fault stops the call), the QM9 team probe, the whole GPU suite, smoke, the default bench line and the
# rocprofv3 evidence of the bench workload (gpurun_out/r4r/, gpurun_out/prof_r4r/)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4r && export TMPDIR=/tmp && \
timeout -k 5 150 python -u tools/diag_small.py dw4 lj13 aldp qm9 > gpurun_out/r4r/diag.log 2>&1 && grep -c " ok " gpurun_out/r4r/diag.log && \
TP_MODES=1,0,7 timeout -k 10 150 python -u tools/team_probe.py qm9 1 4 9 > gpurun_out/r4r/team_qm9.log 2>&1 && tail -c 400 gpurun_out/r4r/team_qm9.log && \
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4r/pytest.log 2>&1 && tail -3 gpurun_out/r4r/pytest.log && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4r/smoke.log 2>&1 && cat gpurun_out/r4r/smoke.log && \
timeout -k 10 600 python -u bench.py > gpurun_out/r4r/bench.json 2> gpurun_out/r4r/bench.err && cat gpurun_out/r4r/bench.json && \
bash tools/profile_round.sh r4r
