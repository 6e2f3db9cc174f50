# round-4 end: the whole GPU suite and smoke on the final tree (gpurun_out/r4v/)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4v && export TMPDIR=/tmp && \
timeout -k 5 150 python -u tools/diag_small.py dw4 lj13 aldp qm9 > gpurun_out/r4v/diag.log 2>&1 && grep -c " ok " gpurun_out/r4v/diag.log && \
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4v/pytest.log 2>&1 && tail -2 gpurun_out/r4v/pytest.log && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4v/smoke.log 2>&1 && cat gpurun_out/r4v/smoke.log
