# round-4 validation at HEAD (after the session restart): the whole GPU suite and smoke (gpurun_out/r4c/)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4c && export TMPDIR=/tmp && \
timeout -k 10 1050 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4c/pytest.log 2>&1; rc=$?; tail -5 gpurun_out/r4c/pytest.log; \
[ $rc -eq 0 ] && timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4c/smoke.log 2>&1; rc2=$?; cat gpurun_out/r4c/smoke.log; exit $(( rc + rc2 ))
