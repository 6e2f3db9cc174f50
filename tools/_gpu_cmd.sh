cd $GRAFT_REPO_ROOT && timeout -k 10 500 python tools/time_variants.py 3 2>&1 | tail -2 && \
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest.log 2>&1; tail -5 gpurun_out/pytest.log
