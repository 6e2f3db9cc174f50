cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest.log 2>&1; tail -3 gpurun_out/pytest.log; \
timeout -k 10 300 python -u tools/time_variants.py 3 2>&1 | tail -3
