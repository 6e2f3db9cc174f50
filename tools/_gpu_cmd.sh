cd $GRAFT_REPO_ROOT && timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest.log 2>&1; tail -5 gpurun_out/pytest.log; \
timeout -k 10 200 python -u bench.py --cpu-molecules 0 > gpurun_out/bench.json 2>gpurun_out/bench.err; cat gpurun_out/bench.json | cut -c1-400
