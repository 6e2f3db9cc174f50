cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
for b in tools/micro/sb_*; do echo $b; timeout -k 5 60 $b || exit 1; done; \
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_f16.log 2>&1; tail -4 gpurun_out/pytest_f16.log; \
timeout -k 10 200 python -u bench.py --cpu-molecules 0 > gpurun_out/bench_f16.json 2>gpurun_out/bench_f16.err; cat gpurun_out/bench_f16.json
