# round 5 end state: aggregation ds_add_f32 at M = 64 / 256, flat at M = 128: the whole GPU suite (with the
# stale-register test), smoke, the bench line, the ALDP and QM9 paths
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5aq && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r5aq/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/r5aq/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5aq/smoke.log 2>&1; rc=$?
tail -1 gpurun_out/r5aq/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/r5aq/bench.json 2> gpurun_out/r5aq/bench.err; rc=$?
tail -1 gpurun_out/r5aq/bench.json | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 150 python -u tools/bench_paths.py --only aldp --reps 3 > gpurun_out/r5aq/paths_aldp.log 2>&1 && grep "^{" gpurun_out/r5aq/paths_aldp.log | cut -c1-200
timeout -k 10 400 python -u tools/bench_paths.py --only qm9 --reps 2 > gpurun_out/r5aq/paths_qm9.log 2>&1; grep "^{" gpurun_out/r5aq/paths_qm9.log | cut -c1-200
