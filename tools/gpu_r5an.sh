# round 5 end state: product with the per-shape aggregation form (ds_add_f32 for M <= 64, flat for M >= 128):
# the whole GPU suite, smoke, the bench line, the ALDP paths, and the fault-study reproducer on the product
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5an && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r5an/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/r5an/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5an/smoke.log 2>&1; rc=$?
tail -2 gpurun_out/r5an/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/r5an/bench.json 2> gpurun_out/r5an/bench.err; rc=$?
tail -1 gpurun_out/r5an/bench.json | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 150 python -u tools/bench_paths.py --only aldp --reps 3 > gpurun_out/r5an/paths_aldp.log 2>&1 && grep "^{" gpurun_out/r5an/paths_aldp.log | cut -c1-300
timeout -k 10 150 python -u tools/diag/jvp_repro.py 3 --poison 7fc00000:3 > gpurun_out/r5an/product_poison_sweep.log 2>&1; rc=$?
grep -c "repeatable True" gpurun_out/r5an/product_poison_sweep.log; exit $rc
