# round-4 validation of the product build with the flat aggregation atomics: the (128, 2, 3) repro through the
# single-shape library (libt_sD) and the product library, the whole GPU suite, smoke, the bench line with its rocprof
# evidence (gpurun_out/r4n/, gpurun_out/prof_r4n/)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4n && export TMPDIR=/tmp && \
ECNF_LIB=tools/libt_sD.so timeout -k 5 90 python -u tools/repro_shapes.py 2 > gpurun_out/r4n/sD.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/r4n/sD.log | tail -4; \
[ $rc -eq 0 ] || exit $rc; grep -q "jvp ok nan" gpurun_out/r4n/sD.log && { echo "sD jvp NaN: stop"; exit 9; }; \
timeout -k 5 90 python -u tools/repro_shapes.py 2 > gpurun_out/r4n/prod.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/r4n/prod.log | tail -4; \
[ $rc -eq 0 ] || exit $rc; grep -q "jvp ok nan" gpurun_out/r4n/prod.log && { echo "product jvp NaN: stop"; exit 9; }; \
timeout -k 5 150 python -u tools/diag_small.py dw4 lj13 aldp qm9 > gpurun_out/r4n/diag.log 2>&1; rc=$?; grep -c " ok " gpurun_out/r4n/diag.log; \
[ $rc -eq 0 ] || exit $rc; \
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4n/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r4n/pytest.log; \
[ $rc -eq 0 ] || exit $rc; \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4n/smoke.log 2>&1 && cat gpurun_out/r4n/smoke.log && \
timeout -k 10 400 python -u bench.py > gpurun_out/r4n/bench.json 2> gpurun_out/r4n/bench.err && cat gpurun_out/r4n/bench.json
