# round-4 evidence at the product build (halves off, column-split team mode): small solves of every config (a fault
# stops the call), the team-mode tests, the default bench line (incl. the reference-latency leg), the rocprof evidence
# of the bench workload (gpurun_out/r4j/, gpurun_out/prof_r4j/)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4j && export TMPDIR=/tmp && \
timeout -k 5 150 python -u tools/diag_small.py dw4 lj13 aldp qm9 > gpurun_out/r4j/diag.log 2>&1; rc=$?; grep -c " ok " gpurun_out/r4j/diag.log; \
[ $rc -eq 0 ] || { cat gpurun_out/r4j/diag.log; exit $rc; }; \
timeout -k 10 300 python -u -m pytest tests/test_gpu_team.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r4j/pytest_team.log 2>&1; rc=$?; tail -3 gpurun_out/r4j/pytest_team.log; \
timeout -k 10 200 python -u tools/team_probe.py qm9 1 4 9 > gpurun_out/r4j/team_qm9.log 2>&1; tail -c 1500 gpurun_out/r4j/team_qm9.log; \
timeout -k 10 420 python -u bench.py > gpurun_out/r4j/bench.json 2> gpurun_out/r4j/bench.err && cat gpurun_out/r4j/bench.json && \
bash tools/profile_round.sh r4j && python tools/pmc_summary.py gpurun_out/prof_r4j gpurun_out/r4j/pmc.json && cat gpurun_out/r4j/pmc.json; exit $rc
