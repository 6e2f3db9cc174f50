#!/bin/bash
# One GPU call: parity tests, smoke, bench line, then the rocprof evidence (tools/profile_round.sh).
# Usage (from gpurun): bash tools/gpu_check.sh TAG
TAG=${1:-r01}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v -s --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo "smoke failed"; cat gpurun_out/smoke_$TAG.log; exit 1; }
cat gpurun_out/smoke_$TAG.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
[ "$2" = "noprof" ] && exit 0
bash tools/profile_round.sh $TAG && python tools/pmc_summary.py gpurun_out/prof_$TAG gpurun_out/pmc_$TAG.json && cat gpurun_out/pmc_$TAG.json
