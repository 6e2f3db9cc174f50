#!/bin/bash
# One GPU call: smoke, the default bench line, and the rocprof evidence of the bench workload (tools/profile_round.sh).
# Usage (from gpurun): bash tools/evidence.sh TAG
TAG=${1:-final}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { cat gpurun_out/smoke_$TAG.log; exit 1; }
cat gpurun_out/smoke_$TAG.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
bash tools/profile_round.sh $TAG && python tools/pmc_summary.py gpurun_out/prof_$TAG gpurun_out/pmc_$TAG.json && cat gpurun_out/pmc_$TAG.json
