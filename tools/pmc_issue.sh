#!/bin/bash
# Issue / stall counters of the bench workload's integrate_kernel (LJ13 B=1024 Euler NFE=100), one rocprofv3 --pmc pass
# (8 SQ counters, no tracing domains): wave cycles split into active / issue-stalled / parked (MI355X_MICROARCH.md
# SQ table) and the VALU-MFMA co-execution.  Usage: tools/pmc_issue.sh TAG  -> gpurun_out/prof_TAG/issue/
TAG=${1:-r4}
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT="$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
B="bench.py --steps 2 --warmup 1 --cpu-molecules 0 --fp32-steps 0 --train-steps 0 --ref-latency-samples 0 --pmc 0 --logprob 0"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --kernel-include-regex integrate_kernel -d "$OUT/issue" -o run --output-format csv -- python3 $B > "$OUT/issue.log" 2>&1 || exit $?
echo "issue pass ok"
