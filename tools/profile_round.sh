#!/bin/bash
# rocprofv3 evidence for the bench workload (LJ13 B=1024 Euler NFE=100):
#   1. kernel trace + stats   2. FETCH_SIZE pass   3. WRITE_SIZE pass   4. MFMA busy / clock pass
# Counter passes are separate (no tracing domains combined with --pmc).  Usage: tools/profile_round.sh TAG
TAG=${1:-r01}
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT="$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
B="bench.py --steps 3 --warmup 1 --cpu-molecules 0 --fp32-steps 0 --train-steps 0 --ref-latency-samples 0 --pmc 0"
# the kernel trace keeps the bench's Hutchinson log-prob leg (its tangent integrate_kernel<4, 1, ...> gets its own
# stats row); the counter passes profile the primal launches alone
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o run --output-format csv -- python3 $B > "$OUT/kt.log" 2>&1 || exit $?
B="$B --logprob 0"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex integrate_kernel -d "$OUT/fetch" -o run --output-format csv -- python3 $B > "$OUT/fetch.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex integrate_kernel -d "$OUT/write" -o run --output-format csv -- python3 $B > "$OUT/write.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --kernel-include-regex integrate_kernel -d "$OUT/mfma" -o run --output-format csv -- python3 $B > "$OUT/mfma.log" 2>&1 || exit $?
echo "profile ok"
