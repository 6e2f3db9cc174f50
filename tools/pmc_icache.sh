#!/bin/bash
# Instruction-cache counters of integrate_kernel (one rocprofv3 --pmc pass each, no tracing domains): the QM9
# one-molecule column-split team mode (TP_MODES=0), the tile-dealt G = 7 mode and the LJ13 bench workload.  Tests the
# hypothesis that the > 64 KiB kernels stall on instruction fetch.
# Usage: tools/pmc_icache.sh TAG  -> gpurun_out/prof_TAG/icache_*/
TAG=${1:-r4}
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT="$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH SQC_ICACHE_REQ SQC_ICACHE_MISSES SQC_ICACHE_HITS"
B="bench.py --steps 2 --warmup 1 --cpu-molecules 0 --fp32-steps 0 --train-steps 0 --ref-latency-samples 0 --pmc 0 --logprob 0"
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex integrate_kernel -d "$OUT/icache_lj13" -o run --output-format csv -- python3 $B > "$OUT/icache_lj13.log" 2>&1 || exit $?
echo "icache lj13 pass ok"
[ "${ICACHE_ONLY:-}" = lj13 ] && exit 0
TP_MODES=0 timeout -s KILL 90 rocprofv3 --pmc $C --kernel-include-regex integrate_kernel -d "$OUT/icache_cols" -o run --output-format csv -- python3 tools/team_probe.py qm9 1 > "$OUT/icache_cols.log" 2>&1 || exit $?
echo "icache cols pass ok"
TP_MODES=7 timeout -s KILL 90 rocprofv3 --pmc $C --kernel-include-regex integrate_kernel -d "$OUT/icache_g7" -o run --output-format csv -- python3 tools/team_probe.py qm9 1 > "$OUT/icache_g7.log" 2>&1 || exit $?
echo "icache g7 pass ok"
