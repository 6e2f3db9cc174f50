#!/bin/bash
# rocprofv3 evidence for every BASELINE.json GPU config and divergence mode (tools/bench_paths.py cases), each case
# from ONE invocation that also prints its bench line (ms per launch), so the profiled kernel time and the line's
# time come from the same process:  1. kernel trace + stats  2. FETCH_SIZE + GRBM_GUI_ACTIVE + MFMA-busy pass
# 3. WRITE_SIZE pass.  Counter passes are separate runs with --kernel-trace only (no other tracing domain).
# Usage (from gpurun): bash tools/profile_configs.sh TAG [CASE ...]
TAG=${1:-round3}; shift
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT="$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
CASES=("$@")
if [ ${#CASES[@]} -eq 0 ]; then
  CASES=(lj13_b1024_euler_hutchinson_sample lj13_b1024_euler_exact_logp aldp_b512_pid_none_sample
         aldp_b512_pid_hutchinson_logp qm9_b2048_euler_none_sample qm9_b512_euler_hutchinson_logp)
fi
for c in "${CASES[@]}"; do
  d="$OUT/$c"; mkdir -p "$d"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$d/kt" -o run --output-format csv -- \
    python3 tools/bench_paths.py --case "$c" --reps 2 > "$d/line_kt.json" 2> "$d/kt.err" || { echo "kt $c failed"; exit 1; }
  timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --kernel-trace \
    --kernel-include-regex integrate_kernel -d "$d/p0" -o run --output-format csv -- \
    python3 tools/bench_paths.py --case "$c" --reps 2 > "$d/line_p0.json" 2> "$d/p0.err" || { echo "p0 $c failed"; exit 1; }
  timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --kernel-include-regex integrate_kernel -d "$d/p1" -o run \
    --output-format csv -- python3 tools/bench_paths.py --case "$c" --reps 2 > "$d/line_p1.json" 2> "$d/p1.err" || { echo "p1 $c failed"; exit 1; }
  echo "profiled $c: $(cat "$d/line_kt.json")"
done
python3 tools/pmc_configs.py "$OUT" > "$OUT/summary.json" && cat "$OUT/summary.json"
