# exact trace: dense vs sparse vs sparse + primal-aggregate cache -- parity check, then interleaved timing (LJ13 B=1024)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 120 python -u tools/exp_sparse_dbg.py || exit 1
export ECNF_PATHS_ONLY=lj13 ECNF_PATHS_DIV=exact
for r in 1 2; do
  ECNF_EXACT_SPARSE=0 timeout -k 10 120 python -u tools/bench_paths.py gpurun_out/pc_dense_$r.json || exit 1
  ECNF_EXACT_PCACHE=0 timeout -k 10 120 python -u tools/bench_paths.py gpurun_out/pc_sparse_$r.json || exit 1
  timeout -k 10 120 python -u tools/bench_paths.py gpurun_out/pc_cache_$r.json || exit 1
done
