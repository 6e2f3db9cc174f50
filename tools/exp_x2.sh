# exact-trace block-1 sparse dual tiles: interleaved A/B of the LJ13 exact log_prob (B = 1024, Euler-100), one library
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
export ECNF_PATHS_ONLY=lj13 ECNF_PATHS_DIV=exact
for r in 1 2; do
  ECNF_EXACT_SPARSE=0 timeout -k 10 120 python -u tools/bench_paths.py gpurun_out/px_dense_$r.json || exit 1
  ECNF_EXACT_SPARSE=1 timeout -k 10 120 python -u tools/bench_paths.py gpurun_out/px_sparse_$r.json || exit 1
done
