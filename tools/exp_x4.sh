# final validation of the build: full GPU suite, smoke, bench line + rocprof evidence (tools/gpu_check.sh), all-mode table
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
bash tools/gpu_check.sh x7 || exit $?
timeout -k 10 300 python -u tools/bench_paths.py gpurun_out/paths_x7.json > gpurun_out/paths_x7.log 2>&1 || { tail -5 gpurun_out/paths_x7.log; exit 1; }
