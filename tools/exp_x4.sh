# final validation of the build: full GPU suite, smoke, bench line + rocprof evidence (tools/gpu_check.sh), all-mode table
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
bash tools/gpu_check.sh x4 || exit $?
timeout -k 10 300 python -u tools/bench_paths.py gpurun_out/paths_x4.json > gpurun_out/paths_x4.log 2>&1 || { tail -5 gpurun_out/paths_x4.log; exit 1; }
