#!/bin/bash
# One GPU call: the full -m gpu suite, then bench_paths.py on the divergence modes (or ECNF_PATHS_DIV / _ONLY).
# Usage (from gpurun): bash tools/gpu_tests_paths.sh TAG
TAG=${1:-t}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
ECNF_PATHS_DIV=${ECNF_PATHS_DIV:-hutchinson,exact} timeout -k 10 400 python -u tools/bench_paths.py gpurun_out/paths_$TAG.json > gpurun_out/paths_$TAG.log 2>&1 || { tail -20 gpurun_out/paths_$TAG.log; exit 1; }
cat gpurun_out/paths_$TAG.log | grep -v amdgpu.ids
