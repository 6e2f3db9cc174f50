#!/bin/bash
# One GPU call: full -m gpu suite, all-mode throughput table, and one rank's shard of BASELINE configs[4]
# (8192 LJ13 molecules = 65536 / 8, sample + Hutchinson eval leg) on one GPU.  Usage: bash tools/gpu_s5.sh TAG
TAG=${1:-s5}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v -s --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 400 python -u tools/bench_paths.py gpurun_out/paths_$TAG.json > gpurun_out/paths_$TAG.log 2>&1 || { echo "paths failed"; tail -5 gpurun_out/paths_$TAG.log; exit 1; }
cat gpurun_out/paths_$TAG.log | grep -v amdgpu.ids
timeout -k 10 300 python -u bench.py --batch 8192 --logprob 1 --steps 3 --warmup 1 --cpu-molecules 0 --fp32-steps 0 --train-steps 0 > gpurun_out/bench_shard8192_$TAG.json 2> gpurun_out/bench_shard8192_$TAG.err || { echo "shard bench failed"; tail -5 gpurun_out/bench_shard8192_$TAG.err; exit 1; }
cat gpurun_out/bench_shard8192_$TAG.json
