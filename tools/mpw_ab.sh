#!/bin/bash
# A/B of the adaptive workgroup-sizing penalty (ECNF_ADAPTIVE_MPW_PENALTY) on the adaptive configs of bench_paths.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for pen in 0 0.15 0.3; do
  echo "penalty $pen"
  ECNF_ADAPTIVE_MPW_PENALTY=$pen ECNF_PATHS_ONLY=aldp,dw4 ECNF_PATHS_DIV=none,hutchinson timeout -k 10 200 python -u tools/bench_paths.py 2>&1 | grep -v amdgpu.ids | grep dopri5 || exit 1
done
