# round 5: per-config rocprofv3 evidence at the round-5 kernels (every BASELINE GPU config and divergence mode)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
bash tools/profile_configs.sh r5m lj13_b1024_euler_none_sample lj13_b1024_euler_hutchinson_sample lj13_b1024_euler_exact_logp \
  aldp_b512_pid_none_sample aldp_b512_pid_hutchinson_logp qm9_b2048_euler_none_sample qm9_b512_euler_hutchinson_logp > gpurun_out/r5m.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r5m.log | tail -5; exit $rc
