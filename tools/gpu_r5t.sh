# round 5, final build: smoke, bench line, rocprofv3 evidence of the bench workload, per-config profiles
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
bash tools/evidence.sh r5t > gpurun_out/r5t_evidence.log 2>&1 && tail -3 gpurun_out/r5t_evidence.log && \
bash tools/profile_configs.sh r5t lj13_b1024_euler_none_sample lj13_b1024_euler_hutchinson_sample lj13_b1024_euler_exact_logp \
  aldp_b512_pid_none_sample aldp_b512_pid_hutchinson_logp qm9_b2048_euler_none_sample qm9_b512_euler_hutchinson_logp > gpurun_out/r5t_configs.log 2>&1
rc=$?; grep "profiled\|failed" gpurun_out/r5t_configs.log | cut -c1-160; exit $rc
