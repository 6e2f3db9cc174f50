# round 5 final: per-config rocprofv3 stats + counter passes of the ALDP and QM9 cases at the per-shape aggregation build
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
timeout -k 10 1000 bash tools/profile_configs.sh r5ar aldp_b512_pid_none_sample aldp_b512_pid_hutchinson_logp qm9_b2048_euler_none_sample qm9_b512_euler_hutchinson_logp > gpurun_out/prof_r5ar.log 2>&1; rc=$?
tail -40 gpurun_out/prof_r5ar.log | cut -c1-250; exit $rc
