# round 5: chunked, re-dealt adaptive solves (ALDP B = 512 PID): one-launch build vs first chunks of 2 / 4 / 8 steps
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5q && export TMPDIR=/tmp && \
ECNF_LIB=tools/libt_rev_5395d96.so timeout -k 10 120 python -u tools/diag/sched_check.py gpurun_out/r5q/ref.npz > gpurun_out/r5q/ref.log 2>&1 && grep "^{" gpurun_out/r5q/ref.log && \
for v in ach4 ach2 ach8; do
  ECNF_LIB=tools/libt_$v.so timeout -k 10 120 python -u tools/diag/sched_check.py gpurun_out/r5q/$v.npz gpurun_out/r5q/ref.npz > gpurun_out/r5q/$v.log 2>&1 || { tail -20 gpurun_out/r5q/$v.log; exit 1; }
  grep "^{" gpurun_out/r5q/$v.log
done
