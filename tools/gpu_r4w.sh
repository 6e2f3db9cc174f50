# round-4: node-GEMM prefetch depth of the M = 256 split primal kernels at the 8-wave cols build (product: 2;
# tools/libt_npw4.so, libt_npw6.so): QM9 B = 1 cols mode (team probe) and QM9 B = 2048 batch path (gpurun_out/r4w/)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4w && export TMPDIR=/tmp && \
ECNF_LIB=tools/libt_npw6.so timeout -k 5 150 python -u tools/diag_small.py qm9 > gpurun_out/r4w/diag_npw6.log 2>&1 && grep -c " ok " gpurun_out/r4w/diag_npw6.log && \
for rep in 1 2; do for lib in ecnf-baseline-neurips-2023_amd/ecnf_amd/libecnf_hip.so tools/libt_npw4.so tools/libt_npw6.so; do \
  ECNF_LIB=$lib TP_MODES=0 timeout -k 10 120 python -u tools/team_probe.py qm9 1 > gpurun_out/r4w/probe.log 2>&1 || exit $?; \
  echo "$rep $lib $(grep -o '"us_per_eval": [0-9.]*' gpurun_out/r4w/probe.log | head -1) $(grep -o '"pid_call_ms": \[[0-9., ]*' gpurun_out/r4w/probe.log | head -1)" | tee -a gpurun_out/r4w/ab_cols.log; \
done; done && \
TV_CASE=qm9 TV_GLOB='libt_npw*.so' timeout -k 10 300 python -u tools/time_variants.py 2 > gpurun_out/r4w/ab_qm9_batch.log 2>&1 && tail -2 gpurun_out/r4w/ab_qm9_batch.log
