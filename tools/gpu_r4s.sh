# round-4: cols prefetch depth at 8 waves (tools/libt_qp4.so, libt_qp12.so vs the product's 8; QM9 B = 1 cols mode,
# interleaved) and the phase stamps of the 8-wave cols kernel (gpurun_out/r4s/)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4s && export TMPDIR=/tmp && \
ECNF_LIB=tools/libt_qp12.so timeout -k 5 150 python -u tools/diag_small.py qm9 > gpurun_out/r4s/diag_qp12.log 2>&1 && grep -c " ok " gpurun_out/r4s/diag_qp12.log && \
for rep in 1 2; do for lib in ecnf-baseline-neurips-2023_amd/ecnf_amd/libecnf_hip.so tools/libt_qp4.so tools/libt_qp12.so; do \
  ECNF_LIB=$lib TP_MODES=0 timeout -k 10 120 python -u tools/team_probe.py qm9 1 > gpurun_out/r4s/probe.log 2>&1 || exit $?; \
  echo "$rep $lib $(grep -o '"us_per_eval": [0-9.]*' gpurun_out/r4s/probe.log | head -1) $(grep -o '"pid_call_ms": \[[0-9., ]*' gpurun_out/r4s/probe.log | head -1)" | tee -a gpurun_out/r4s/ab_pf.log; \
done; done && \
ECNF_STAMPS_LIB=tools/libecnf_hip_stamps_qm9.so timeout -k 10 90 python -u tools/phase_stamps.py qm9 1 > gpurun_out/r4s/stamps_qm9_cols8.json 2>&1 && \
grep -h -A16 '"shares"' gpurun_out/r4s/stamps_qm9_cols8.json
