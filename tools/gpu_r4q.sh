# round-4: the 8-wave M = 256 experiment (tools/libt_qw8.so, -DECNF_WIDE_NW=8: one cols output block per wave):
# small solves first (a fault stops the call), then team probes of the product library and of the experiment, with
# the batch-path samples dumped for a cross-library comparison (gpurun_out/r4q/)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4q && export TMPDIR=/tmp && \
ECNF_LIB=tools/libt_qw8.so timeout -k 5 150 python -u tools/diag_small.py qm9 > gpurun_out/r4q/diag_w8.log 2>&1 && grep -c " ok " gpurun_out/r4q/diag_w8.log && \
TP_MODES=1,0,7 TP_DUMP=gpurun_out/r4q/prod timeout -k 10 150 python -u tools/team_probe.py qm9 1 4 > gpurun_out/r4q/team_prod.log 2>&1 && tail -c 600 gpurun_out/r4q/team_prod.log && \
ECNF_LIB=tools/libt_qw8.so TP_MODES=1,0,7 TP_DUMP=gpurun_out/r4q/w8 timeout -k 10 150 python -u tools/team_probe.py qm9 1 4 > gpurun_out/r4q/team_w8.log 2>&1 && tail -c 600 gpurun_out/r4q/team_w8.log
