# round-4: sub-phase stamps of the QM9 column-split edge tile (tools/libecnf_hip_stamps_qm9.so), then the
# instruction-cache counter passes (tools/pmc_icache.sh) (gpurun_out/r4p/, gpurun_out/prof_r4p/)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4p && export TMPDIR=/tmp && \
timeout -k 5 150 python -u tools/diag_small.py qm9 > gpurun_out/r4p/diag.log 2>&1 && grep -c " ok " gpurun_out/r4p/diag.log && \
ECNF_STAMPS_LIB=tools/libecnf_hip_stamps_qm9.so timeout -k 10 90 python -u tools/phase_stamps.py qm9 1 > gpurun_out/r4p/stamps_qm9_cols.json 2>&1 && \
grep -h -A14 '"shares"' gpurun_out/r4p/stamps_qm9_cols.json && \
bash tools/pmc_icache.sh r4p
