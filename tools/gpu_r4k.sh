# round-4: small solves of every config (a fault stops the call); phase stamps of the QM9 one-molecule team modes
# (column-split auto / tile-dealt G = 7) and of ALDP B = 512 (primal and Hutchinson); team probes of the product
# library and the exchange / prefetch variants (tools/libt_q*.so); the issue-counter PMC pass of the headline kernel;
# LJ13 A/B of the packed-f32 activation and node-GEMM prefetch depth (tools/libt_[bn]*.so); then the whole GPU suite
# and smoke at the product build (gpurun_out/r4k/)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4k && export TMPDIR=/tmp && \
timeout -k 5 150 python -u tools/diag_small.py dw4 lj13 aldp qm9 > gpurun_out/r4k/diag.log 2>&1; rc=$?; grep -c " ok " gpurun_out/r4k/diag.log; \
[ $rc -eq 0 ] || { cat gpurun_out/r4k/diag.log; exit $rc; }; \
ECNF_STAMPS_LIB=tools/libecnf_hip_stamps_qm9.so timeout -k 10 90 python -u tools/phase_stamps.py qm9 1 > gpurun_out/r4k/stamps_qm9_cols.json 2>&1; \
ECNF_PROBE_TEAM=7 ECNF_STAMPS_LIB=tools/libecnf_hip_stamps_qm9.so timeout -k 10 90 python -u tools/phase_stamps.py qm9 1 > gpurun_out/r4k/stamps_qm9_g7.json 2>&1; \
ECNF_STAMPS_LIB=tools/libecnf_hip_stamps_aldp.so timeout -k 10 90 python -u tools/phase_stamps.py aldp 512 > gpurun_out/r4k/stamps_aldp.json 2>&1; \
ECNF_STAMPS_LIB=tools/libecnf_hip_stamps_aldp.so timeout -k 10 90 python -u tools/phase_stamps.py aldp 512 hutchinson > gpurun_out/r4k/stamps_aldp_hutch.json 2>&1; \
grep -h -A12 '"shares"' gpurun_out/r4k/stamps_qm9_cols.json gpurun_out/r4k/stamps_qm9_g7.json; \
ECNF_LIB=tools/libt_q2.so timeout -k 10 120 python -u tools/team_probe.py qm9 1 > gpurun_out/r4k/team_q2.log 2>&1; tail -c 500 gpurun_out/r4k/team_q2.log; \
ECNF_LIB=tools/libt_qx.so timeout -k 10 120 python -u tools/team_probe.py qm9 1 > gpurun_out/r4k/team_qx.log 2>&1; tail -c 500 gpurun_out/r4k/team_qx.log; \
ECNF_LIB=tools/libt_q6.so timeout -k 10 120 python -u tools/team_probe.py qm9 1 > gpurun_out/r4k/team_q6.log 2>&1; tail -c 500 gpurun_out/r4k/team_q6.log; \
bash tools/pmc_issue.sh r4k; tail -2 gpurun_out/prof_r4k/issue.log; \
TV_GLOB='libt_[bn]*.so' timeout -k 10 240 python -u tools/time_variants.py 3 > gpurun_out/r4k/ab_lj13.log 2>&1; tail -4 gpurun_out/r4k/ab_lj13.log; \
TV_CASE=qm9 TV_GLOB='libt_q[26].so' timeout -k 10 150 python -u tools/time_variants.py 2 > gpurun_out/r4k/ab_pfa_qm9.log 2>&1; tail -2 gpurun_out/r4k/ab_pfa_qm9.log; \
timeout -k 10 450 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4k/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r4k/pytest.log; \
[ $rc -eq 0 ] || exit $rc; \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4k/smoke.log 2>&1; cat gpurun_out/r4k/smoke.log
