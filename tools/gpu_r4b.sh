# round-4 batch b: A/B (HEAD vs working tree: LJ13 primal / Hutchinson, ALDP PID sample / Hutchinson), team-mode probe
# and QM9 phase stamps, then the whole GPU suite (gpurun_out/r4b/)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4b && export TMPDIR=/tmp && \
TV_GLOB='libt_[hc]*.so' timeout -k 10 300 python -u tools/time_variants.py 3 > gpurun_out/r4b/ab_lj13.log 2>&1 && tail -2 gpurun_out/r4b/ab_lj13.log && \
TV_CASE=lj13_hutch TV_GLOB='libt_[hc]*.so' timeout -k 10 300 python -u tools/time_variants.py 3 > gpurun_out/r4b/ab_lj13h.log 2>&1 && tail -2 gpurun_out/r4b/ab_lj13h.log && \
TV_CASE=aldp_sample TV_GLOB='libt_a*.so' timeout -k 10 300 python -u tools/time_variants.py 3 > gpurun_out/r4b/ab_aldps.log 2>&1 && tail -2 gpurun_out/r4b/ab_aldps.log && \
TV_CASE=aldp_hutch TV_GLOB='libt_a*.so' timeout -k 10 300 python -u tools/time_variants.py 3 > gpurun_out/r4b/ab_aldph.log 2>&1 && tail -2 gpurun_out/r4b/ab_aldph.log && \
TV_CASE=qm9 TV_GLOB='libt_q*.so' timeout -k 10 300 python -u tools/time_variants.py 2 > gpurun_out/r4b/ab_qm9_wload.log 2>&1 && tail -2 gpurun_out/r4b/ab_qm9_wload.log && \
timeout -k 10 300 python -u tools/team_probe.py qm9 1 4 16 > gpurun_out/r4b/team_qm9.log 2>&1 && tail -c 1500 gpurun_out/r4b/team_qm9.log && \
ECNF_STAMPS_LIB=tools/libecnf_hip_stamps_qm9.so timeout -k 10 300 python -u tools/phase_stamps.py qm9 1 > gpurun_out/r4b/stamps_qm9_team.json 2>&1 && \
ECNF_PROBE_TEAM=1 ECNF_STAMPS_LIB=tools/libecnf_hip_stamps_qm9.so timeout -k 10 300 python -u tools/phase_stamps.py qm9 1 > gpurun_out/r4b/stamps_qm9_batch.json 2>&1 && \
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r4b/pytest.log 2>&1; rc=$?; tail -4 gpurun_out/r4b/pytest.log; exit $rc
