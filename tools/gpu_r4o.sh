# round-4: column-split chain prefetch depth A/B (ECNF_COLS_PF 8 / 16 / 24, tools/libt_qc*.so): QM9 one-molecule team
# probe (batch path, auto = cols, tile-dealt G = 7), interleaved twice (gpurun_out/r4o/)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4o && export TMPDIR=/tmp && \
for r in 1 2; do for v in qc8 qc16 qc24; do \
TP_MODES=0,7 ECNF_LIB=tools/libt_$v.so timeout -k 10 100 python -u tools/team_probe.py qm9 1 > gpurun_out/r4o/team_${v}_$r.log 2>&1 || exit $?; \
echo $v $r $(grep -o '"auto_G26": {[^}]*}' gpurun_out/r4o/team_${v}_$r.log | head -1) $(grep -o '"pid_call_ms": \[[^]]*\]' gpurun_out/r4o/team_${v}_$r.log | head -1); \
done; done
