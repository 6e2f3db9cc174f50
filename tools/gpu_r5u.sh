# round 5: phase stamps at the final kernels: ALDP (one molecule alone, B = 512), LJ13 B = 1024 (primal and Hutchinson)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5u && export TMPDIR=/tmp && \
for a in "aldp 1 hutchinson" "aldp 512 hutchinson" "aldp 1 none" "lj13 1024 none" "lj13 1024 hutchinson"; do
  set -- $a
  lib=$PWD/tools/libecnf_hip_stamps_aldp.so; [ $1 = lj13 ] && lib=$PWD/tools/libecnf_hip_stamps.so
  ECNF_STAMPS_LIB=$lib timeout -k 10 120 python -u tools/phase_stamps.py $1 $2 $3 > gpurun_out/r5u/stamps_$1_b$2_$3.json 2>gpurun_out/r5u/err_$1_$2_$3.log || exit 1
  cat gpurun_out/r5u/stamps_$1_b$2_$3.json; echo
done
