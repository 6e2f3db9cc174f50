# round 5: ALDP phase stamps (one molecule alone, and the B = 512 batch), Euler-100, primal and Hutchinson kernels
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5g && export TMPDIR=/tmp && export ECNF_STAMPS_LIB=$PWD/tools/libecnf_hip_stamps_aldp.so && \
for a in "1 hutchinson" "1 none" "512 hutchinson" "512 none"; do
  set -- $a
  timeout -k 10 120 python -u tools/phase_stamps.py aldp $1 $2 > gpurun_out/r5g/stamps_aldp_b$1_$2.json 2>gpurun_out/r5g/err_$1_$2.log || exit 1
  cat gpurun_out/r5g/stamps_aldp_b$1_$2.json
done
