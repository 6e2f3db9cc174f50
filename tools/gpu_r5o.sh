# round 5: ALDP adaptive batch sizing A/B (tools/libt_abase.so: m = 2 per workgroup; libt_apen.so: the adaptive
# penalty 0.15 -> m = 1, one molecule per workgroup, workgroups list-scheduled onto CUs as they retire)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5o && export TMPDIR=/tmp && \
for r in 1 2 3; do
  for v in abase apen; do
    for c in aldp_b512_pid_hutchinson_logp aldp_b512_pid_none_sample; do
      ECNF_LIB=tools/libt_$v.so timeout -k 10 120 python -u tools/bench_paths.py --case $c --reps 3 > gpurun_out/r5o/${v}_${c}_$r.json 2> gpurun_out/r5o/${v}_${c}_$r.err || exit 1
      echo "$r $v $c $(grep -o '"ms": [0-9.]*' gpurun_out/r5o/${v}_${c}_$r.json) $(grep -o '"nfe_mean": [0-9.]*' gpurun_out/r5o/${v}_${c}_$r.json)"
    done
  done
done
