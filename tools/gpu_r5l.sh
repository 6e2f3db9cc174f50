# round 5: the DW4 exact-trace PID envelope at HEAD, at the pipelined-dot build, and with the shift's exact division
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5l && export TMPDIR=/tmp && \
for v in head new newdiv; do
  ECNF_LIB=tools/libt_$v.so timeout -k 10 200 python -u -m pytest tests/test_gpu_eval_modes.py -k "exact_pid and dw4" -s -q --timeout 150 --timeout-method thread > gpurun_out/r5l/$v.log 2>&1
  echo "== $v rc $?"; grep -E "exact pid|passed|failed" gpurun_out/r5l/$v.log | head -8
done
