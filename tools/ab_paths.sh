#!/bin/bash
# One GPU call: interleaved A/B of tools/libt_<A>.so vs tools/libt_<B>.so on the bench_paths cases of one config
# (ECNF_PATHS_ONLY), ROUNDS rounds.  Usage (from gpurun): bash tools/ab_paths.sh CONFIG A B [ROUNDS] [DIVS]
CONF=$1; A=$2; B=$3; ROUNDS=${4:-2}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp ECNF_PATHS_ONLY=$CONF
[ -n "$5" ] && export ECNF_PATHS_DIV=$5
for r in $(seq 1 "$ROUNDS"); do
  for v in "$A" "$B"; do
    echo "== $v round $r"
    ECNF_LIB="$GRAFT_REPO_ROOT/tools/libt_$v.so" timeout -k 10 300 python -u tools/bench_paths.py > "gpurun_out/ab_${CONF}_${v}_$r.log" 2>&1 || { tail -5 "gpurun_out/ab_${CONF}_${v}_$r.log"; exit 1; }
    cat "gpurun_out/ab_${CONF}_${v}_$r.log"
  done
done
