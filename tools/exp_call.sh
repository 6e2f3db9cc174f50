#!/bin/bash
# One GPU call for kernel experiments: A/B timing of tools/libt_*.so (time_variants.py) and one SQ counter pass
# (wave-cycle buckets, VALU / MFMA activity) of the current library on the bench workload.
# Usage (from gpurun): bash tools/exp_call.sh TAG [ROUNDS]
TAG=${1:-exp}
ROUNDS=${2:-3}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/time_variants.py "$ROUNDS" > gpurun_out/variants_$TAG.log 2>&1 || { tail -20 gpurun_out/variants_$TAG.log; exit 1; }
tail -12 gpurun_out/variants_$TAG.log
[ "$3" = "nopmc" ] && exit 0
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters_$TAG.txt 2>&1
WANT="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_INSTS_VALU SQ_INSTS_MFMA"
HAVE=""
for c in $WANT; do grep -q -w "$c" gpurun_out/counters_$TAG.txt && HAVE="$HAVE $c"; done
echo "counters:$HAVE"
B="bench.py --steps 2 --warmup 1 --cpu-molecules 0 --fp32-steps 0 --train-steps 0"
timeout -s KILL 120 rocprofv3 --pmc $HAVE --kernel-include-regex integrate_kernel -d gpurun_out/sq_$TAG -o run \
  --output-format csv -- python3 $B > gpurun_out/sq_$TAG.log 2>&1 || { tail -5 gpurun_out/sq_$TAG.log; exit 1; }
python3 - "$TAG" <<'EOF'
import csv, glob, sys, collections
tag = sys.argv[1]
tot = collections.defaultdict(float)
n = collections.Counter()
for f in glob.glob(f"gpurun_out/sq_{tag}/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        tot[row["Counter_Name"]] += float(row["Counter_Value"])
        n[row["Counter_Name"]] += 1
for k, v in sorted(tot.items()):
    print(f"{k:28s} {v:.4e}  (rows {n[k]})")
EOF
