cd $GRAFT_REPO_ROOT && timeout -k 10 500 python tools/time_variants.py 3 2>&1 | tail -4
