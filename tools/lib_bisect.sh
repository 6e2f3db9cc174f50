#!/bin/bash
# Run a pytest selection against each tools/libt_*.so (ECNF_LIB), one library per pytest process.
# Usage: gpurun -- bash tools/lib_bisect.sh "pytest -k expression"
cd "$GRAFT_REPO_ROOT" || exit 1
for lib in tools/libt_*.so; do
  echo "== $lib"
  ECNF_LIB=$PWD/$lib timeout -k 10 200 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rA -k "$1" 2>&1 | grep -E "^(PASSED|FAILED)|assert .*<=" | cut -c1-150
done
