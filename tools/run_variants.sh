#!/bin/bash
# run phase_stamps for every tools/libvar_*.so (timing experiments), one process each, bounded
cd "$GRAFT_REPO_ROOT"
for lib in tools/libvar_*.so; do
  name=$(basename "$lib" .so)
  ECNF_STAMPS_LIB="$PWD/$lib" timeout -k 10 120 python tools/phase_stamps.py lj13 1024 > "gpurun_out/${name}.json" 2> "gpurun_out/${name}.err"
  rc=$?
  echo "$name $rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
