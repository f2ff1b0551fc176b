#!/bin/bash
# Mesh engine hop analysis: timing-only builds and the stamped build of each variant
# given on the command line (tools/stamps_mesh_<v> / tools/stamps_mesh_<v>_st).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export OTF_STALL_MS=3000
for v in "$@"; do
  for b in "tools/stamps_mesh_$v" "tools/stamps_mesh_${v}_st"; do
    [ -x "$b" ] || continue
    echo "=== $b"
    timeout -k 10 60 "$b" 4096 100 7 > "gpurun_out/$(basename $b).txt" 2>&1; rc=$?
    cat "gpurun_out/$(basename $b).txt"
    [ $rc -eq 0 ] || { echo "rc=$rc"; exit $rc; }
  done
done
