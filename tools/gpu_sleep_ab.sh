#!/bin/bash
# Mesh poll back-off A/B: s_sleep 1 / 2 / 4 between polls (stamps builds), twice each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export OTF_STALL_MS=3000
for r in 1 2; do
  for v in "" _sl0; do
    timeout -k 10 60 ./tools/stamps_resident$v 4096 mesh > gpurun_out/sl$v.txt 2>&1 || exit 1
    echo "sleep$v: $(sed -n 3p gpurun_out/sl$v.txt)"
  done
done
