#!/bin/bash
# r03 (m): register-staged 256^2 cost kernel ablations (stamps): full / no stores /
# no stores + no MFMA / no stores + no loop loads / none of the three.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in s0 s1 s3 s5 s7; do
  for shp in "4096 512 f32" "8192 1024 f16in"; do
    echo "=== $v $shp"; timeout -k 10 60 ./tools/ubench_cost_$v $shp 20 || exit $?
  done
done
