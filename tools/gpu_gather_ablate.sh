#!/bin/bash
# Gather engine timing (config 2: 512 x 512 float64, 1999 iterations): the library build
# (no stamps) and diagnostic ablations; 1 = no producer wait, 2 = no row FMAs,
# 4 = no column FMAs, 6 = neither.  Stamped builds also print the phase split.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in _nost _nost_ab1 _nost_ab6 "" _ab1 _ab2 _ab4 _ab6; do
  echo "== stamps_resident$v"
  timeout -k 10 60 ./tools/stamps_resident$v 512 gather double > gpurun_out/gab$v.txt 2>&1 || exit 1
  grep -v "^rc=0 status=[23] engine=5 solve 1[0-9]\.\|stream rc" gpurun_out/gab$v.txt
done
