#!/bin/bash
# r03 (rpend): the mesh reducer's polls reloading all producers each pass (r0) against
# only the pending ones (r1, the r03 default), interleaved, plus the stamped builds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03rpend; mkdir -p $O
export TMPDIR=/tmp OTF_STALL_MS=3000
for rep in 1 2 3; do
  for v in r1 r0; do
    timeout -k 10 60 tools/stamps_mesh_$v 4096 100 9 > $O/$v.$rep.txt 2>&1; rc=$?
    echo "$v.$rep $(grep -E 'median|MISMATCH' $O/$v.$rep.txt)"; [ $rc -eq 0 ] || exit $rc
  done
done
for v in r1_st r0_st; do
  timeout -k 10 60 tools/stamps_mesh_$v 4096 100 7 > $O/$v.txt 2>&1; rc=$?
  echo "== $v"; grep -E "median|iteration|row hop|hop B|reducer|publish|u \+ col" $O/$v.txt; [ $rc -eq 0 ] || exit $rc
done
