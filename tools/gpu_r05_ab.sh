#!/bin/bash
# Run prebuilt float64 mesh stamp binaries (built here: tools/build_stamps_ab.sh) interleaved,
# two rounds each, on the box.  BINS="tools/bin/stamps_a tools/bin/stamps_b".
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r05}
mkdir -p $OUT
for rep in 1 2; do
  for b in $BINS; do
    n=$(basename $b)
    timeout -k 10 120 ./$b 4096 100 > $OUT/${n}_$rep.txt 2>&1
    rc=$?; echo "$n rc=$rc"; tail -9 $OUT/${n}_$rep.txt
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
exit 0
