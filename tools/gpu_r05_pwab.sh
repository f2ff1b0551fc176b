#!/bin/bash
# f64 MFMA throughput microbenchmark, then the pairwise prologue stamps of the library's
# source (tools/st_pw) and an alternative (tools/st_p1), interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r05pw}
mkdir -p $OUT
export LD_LIBRARY_PATH=$PWD/ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd/otfuse/lib:${LD_LIBRARY_PATH:-}
timeout -k 10 120 ./tools/ubench_mfma64 > $OUT/ubench_mfma64.txt 2>&1 || { echo "ubench rc=$?"; cat $OUT/ubench_mfma64.txt; exit 1; }
cat $OUT/ubench_mfma64.txt
for rep in 1 2; do
  for b in st_pw st_p1; do
    timeout -k 10 120 ./tools/$b 4096 100 pw > $OUT/${b}_$rep.txt 2>&1 || { echo "$b rc=$?"; tail $OUT/${b}_$rep.txt; exit 1; }
    echo "== $b $rep"; grep -E "solve|roles|block|grid max|exp|iteration " $OUT/${b}_$rep.txt | tail -9
  done
done
