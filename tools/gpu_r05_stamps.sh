#!/bin/bash
# Build and run the float64 mesh phase-stamp tool on the box (the binary is not pushed).
# ALT="a.hip b.hip": also time these alternative float64 mesh sources (A/B), interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r05}
mkdir -p $OUT
CS=ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd/csrc
build() {  # $1 = output, $2 = optional alternative source
  local def=""
  if [ -n "${2:-}" ]; then def="-DOTF_M64_ALT=\"$PWD/$2\""; fi
  timeout -k 10 300 /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -munsafe-fp-atomics -DOTF_M64_STAMPS $def -I include -I $CS tools/stamps_mesh64.hip -o $1 -ldl >> $OUT/stamps_build.log 2>&1
}
build /tmp/stamps_mesh64 || { echo "build failed"; tail -20 $OUT/stamps_build.log; exit 1; }
k=0
for a in ${ALT:-}; do
  build /tmp/stamps_alt$k $a || { echo "build $a failed"; tail -20 $OUT/stamps_build.log; exit 1; }
  k=$((k + 1))
done
for rep in 1 2; do
  timeout -k 10 120 /tmp/stamps_mesh64 4096 100 > $OUT/stamps_mesh64_$rep.txt 2>&1
  rc=$?; echo "stamps (tree) rc=$rc"; tail -9 $OUT/stamps_mesh64_$rep.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
  k=0
  for a in ${ALT:-}; do
    timeout -k 10 120 /tmp/stamps_alt$k 4096 100 > $OUT/stamps_alt${k}_$rep.txt 2>&1
    rc=$?; echo "stamps ($a) rc=$rc"; tail -9 $OUT/stamps_alt${k}_$rep.txt
    if [ $rc -ne 0 ]; then exit $rc; fi
    k=$((k + 1))
  done
done
exit 0
