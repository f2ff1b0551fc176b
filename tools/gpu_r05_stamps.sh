#!/bin/bash
# Build and run the float64 mesh phase-stamp tool on the box (the binary is not pushed).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r05}
mkdir -p $OUT
timeout -k 10 300 /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -munsafe-fp-atomics -DOTF_M64_STAMPS -I include tools/stamps_mesh64.hip -o /tmp/stamps_mesh64 -ldl > $OUT/stamps_build.log 2>&1 || { echo "build failed"; tail -20 $OUT/stamps_build.log; exit 1; }
timeout -k 10 120 /tmp/stamps_mesh64 4096 100 > $OUT/stamps_mesh64.txt 2>&1
rc=$?; echo "stamps rc=$rc"; cat $OUT/stamps_mesh64.txt
exit $rc
