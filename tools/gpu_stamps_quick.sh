#!/bin/bash
# Stamps of the mesh engine at the metric shape and at config-2-like sizes, then its tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export OTF_STALL_MS=3000
timeout -k 10 60 ./tools/stamps_resident 4096 mesh > gpurun_out/st_mesh4096.txt 2>&1; rc=$?; cat gpurun_out/st_mesh4096.txt
[ $rc -eq 0 ] || exit $rc
OTF_MESH_XCD_ROWS=1 timeout -k 10 60 ./tools/stamps_resident 4096 mesh > gpurun_out/st_mesh4096x.txt 2>&1; rc=$?; cat gpurun_out/st_mesh4096x.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_mesh.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/mesh_tests.log 2>&1
rc=$?; tail -3 gpurun_out/mesh_tests.log; echo "mesh pytest rc=$rc"
