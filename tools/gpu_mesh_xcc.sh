#!/bin/bash
# Mesh engine with XCC-local column path: stamps (both role modes), mesh + parity + config tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export OTF_STALL_MS=3000
timeout -k 10 60 ./tools/stamps_resident 4096 mesh > gpurun_out/st_mesh_xcc.txt 2>&1; rc=$?; cat gpurun_out/st_mesh_xcc.txt
[ $rc -eq 0 ] || exit $rc
OTF_MESH_XCC=0 timeout -k 10 60 ./tools/stamps_resident 4096 mesh > gpurun_out/st_mesh_wt.txt 2>&1; rc=$?; cat gpurun_out/st_mesh_wt.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_mesh.py tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/mesh_tests.log 2>&1
rc=$?; grep -E "FAIL|Error" gpurun_out/mesh_tests.log | head; tail -3 gpurun_out/mesh_tests.log; echo "pytest rc=$rc"
