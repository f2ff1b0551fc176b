#!/bin/bash
# Mesh engine: stamps at the metric shape (vs tiled), then its tests and the parity file.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export OTF_STALL_MS=3000
timeout -k 10 60 ./tools/stamps_resident 4096 mesh > gpurun_out/st_mesh4096.txt 2>&1; rc=$?; cat gpurun_out/st_mesh4096.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 60 ./tools/stamps_resident 4096 tiled > gpurun_out/st_tiled4096.txt 2>&1; rc=$?; cat gpurun_out/st_tiled4096.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_mesh.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/mesh_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|Error|assert" gpurun_out/mesh_tests.log | head -40; tail -3 gpurun_out/mesh_tests.log; echo "mesh pytest rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/parity_tests.log 2>&1
rc=$?; tail -3 gpurun_out/parity_tests.log; echo "parity pytest rc=$rc"
