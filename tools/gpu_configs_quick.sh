#!/bin/bash
# Config / robustness tests (concurrent persistent grids, long solves) and the mesh tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_mesh.py tests/test_gpu_gather.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/cfg_tests.log 2>&1
rc=$?; grep -E "FAIL|Error|concurrent|outlives" gpurun_out/cfg_tests.log | head -20; tail -2 gpurun_out/cfg_tests.log; echo "pytest rc=$rc"
