#!/bin/bash
# r03 final: mesh-path tests on the final build, then the evidence session (bench, rocprof, PMC)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
OTF_STALL_MS=5000 timeout -k 10 300 python -u -m pytest tests/test_gpu_mesh.py tests/test_gpu_parity.py tests/test_gpu_precision.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/final_tests.log 2>&1
rc=$?; grep -E "FAIL|Error|passed|failed" gpurun_out/final_tests.log | tail -5; [ $rc -eq 0 ] || exit $rc
TESTS=0 BENCH=1 PROFILE=1 PMC=1 bash tools/gpu_session.sh
