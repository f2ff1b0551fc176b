#!/bin/bash
# Drop-in API tests (NumPy returns through pinned copies) and the config-3 split probe.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/dropin_tests.log 2>&1
rc=$?; grep -E "FAIL|Error" gpurun_out/dropin_tests.log | head; tail -2 gpurun_out/dropin_tests.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python tools/c3_probe.py > gpurun_out/c3.log 2>&1; rc=$?; grep "rep" gpurun_out/c3.log; echo "probe rc=$rc"
