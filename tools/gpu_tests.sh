#!/bin/bash
# GPU-box test run: `bash tools/gpu_tests.sh [pytest targets...]` (default: the whole -m gpu
# suite).  One pytest process, its own time limit; a crash / abort / timeout stops the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
targets=("$@")
[ ${#targets[@]} -eq 0 ] && targets=(tests)
timeout -k 10 ${PYTEST_LIMIT:-900} python -u -m pytest "${targets[@]}" -m gpu -v --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
grep -E "PASSED|FAILED|ERROR|SKIPPED" gpurun_out/gpu_tests.log | grep -vE "PASSED" | head -40
tail -3 gpurun_out/gpu_tests.log
exit $rc
