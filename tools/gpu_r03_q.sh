#!/bin/bash
# r03 (q): gather engine with two tagged doubles per chunk (tests, config-2 step),
# MFMA16 cost default for fp32 storage (parity), driver bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03q; mkdir -p $O
export OTF_STALL_MS=5000
timeout -k 10 500 python -u -m pytest tests/test_gpu_gather.py tests/test_gpu_configs.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; grep -E "FAIL|Error|passed|failed" $O/tests.log | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/c2_probe.py 30 || exit $?
unset OTF_STALL_MS
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.log 2>&1; rc=$?; tail -c 300 $O/bench.log; exit $rc
