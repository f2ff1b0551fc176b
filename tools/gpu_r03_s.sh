#!/bin/bash
# r03 (s): loss kernel checks the solve info itself (no torch launches for ok); align,
# gather, configs tests; config-2 step; MFMA16 cost stamps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03s; mkdir -p $O
export OTF_STALL_MS=5000
timeout -k 10 500 python -u -m pytest tests/test_gpu_align.py tests/test_gpu_gather.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; grep -E "FAIL|Error|passed|failed" $O/tests.log | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/c2_probe.py 30 || exit $?
timeout -k 10 60 ./tools/ubench_cost_s0 4096 512 f32 20 || exit $?
