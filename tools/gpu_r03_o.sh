#!/bin/bash
# r03 (o): two-hop gather engine -- gather tests (both forms), config-2 golden / configs,
# config-2 step A/B (one-hop / two-hop R = 4 / R = 2), MFMA16 cost kernel full parity.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03o; mkdir -p $O
export OTF_STALL_MS=5000
timeout -k 10 500 python -u -m pytest tests/test_gpu_gather.py tests/test_gpu_configs.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; grep -E "FAIL|Error|passed|failed" $O/tests.log | tail -12; [ $rc -eq 0 ] || exit $rc
for cfg in "OTF_GATHER2=0" "OTF_GATHER2=1 OTF_GATHER2_R=4" "OTF_GATHER2=1 OTF_GATHER2_R=2"; do
  env $cfg timeout -k 10 120 python -u tools/c2_probe.py 30 || exit $?
done
timeout -k 10 60 ./tools/stamps_sweep 8192 f16 > $O/sweep_stamps.txt 2>&1; rc=$?; tail -30 $O/sweep_stamps.txt; exit $rc
