#!/bin/bash
# r03: sweep engine with the granule flush -- parity tests, then config 5 / N = 16384
# per-sweep times with the granule flush (default) and the r02 flush (OTF_SWEEP_GRAN=0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sweep_gran
export OTF_STALL_MS=3000
timeout -k 10 400 python -u -m pytest tests/test_gpu_config5.py tests/test_gpu_parity.py -k "sweep or config5 or fp16" -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/sweep_gran/tests.log 2>&1
rc=$?; grep -E "FAIL|Error" gpurun_out/sweep_gran/tests.log | head; tail -2 gpurun_out/sweep_gran/tests.log; [ $rc -eq 0 ] || exit $rc
for g in 1 0; do
  echo "=== OTF_SWEEP_GRAN=$g"; OTF_SWEEP_GRAN=$g timeout -k 10 200 python -u tools/sweep_probe.py --cases c5,n16k || exit $?
done
