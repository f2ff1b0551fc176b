#!/bin/bash
# r03 (r): gather engine with tagged-double chunks, MFMA16 cost default (+ L2 prefetch
# A/B), parity tests, config-2 step, driver bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03r; mkdir -p $O
export OTF_STALL_MS=5000
timeout -k 10 500 python -u -m pytest tests/test_gpu_gather.py tests/test_gpu_configs.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; grep -E "FAIL|Error|passed|failed" $O/tests.log | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/c2_probe.py 30 || exit $?
for v in s0 s8 s0 s8; do
  for shp in "4096 512 f32"; do
    echo "=== $v $shp"; timeout -k 10 60 ./tools/ubench_cost_$v $shp 20 || exit $?
  done
done
unset OTF_STALL_MS
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/bench.log 2>&1; rc=$?; tail -c 300 $O/bench.log; exit $rc
