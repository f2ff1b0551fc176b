#!/bin/bash
# r03 (h): ring cost kernel phase stamps (full / no stores / no stores-MFMA-DMA); sweep
# engine with float S + slice ready words: parity tests, stamps, cross-rank tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03h; mkdir -p $O
export OTF_STALL_MS=5000 OTF_COST_RING=1
for v in s0 s1 s7; do
  echo "=== ubench_cost_$v"; timeout -k 10 60 ./tools/ubench_cost_$v 4096 512 f32 10 || exit $?
done
unset OTF_COST_RING
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_config5.py tests/test_gpu_xsweep.py -k "sweep or config5 or fp16 or break_all" -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; grep -E "FAIL|Error|passed|failed" $O/tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 60 ./tools/stamps_sweep 8192 f16 > $O/sweep_stamps.txt 2>&1; rc=$?; cat $O/sweep_stamps.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 60 ./tools/stamps_sweep 16384 f32 > $O/sweep16_stamps.txt 2>&1; rc=$?; head -4 $O/sweep16_stamps.txt; exit $rc
