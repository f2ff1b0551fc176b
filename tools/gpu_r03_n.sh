#!/bin/bash
# r03 (n): 32x32x16 vs 16x16x32 256^2 cost kernels -- parity (oracle / register kernel),
# stamps of both, ablations (1 no stores, 3 + no MFMA, 5 + no loop loads, 7 all three).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03n; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "mfma16 or pairwise_cost_vs" -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; grep -E "FAIL|Error|passed|failed" $O/tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
for mf in 0 1; do
  for v in s0 s1 s3 s5 s7; do
    for shp in "4096 512 f32" "8192 1024 f16in"; do
      echo "=== mfma16=$mf $v $shp"; OTF_COST_MFMA16=$mf timeout -k 10 60 ./tools/ubench_cost_$v $shp 20 || exit $?
    done
  done
done
