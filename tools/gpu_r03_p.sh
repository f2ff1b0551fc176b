#!/bin/bash
# r03 (p): two-hop gather engine (tests, config-2 step A/B), MFMA16 cost kernel with
# transposed accumulators (parity, stamps), sweep-engine stamps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03p; mkdir -p $O
export OTF_STALL_MS=5000
timeout -k 10 500 python -u -m pytest tests/test_gpu_gather.py tests/test_gpu_configs.py tests/test_gpu_parity.py -k "gather or config or mfma16 or pairwise_cost" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; grep -E "FAIL|Error|passed|failed" $O/tests.log | tail -12; [ $rc -eq 0 ] || exit $rc
for cfg in "OTF_GATHER2=0" "OTF_GATHER2=1 OTF_GATHER2_R=4" "OTF_GATHER2=1 OTF_GATHER2_R=2"; do
  env $cfg timeout -k 10 120 python -u tools/c2_probe.py 30 || exit $?
done
for mf in 0 1; do
  for v in s0 s1; do
    for shp in "4096 512 f32" "8192 1024 f16in"; do
      echo "=== mfma16=$mf $v $shp"; OTF_COST_MFMA16=$mf timeout -k 10 60 ./tools/ubench_cost_$v $shp 20 || exit $?
    done
  done
done
timeout -k 10 60 ./tools/stamps_sweep 8192 f16 > $O/sweep_stamps.txt 2>&1; rc=$?; tail -30 $O/sweep_stamps.txt; exit $rc
