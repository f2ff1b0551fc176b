#!/bin/bash
# r03 (c): cost ring A/B, sweep granule-flush stamps A/B, precision / EMD / GW-cap tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03c
export OTF_STALL_MS=3000
O=gpurun_out/r03c
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "ring or break_all" -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/t_ring.log 2>&1
rc=$?; tail -3 $O/t_ring.log; [ $rc -le 1 ] || exit $rc
for r in 0 1; do
  echo "=== cost ring=$r"; OTF_COST_RING=$r timeout -k 10 120 python -u tools/bench_cost.py 4096 512 > $O/cost_ring$r.txt 2>&1 || exit $?
  cat $O/cost_ring$r.txt
  OTF_COST_RING=$r timeout -k 10 120 python -u tools/bench_cost.py 8192 1024 > $O/cost5_ring$r.txt 2>&1 || exit $?
  cat $O/cost5_ring$r.txt
done
for g in 1 0; do
  echo "=== sweep stamps gran=$g (config 5)"; OTF_SWEEP_GRAN=$g timeout -k 10 60 ./tools/stamps_sweep 8192 f16 > $O/sweep_stamps_g$g.txt 2>&1; rc=$?; cat $O/sweep_stamps_g$g.txt; [ $rc -eq 0 ] || exit $rc
  echo "=== sweep stamps gran=$g (N=16384 f32)"; OTF_SWEEP_GRAN=$g timeout -k 10 60 ./tools/stamps_sweep 16384 f32 > $O/sweep16_stamps_g$g.txt 2>&1; rc=$?; cat $O/sweep16_stamps_g$g.txt; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_precision.py tests/test_gpu_emd.py tests/test_gpu_gw.py -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/t_prec_emd_gw.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR" $O/t_prec_emd_gw.log | tail -40; echo "pytest rc=$rc"
exit $rc
