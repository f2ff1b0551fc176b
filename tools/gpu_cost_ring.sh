#!/bin/bash
# r03: ring vs register-staged 256 x 256 cost kernel: parity test, event times at the
# metric shape and config 5, rocprofv3 kernel stats of each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/cost_ring
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "ring or pairwise_cost_vs" -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/cost_ring/tests.log 2>&1
rc=$?; tail -3 gpurun_out/cost_ring/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 0 1; do
  for shp in "4096 512" "8192 1024"; do
    echo "=== ring=$r $shp"; OTF_COST_RING=$r timeout -k 10 120 python -u tools/bench_cost.py $shp || exit $?
  done
done
export TMPDIR=/tmp
for r in 0 1; do
  OTF_COST_RING=$r timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/cost_ring/prof$r -o run -- python3 tools/bench_cost.py 4096 512 > gpurun_out/cost_ring/prof$r.log 2>&1 || exit $?
done
find gpurun_out/cost_ring -name "*kernel_stats.csv" | while read f; do echo "== $f"; head -8 "$f" | cut -c1-200; done
