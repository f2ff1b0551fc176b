#!/bin/bash
# r03 (f): cost kernels -- parity of the LDS-DMA kernels against the register-staged one,
# then per-kernel times (rocprofv3) of big / ring / ws, with and without the C stores.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03f; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "ring or pairwise_cost or split16" -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; grep -E "FAIL|Error|passed|failed" $O/tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
for cfg in "big:" "ring:OTF_COST_RING=1" "ws:OTF_COST_WS=1"; do
  name=${cfg%%:*}; envs=${cfg#*:}
  for v in "" _a1; do
    for shp in "4096 512 f32" "8192 1024 f16in"; do
      tag=${name}${v}_$(echo $shp | tr ' ' '_')
      echo "=== $name$v $shp"
      env $envs timeout -k 10 60 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag -o run -- ./tools/ubench_cost$v $shp 20 > $O/$tag.log 2>&1 || exit $?
      grep "per call" $O/$tag.log
      f=$(find $O/$tag -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cut -d, -f1-4 "$f" | head -4
    done
  done
done
