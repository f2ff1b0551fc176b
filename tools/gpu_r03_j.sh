#!/bin/bash
# r03 (j): cost epilogue v2 -- parity, kernel times (big / ring), phase stamps of both.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03j; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_config5.py -k "ring or pairwise_cost or split16 or fp16" -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; grep -E "FAIL|Error|passed|failed" $O/tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
for cfg in "big:" "ring:OTF_COST_RING=1"; do
  name=${cfg%%:*}; envs=${cfg#*:}
  for shp in "4096 512 f32" "8192 1024 f16in"; do
    tag=${name}_$(echo $shp | tr ' ' '_'); echo "=== $tag"
    env $envs timeout -k 10 60 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag -o run -- ./tools/ubench_cost $shp 20 > $O/$tag.log 2>&1 || exit $?
    grep "per call" $O/$tag.log; f=$(find $O/$tag -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cut -d, -f1-4 "$f" | sed -n 2,3p
  done
  for v in s0 s1; do echo "=== $name $v"; env $envs timeout -k 10 60 ./tools/ubench_cost_$v 4096 512 f32 10 || exit $?; done
done
