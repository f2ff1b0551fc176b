#!/bin/bash
# r03 (k): re-entry baseline on the current build -- full GPU suite, driver bench,
# rocprofv3 kernel stats of the bench, cost kernel times + stamps, mesh stamps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03k; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; grep -E "FAIL|Error|passed|failed" $O/tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1; rc=$?; tail -c 600 $O/bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 10 --warmup 3 --no-gw --no-config5 --no-cpu-baseline --no-hbm-probe > $O/prof_bench.log 2>&1 || exit $?
for shp in "4096 512 f32" "8192 1024 f16in"; do
  echo "=== cost $shp"; timeout -k 10 60 ./tools/ubench_cost_s0 $shp 20 || exit $?
done
timeout -k 10 60 ./tools/stamps_resident 4096 mesh > $O/mesh_stamps.txt 2>&1; rc=$?; tail -25 $O/mesh_stamps.txt; exit $rc
