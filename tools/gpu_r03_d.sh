#!/bin/bash
# r03 (d): granule-flush hop stamps (config 5), kernel-only times of the two cost kernels,
# cross-rank sweep tests (1 and 2 ranks on one device), config-5 sharded leg at one rank.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03d; mkdir -p $O
export OTF_STALL_MS=5000 TMPDIR=/tmp
timeout -k 10 60 ./tools/stamps_sweep 8192 f16 > $O/sweep_stamps.txt 2>&1; rc=$?; cat $O/sweep_stamps.txt; [ $rc -eq 0 ] || exit $rc
for r in 0 1; do
  OTF_COST_RING=$r timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof$r -o run -- python3 tools/bench_cost.py 4096 512 > $O/prof$r.log 2>&1 || exit $?
done
find $O -name "*kernel_stats.csv" | sort | while read f; do echo "== $f"; cut -d, -f1-8 "$f" | head -8; done
for r in 0 1; do for v in "" _a1; do
  echo "=== ubench_cost$v ring=$r"
  OTF_COST_RING=$r timeout -k 10 60 rocprofv3 --kernel-trace --stats -d $O/ub$r$v -o run -- ./tools/ubench_cost$v 4096 512 f32 20 > $O/ub$r$v.log 2>&1 || exit $?
  grep "per call" $O/ub$r$v.log; f=$(find $O/ub$r$v -name "*kernel_stats.csv" | head -1); cut -d, -f1-8 "$f" | head -5
done; done
bash tools/gpu_r03_e.sh
