#!/bin/bash
# r03 (g): ring cost kernel ablations (no stores / no MFMA / no DMA) + L2 hit counters.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03g; mkdir -p $O
export TMPDIR=/tmp OTF_COST_RING=1
for v in _a1 _a3 _a5 _a7; do
  echo "=== ring$v"
  timeout -k 10 60 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ring$v -o run -- ./tools/ubench_cost$v 4096 512 f32 20 > $O/ring$v.log 2>&1 || exit $?
  grep "per call" $O/ring$v.log; f=$(find $O/ring$v -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cut -d, -f1-4 "$f" | sed -n 2,2p
done
timeout -s KILL 60 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/pmc_tcc -o run -- ./tools/ubench_cost_a1 4096 512 f32 5 > $O/pmc_tcc.log 2>&1 || exit $?
f=$(find $O/pmc_tcc -name "*counter_collection.csv" | head -1); [ -n "$f" ] && python3 - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    acc[r.get("Kernel_Name", r.get("Kernel-Name", "?"))[:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k, {c: sum(v) / len(v) for c, v in d.items()})
PY
exit 0
