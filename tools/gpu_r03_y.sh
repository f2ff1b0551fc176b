#!/bin/bash
# r03 (y): unrolled align-backward loop: align tests, config-2 step, kernel time.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03y; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_align.py tests/test_gpu_configs.py -k "align or config2 or batch" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; grep -E "FAIL|Error|passed|failed" $O/tests.log | tail -6; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/c2_probe.py 30 > $O/c2.log 2>&1 || exit $?
grep "config-2" $O/c2.log; python3 -c "
import csv
for r in csv.DictReader(open('$O/prof/run_kernel_stats.csv')):
    if any(k in r['Name'] for k in ('align','gather','postprocess','gemm','cost')): print(r['Calls'], round(float(r['AverageNs'])/1e3,1), r['Name'][:80])
"
