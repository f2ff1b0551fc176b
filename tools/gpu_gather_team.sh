#!/bin/bash
# Gather engine XCC team mode: config-2 stamps (team / write-through), gather tests, batch-OT leg.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export OTF_STALL_MS=3000
timeout -k 10 60 ./tools/stamps_resident 512 gather double > gpurun_out/st_gather_team.txt 2>&1; rc=$?; cat gpurun_out/st_gather_team.txt
[ $rc -eq 0 ] || exit $rc
OTF_GATHER_TEAM=0 timeout -k 10 60 ./tools/stamps_resident 512 gather double > gpurun_out/st_gather_wt.txt 2>&1; rc=$?; cat gpurun_out/st_gather_wt.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_gather.py tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gather_tests.log 2>&1
rc=$?; grep -E "FAIL|Error" gpurun_out/gather_tests.log | head; tail -3 gpurun_out/gather_tests.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-gw --no-config5 --no-cpu-baseline --no-hbm-probe > gpurun_out/bench_b.log 2>&1; rc=$?; python -c "
import json
for l in open('gpurun_out/bench_b.log'):
    if l.startswith('{'): d=json.loads(l); print(d['batch_ot_per_step'])"
