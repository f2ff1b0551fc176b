#!/bin/bash
# r03 (e): cross-rank sweep tests (1 and 2 ranks on one device), config-5 sharded leg.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03e; mkdir -p $O
export OTF_STALL_MS=5000
timeout -k 10 300 python -u -m pytest tests/test_gpu_xsweep.py tests/test_gpu_parity.py -k "xsweep or break_all or ragged" -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/t_xsweep.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|Error" $O/t_xsweep.log | tail -30; echo "pytest rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u -c "
import sys, json, torch
sys.path.insert(0, '.'); sys.path.insert(0, 'ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd')
import bench
print(json.dumps(bench.sharded_config5_leg(torch.device('cuda', 0), 1)))
print(json.dumps(bench.config3_leg(torch.device('cuda', 0), 1)))
" > $O/sharded1.json 2>&1; rc=$?; tail -3 $O/sharded1.json; exit $rc
