#!/bin/bash
# r03 (u): training-step launch trims (cached marginals, gather region zeroed by init):
# gather / align / configs tests, config-2 step (pipelined + isolated), config-3 trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03u; mkdir -p $O
export TMPDIR=/tmp OTF_STALL_MS=5000
timeout -k 10 500 python -u -m pytest tests/test_gpu_align.py tests/test_gpu_gather.py tests/test_gpu_configs.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; grep -E "FAIL|Error|passed|failed" $O/tests.log | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/c2_probe.py 30 || exit $?
unset OTF_STALL_MS
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 2 --warmup 1 --multi-legs --no-gw --no-cpu-baseline --no-hbm-probe --no-config5 --no-f64 > $O/bench.log 2>&1; rc=$?
grep -o '"config3_epoch_chain": {[^}]*}' $O/bench.log; grep -o '"batch_ot_per_step": {[^}]*}' $O/bench.log; exit $rc
