#!/bin/bash
# r03 (z): wave-form LSE sweeps in the entropic GW (<= 64 x 64): GW / configs tests,
# GW per-epoch leg, config-3 chain.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03z; mkdir -p $O
export TMPDIR=/tmp OTF_STALL_MS=5000
timeout -k 10 600 python -u -m pytest tests/test_gpu_gw.py tests/test_gpu_configs.py tests/test_gpu_coot.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; grep -E "FAIL|Error|passed|failed" $O/tests.log | tail -12; [ $rc -eq 0 ] || exit $rc
unset OTF_STALL_MS
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --multi-legs --no-batch-ot --no-cpu-baseline --no-hbm-probe --no-config5 --no-f64 > $O/bench.log 2>&1; rc=$?
grep -o '"config3_epoch_chain": {[^}]*}' $O/bench.log; grep -o '"gw_per_epoch": {.*"pot_entropic_pgd' $O/bench.log | cut -c1-500; exit $rc
