#!/bin/bash
# Cost kernels: parity tests, then the timing / accuracy probe (both tile sizes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_config5.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "cost or split16 or config5 or metric" > gpurun_out/cost_tests.log 2>&1
rc=$?; tail -3 gpurun_out/cost_tests.log; echo "cost pytest rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python tools/cost_probe.py > gpurun_out/cost_probe_big.log 2>&1; rc=$?; cat gpurun_out/cost_probe_big.log
[ $rc -eq 0 ] || exit $rc
OTF_COST_BIG=0 timeout -k 10 120 python tools/cost_probe.py > gpurun_out/cost_probe_small.log 2>&1; rc=$?; cat gpurun_out/cost_probe_small.log
