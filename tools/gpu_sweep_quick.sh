#!/bin/bash
# Sweep engine: parity tests (config 5, deterministic, ragged), then the config-5 / HBM legs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export OTF_STALL_MS=5000
timeout -k 10 400 python -u -m pytest tests/test_gpu_config5.py tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/sweep_tests.log 2>&1
rc=$?; grep -E "FAIL|Error" gpurun_out/sweep_tests.log | head; tail -2 gpurun_out/sweep_tests.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-gw --no-batch-ot --no-cpu-baseline > gpurun_out/bench_s.log 2>&1; rc=$?; python -c "
import json
for l in open('gpurun_out/bench_s.log'):
    if l.startswith('{'): d=json.loads(l); print(d['sweep_config5']['us_per_sweep'], d['sweep_config5']['roofline']['frac'], d['hbm_probe']['us_per_sweep'], d['hbm_probe']['frac'])"
