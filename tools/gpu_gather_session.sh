#!/bin/bash
# Gather-engine session: config-2 stamps, gather / parity tests, the config-2 bench leg.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 60 ./tools/stamps_resident 512 gather double > gpurun_out/st_g512d.txt 2>&1; cat gpurun_out/st_g512d.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_gather.py tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread -k "gather or deterministic or f2 or f3 or stop_and_break or early_stop" > gpurun_out/gather_tests.log 2>&1
rc=$?; tail -15 gpurun_out/gather_tests.log; echo "pytest rc=$rc"
[ $rc -le 1 ] && timeout -k 10 120 python -c "
import json, torch, bench
print(json.dumps(bench.batch_ot_leg(torch.device('cuda:0'), False)))
" > gpurun_out/batch_ot.log 2>&1; cat gpurun_out/batch_ot.log | tail -3
