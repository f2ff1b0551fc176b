#!/bin/bash
# r03 (kpre): the mesh engine's K built before the registration barrier (stamps_mesh_k1)
# against after it (k0), interleaved; mesh tests; headline bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03kpre; mkdir -p $O
export TMPDIR=/tmp OTF_STALL_MS=3000
for rep in 1 2 3; do
  for v in k0 k1; do
    timeout -k 10 60 tools/stamps_mesh_$v 4096 100 9 > $O/$v.$rep.txt 2>&1; rc=$?
    echo "$v.$rep $(grep -E 'median|MISMATCH' $O/$v.$rep.txt)"; [ $rc -eq 0 ] || exit $rc
  done
done
export OTF_STALL_MS=5000
timeout -k 10 400 python -u -m pytest tests/test_gpu_mesh.py tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; grep -E "FAIL|Error|passed|failed" $O/tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
unset OTF_STALL_MS
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-hbm-probe --no-config5 --no-f64 --no-gw --no-batch-ot > $O/bench.log 2>&1; rc=$?
head -c 400 $O/bench.log; exit $rc
