#!/bin/bash
# r03 (poll): the mesh engine's granule polls with two loads in flight (OTF_POLL2=1,
# stamps_mesh_p1) against load-wait-reload (p0); mesh tests; headline bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03poll; mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu_mesh_stamps.sh p0 p1 > $O/stamps.txt 2>&1; rc=$?
grep -E "median|===|iteration|row hop|hop B|reducer" $O/stamps.txt; [ $rc -eq 0 ] || exit $rc
export OTF_STALL_MS=5000
timeout -k 10 400 python -u -m pytest tests/test_gpu_mesh.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; grep -E "FAIL|Error|passed|failed" $O/tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
unset OTF_STALL_MS
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-hbm-probe --no-config5 --no-f64 > $O/bench.log 2>&1; rc=$?
tail -c 600 $O/bench.log; exit $rc
