#!/bin/bash
# r03 (gpend): gather polls reloading only the producers not yet seen (OTF_GATHER_PEND=1,
# stamps_resident_gt1 / gp1) against reloading all of them (gt0 / gp0), config-2 shape
# (512^2 float64); gather tests; config-2 training step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03gpend; mkdir -p $O
export TMPDIR=/tmp OTF_STALL_MS=3000
for rep in 1 2 3; do
  for v in gt0 gt1; do
    timeout -k 10 60 tools/stamps_resident_$v 512 gather double > $O/$v.$rep.txt 2>&1; rc=$?
    echo "$v.$rep $(grep -E 'solve' $O/$v.$rep.txt | tail -1) $(grep -E 'MISMATCH' $O/$v.$rep.txt)"; [ $rc -eq 0 ] || exit $rc
  done
done
for v in gp0 gp1; do
  timeout -k 10 60 tools/stamps_resident_$v 512 gather double > $O/$v.txt 2>&1; rc=$?
  echo "== $v"; tail -9 $O/$v.txt; [ $rc -eq 0 ] || exit $rc
done
export OTF_STALL_MS=5000
timeout -k 10 400 python -u -m pytest tests/test_gpu_gather.py tests/test_gpu_align.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; grep -E "FAIL|Error|passed|failed" $O/tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
unset OTF_STALL_MS
timeout -k 10 120 python -u tools/c2_probe.py 30 > $O/c2.log 2>&1; rc=$?; tail -5 $O/c2.log; exit $rc
