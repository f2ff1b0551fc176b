#!/bin/bash
# r03 (w): mesh reducer spread over 1 / 2 / 4 waves (stamps A/B), gather zero-column test.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03w; mkdir -p $O
export OTF_STALL_MS=3000
timeout -k 10 300 python -u -m pytest tests/test_gpu_gather.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; grep -E "FAIL|Error|passed|failed" $O/tests.log | tail -5; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in "" _rw2 _rw4; do
    timeout -k 10 60 ./tools/stamps_resident$v 4096 mesh > $O/mesh$v.$rep.txt 2>&1 || exit $?
    echo "== rw$v rep $rep: $(grep median $O/mesh$v.$rep.txt) $(grep '= iteration' $O/mesh$v.$rep.txt)"
  done
done
