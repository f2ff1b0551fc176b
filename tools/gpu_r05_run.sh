#!/bin/bash
# r05 GPU session: targeted tests first ($FIRST, default the float64 mesh), then the whole
# -m gpu suite (FULL=1), then the default bench (BENCH=1) -- each under its own limit,
# stop at the first fatal status.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r05}
mkdir -p $OUT
export TMPDIR=/tmp
FIRST=${FIRST:-tests/test_gpu_mesh64.py}
timeout -k 10 ${FIRST_LIMIT:-300} python -u -m pytest $FIRST -m gpu -v -x --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/first_tests.log 2>&1
rc=$?; echo "first rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" $OUT/first_tests.log | tail -30
if [ $rc -ne 0 ]; then exit $rc; fi
if [ "${FULL:-0}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|ERROR" $OUT/gpu_tests.log | head -30; tail -2 $OUT/gpu_tests.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
if [ "${BENCH:-0}" = "1" ]; then
  timeout -k 10 600 python bench.py --steps 20 --warmup 3 ${BENCH_ARGS:-} > $OUT/bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -c 4000 $OUT/bench.log
  exit $rc
fi
exit 0
