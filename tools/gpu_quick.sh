#!/bin/bash
# Targeted GPU check: the pytest node ids in $TESTS (each under one time limit), then
# (BENCH=1) a short bench with the extra legs named in $BENCH_ARGS.  Stops at the first
# fatal status (anything but pytest's 0 / 1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 "${TEST_LIMIT:-400}" python -u -m pytest $TESTS -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/quick_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/quick_tests.log | tail -40
  if [ $rc -gt 1 ]; then exit $rc; fi
fi
if [ "${BENCH:-0}" = "1" ]; then
  timeout -k 10 300 python bench.py --steps "${STEPS:-5}" --warmup 1 ${BENCH_ARGS:-} > gpurun_out/quick_bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/quick_bench.log | cut -c1-3000
  [ $rc -ne 0 ] && exit $rc
fi
exit 0
