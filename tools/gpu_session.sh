#!/bin/bash
# One GPU-box session: parity tests, bench, rocprofv3 kernel trace (+ optional PMC
# passes).  Each GPU step has its own time limit; a crash / abort / timeout (rc not
# 0 or 1) ends the session.  Env: TESTS=0/1 BENCH=0/1 PROFILE=0/1 PMC=0/1
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_if_fatal() { if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "fatal rc=$1 in $2, stopping"; exit "$1"; fi; }

if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_tests.log; stop_if_fatal $rc pytest
fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 420 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log; stop_if_fatal $rc bench
fi
if [ "${PROFILE:-1}" = "1" ]; then
  timeout -k 10 420 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --profile-only --steps 10 --warmup 2 > gpurun_out/rocprof.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; stop_if_fatal $rc rocprof
fi
if [ "${PROFILE:-1}" = "1" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o run --output-format csv -- python3 bench.py --profile-only --profile-config5 --steps 3 > gpurun_out/rocprof_c5.log 2>&1
  rc=$?; echo "rocprof c5 rc=$rc"; stop_if_fatal $rc rocprof_c5
fi
if [ "${PROFILE:-1}" = "1" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_f64 -o run --output-format csv -- python3 bench.py --profile-only --profile-f64 --steps 5 > gpurun_out/rocprof_f64.log 2>&1
  rc=$?; echo "rocprof f64 rc=$rc"; stop_if_fatal $rc rocprof_f64
fi
if [ "${PMC:-0}" = "1" ]; then
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace --stats -d gpurun_out/pmc_${ctr}_c5 -o run --output-format csv -- python3 bench.py --profile-only --profile-config5 --steps 2 > gpurun_out/pmc_${ctr}_c5.log 2>&1
    rc=$?; echo "pmc $ctr c5 rc=$rc"; stop_if_fatal $rc pmc_c5
  done
fi
if [ "${PMC:-0}" = "1" ]; then
  for eng in auto stream; do
    for ctr in FETCH_SIZE WRITE_SIZE; do
      timeout -k 10 420 rocprofv3 --pmc $ctr --kernel-trace --stats -d gpurun_out/pmc_${ctr}_$eng -o run --output-format csv -- python3 bench.py --profile-only --engine $eng --steps 3 --warmup 1 > gpurun_out/pmc_${ctr}_$eng.log 2>&1
      rc=$?; echo "pmc $ctr $eng rc=$rc"; stop_if_fatal $rc pmc
    done
  done
fi
if [ "${PMC:-0}" = "1" ]; then
  # MFMA utilisation of the cost kernel (SQ_VALU_MFMA_BUSY_CYCLES over all SIMDs; clock
  # from GRBM_GUI_ACTIVE / 8 XCDs), one pass of its own
  timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --stats -d gpurun_out/pmc_MFMA_auto -o run --output-format csv -- python3 bench.py --profile-only --steps 3 --warmup 1 > gpurun_out/pmc_MFMA_auto.log 2>&1
  rc=$?; echo "pmc MFMA rc=$rc"; stop_if_fatal $rc pmc_mfma
fi
exit 0
