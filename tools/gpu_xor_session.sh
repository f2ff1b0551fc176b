#!/bin/bash
# Lane-exchange check, then config-2 / metric stamps and the full GPU suite.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 30 ./tools/ubench_xor > gpurun_out/xor.txt 2>&1; rc=$?; cat gpurun_out/xor.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 60 ./tools/stamps_resident 512 gather double > gpurun_out/st_g512d.txt 2>&1 && cat gpurun_out/st_g512d.txt
timeout -k 10 60 ./tools/stamps_resident 4096 tiled > gpurun_out/st_tiled4096.txt 2>&1 && cat gpurun_out/st_tiled4096.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -4 gpurun_out/gpu_tests.log; echo "pytest rc=$rc"
