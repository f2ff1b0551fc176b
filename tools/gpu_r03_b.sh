#!/bin/bash
# r03: gather-engine stamps (config 2), the fused alignment kernels, engine tests, a
# short bench without the CPU baseline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export OTF_STALL_MS=3000
for b in stamps_resident_g stamps_resident_g_st; do
  echo "=== $b"; timeout -k 10 60 ./tools/$b 512 gather double > gpurun_out/$b.txt 2>&1; rc=$?; cat gpurun_out/$b.txt; [ $rc -eq 0 ] || exit $rc
done
bash tools/gpu_mesh_stamps.sh v2 || exit $?
timeout -k 10 900 python -u -m pytest tests/test_gpu_align.py tests/test_gpu_gather.py tests/test_gpu_mesh.py tests/test_gpu_parity.py tests/test_gpu_precision.py tests/test_gpu_coot.py tests/test_gpu_configs.py -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r03b_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r03b_tests.log; echo "pytest rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-hbm-probe --no-gw > gpurun_out/r03b_bench.log 2>&1; rc=$?; tail -c 3000 gpurun_out/r03b_bench.log; exit $rc
