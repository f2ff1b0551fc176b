set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|ERROR" gpurun_out/gpu_tests.log | head; tail -2 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --multi-legs --no-gw --no-batch-ot --no-cpu-baseline --no-hbm-probe --no-config5 > gpurun_out/bench_multi.log 2>&1
rc=$?; echo "bench-multi rc=$rc"; tail -c 1500 gpurun_out/bench_multi.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 4000 gpurun_out/bench.log
