set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_config5.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "sweep or config5_full or ragged or stop" > gpurun_out/t_sweep.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/t_sweep.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/sweep_probe.py > gpurun_out/sweep_probe.log 2>&1
rc=$?; echo "probe rc=$rc"; cat gpurun_out/sweep_probe.log | tail -5
