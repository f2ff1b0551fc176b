# GPU session for the sweep engine: parity tests, timing probe, phase stamps.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_config5.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "sweep or config5_full or ragged or stop" > gpurun_out/t_sweep.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/t_sweep.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/sweep_probe.py > gpurun_out/sweep_probe.log 2>&1
rc=$?; echo "probe rc=$rc"; tail -3 gpurun_out/sweep_probe.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 60 tools/stamps_sweep 8192 f16 > gpurun_out/stamps_sweep.log 2>&1
rc=$?; echo "stamps rc=$rc"; cat gpurun_out/stamps_sweep.log
