# GPU session: sweep-engine pipeline variants (OTF_SWEEP_PIPE 1 = default library,
# 2 = otfuse/lib/libotfuse_pipe2.so): parity of the default, probe + stamps of both.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
LIB=ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd/otfuse/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_config5.py tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "sweep or config5_full or ragged or stop or nan or determin" > gpurun_out/t_sweep.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/t_sweep.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/sweep_probe.py --cases c5,n16k > gpurun_out/sweep_probe_p1.log 2>&1
rc=$?; echo "probe1 rc=$rc"; cat gpurun_out/sweep_probe_p1.log | tail -2
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 60 tools/stamps_sweep 8192 f16 > gpurun_out/stamps_p1.log 2>&1
rc=$?; echo "stamps1 rc=$rc"; cat gpurun_out/stamps_p1.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 60 tools/stamps_sweep_p2 8192 f16 > gpurun_out/stamps_p2.log 2>&1
rc=$?; echo "stamps2 rc=$rc"; cat gpurun_out/stamps_p2.log
if [ $rc -ne 0 ]; then exit $rc; fi
cp $LIB/libotfuse.so /tmp/libotfuse_p1.so && cp $LIB/libotfuse_pipe2.so $LIB/libotfuse.so
timeout -k 10 300 python tools/sweep_probe.py --cases c5,n16k > gpurun_out/sweep_probe_p2.log 2>&1
rc=$?; echo "probe2 rc=$rc"; tail -2 gpurun_out/sweep_probe_p2.log
cp /tmp/libotfuse_p1.so $LIB/libotfuse.so
exit $rc
