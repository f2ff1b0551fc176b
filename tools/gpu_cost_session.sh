# GPU session: cost-kernel parity tests, then the cost probe for the current library and
# (if present) tools/alt/libotfuse_old.so swapped in for an A/B.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
LIB=ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd/otfuse/lib
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "cost or split16 or config5 or feature" > gpurun_out/t_cost.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR" gpurun_out/t_cost.log | head -40; tail -2 gpurun_out/t_cost.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python tools/cost_probe.py > gpurun_out/cost_probe_new.log 2>&1
rc=$?; echo "probe new rc=$rc"; cat gpurun_out/cost_probe_new.log | grep case
if [ $rc -ne 0 ]; then exit $rc; fi
if [ -f tools/alt/libotfuse_old.so ]; then
  cp $LIB/libotfuse.so /tmp/libnew.so && cp tools/alt/libotfuse_old.so $LIB/libotfuse.so
  timeout -k 10 120 python tools/cost_probe.py > gpurun_out/cost_probe_old.log 2>&1
  rc=$?; echo "probe old rc=$rc"; grep case gpurun_out/cost_probe_old.log
  cp /tmp/libnew.so $LIB/libotfuse.so
fi
exit $rc
