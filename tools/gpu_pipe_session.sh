# GPU session: sweep-engine parity subset, then the timing probe and phase stamps under
# each environment variant in $VARIANTS (space-separated VAR=value, "-" = defaults).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_config5.py tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "sweep or config5_full or ragged or stop or nan or determin" > gpurun_out/t_sweep.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/t_sweep.log
if [ $rc -ne 0 ]; then exit $rc; fi
i=0
for var in ${VARIANTS:--}; do
  i=$((i+1))
  envs=""; [ "$var" != "-" ] && envs="$var"
  env $envs timeout -k 10 300 python tools/sweep_probe.py --cases ${CASES:-c5,n16k} > gpurun_out/sweep_probe_v$i.log 2>&1
  rc=$?; echo "== variant $var: probe rc=$rc"; cut -c1-260 gpurun_out/sweep_probe_v$i.log | grep case
  if [ $rc -ne 0 ]; then exit $rc; fi
  env $envs timeout -k 10 60 tools/stamps_sweep 8192 f16 > gpurun_out/stamps_v$i.log 2>&1
  rc=$?; echo "stamps rc=$rc"; grep -v "^rc=" gpurun_out/stamps_v$i.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
