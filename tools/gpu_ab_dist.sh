set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
TESTS="tests/test_gpu_gw.py tests/test_gpu_precision.py::test_metric_shape_float64_leg_vs_oracle tests/test_gpu_mesh64.py" bash tools/gpu_quick.sh || exit $?
for v in 1 0 1 0; do
  OTF_DIST_MFMA=$v timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-gw --no-config5 --no-cpu-baseline --no-hbm-probe --no-batch-ot > gpurun_out/ab_dist_$v.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/ab_dist_$v.log').read().strip().splitlines()[-1]); m=d['metric_f64']; print('mfma=$v', m['cost_ms'], m['sinkhorn_incl_plan_ms'], m['ms_per_step'])"
done
