#!/bin/bash
# A/B of the two-hop mesh (OTF_MESH2=1) against the three-hop mesh at the metric shape:
# headline bench (no extra legs) and a rocprofv3 kernel trace of each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
ARGS="--steps 20 --warmup 3 --no-gw --no-config5 --no-cpu-baseline --no-hbm-probe --no-batch-ot --no-f64"
for m2 in 0 1 0 1; do
  OTF_MESH2=$m2 timeout -k 10 300 python bench.py $ARGS > gpurun_out/ab/bench_m2_$m2.log 2>&1 || exit $?
  echo "mesh2=$m2: $(python -c "import json,sys; d=json.loads(open('gpurun_out/ab/bench_m2_$m2.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['achieved'], d['breakdown_ms'])")"
done
for m2 in 0 1; do
  OTF_MESH2=$m2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab/prof_m2_$m2 -o run --output-format csv -- python3 bench.py --profile-only --steps 10 --warmup 2 > gpurun_out/ab/rocprof_m2_$m2.log 2>&1 || exit $?
done
python tools/summarize_profile.py gpurun_out/ab/prof_m2_0 > gpurun_out/ab/sum0.txt 2>&1 || true
python tools/summarize_profile.py gpurun_out/ab/prof_m2_1 > gpurun_out/ab/sum1.txt 2>&1 || true
grep -h "sk_mesh" gpurun_out/ab/prof_m2_*/*/*kernel_stats.csv 2>/dev/null | cut -c1-200 || true
exit 0
