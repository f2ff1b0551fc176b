#!/bin/bash
# A/B of library environment switches on the headline bench (no extra legs): every
# configuration in $AB (space-separated; a configuration is comma-separated NAME=VALUE
# pairs, "-" = defaults) runs $REPS times, interleaved.
#   AB="- OTF_FALLBACK=0" REPS=3 bash tools/gpu_ab_env.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abenv
export TMPDIR=/tmp
ARGS="--steps 20 --warmup 3 --no-gw --no-config5 --no-cpu-baseline --no-hbm-probe --no-batch-ot --no-f64 ${EXTRA:-}"
k=0
for rep in $(seq 1 "${REPS:-2}"); do
  for cfg in ${AB:--}; do
    k=$((k + 1))
    envs=()
    if [ "$cfg" != "-" ]; then IFS=',' read -r -a envs <<< "$cfg"; fi
    log=gpurun_out/abenv/run_$k.log
    env "${envs[@]}" timeout -k 10 300 python bench.py $ARGS > "$log" 2>&1 || { echo "rc=$? in $cfg"; exit 1; }
    echo "$cfg: $(python -c "import json; d=json.loads(open('$log').read().strip().splitlines()[-1]); print(round(d['value']), round(d['ms_per_step'] * 1000, 2), 'us/step', d['breakdown_ms'], 'prep', d.get('cost_roofline', {}).get('prep_us'), 'kernel', d.get('cost_roofline', {}).get('kernel_us'))")"
  done
done
exit 0
