#!/bin/bash
# r03 (l): cost kernel variants (register-staged 256^2 / LDS-DMA ring / warp-specialised)
# with phase stamps at the metric shape and config 5; mesh phase stamps; bench multi-legs
# (config-3 chain, sharded config 5).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03l; mkdir -p $O
export TMPDIR=/tmp
for cfg in "big:" "ring:OTF_COST_RING=1" "ws:OTF_COST_WS=1"; do
  name=${cfg%%:*}; envs=${cfg#*:}
  for shp in "4096 512 f32" "8192 1024 f16in"; do
    echo "=== $name $shp"; env $envs timeout -k 10 60 ./tools/ubench_cost_s0 $shp 20 || exit $?
  done
done
timeout -k 10 60 ./tools/stamps_resident 4096 mesh > $O/mesh_stamps.txt 2>&1; rc=$?; tail -22 $O/mesh_stamps.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --multi-legs --no-cpu-baseline --no-hbm-probe --no-gw > $O/bench_multi.log 2>&1; rc=$?
python3 - <<'PY'
import json
l=[x for x in open('gpurun_out/r03l/bench_multi.log') if x.startswith('{')]
d=json.loads(l[-1]) if l else {}
for k in ('sharded_config5','config3_epoch_chain'): print(k, json.dumps(d.get(k))[:900])
PY
exit $rc
