#!/bin/bash
# Headline A/B of library builds (tools/alt/lib_<v>.so): bench.py's float64 step only,
# alternating builds, two rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-libab}
mkdir -p $OUT
L=ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd/otfuse/lib/libotfuse.so
for r in 1 2; do for v in ${VARS:-z cd}; do
  cp tools/alt/lib_$v.so $L
  timeout -k 10 240 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-hbm-probe --no-gw --no-f32 \
      --no-config5 --no-batch-ot > $OUT/$v.$r.log 2>&1 || exit 1
  python3 - "$OUT/$v.$r.log" "$v" "$r" <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
b = d.get("breakdown_ms", {})
print(sys.argv[2], sys.argv[3], "ms_per_step %.4f fused_call %.4f per_iter_us %.3f intercept_us %.1f" % (
    d["ms_per_step"], b.get("fused_call", 0), 1e3 * b.get("per_iteration", 0), 1e3 * b.get("intercept", 0)), flush=True)
PY
done; done
