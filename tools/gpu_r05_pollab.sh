#!/bin/bash
# A/B of float32 mesh poll variants (tools/alt/lib_<v>.so): kernel time + FETCH_SIZE of
# the float32 metric leg for each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-pollab}
mkdir -p $OUT
export TMPDIR=/tmp
L=ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd/otfuse/lib/libotfuse.so
B="python3 bench.py --profile-only --profile-f32 --steps 5 --warmup 1"
for v in ${VARS:-z a b c d e}; do
  mkdir -p $OUT/$v && cp tools/alt/lib_$v.so $L
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/$v/kt -o run --output-format csv -- $B > $OUT/$v/kt.log 2>&1 || exit 1
  timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/$v/f -o run --output-format csv -- $B > $OUT/$v/f.log 2>&1 || exit 1
  python3 - "$OUT/$v" "$v" <<'PY'
import csv, sys
o, v = sys.argv[1], sys.argv[2]
t = [r for r in csv.DictReader(open(f"{o}/kt/run_kernel_stats.csv")) if "sk_mesh_kernel" in r["Name"]][0]
x = sorted(float(r["Counter_Value"]) for r in csv.DictReader(open(f"{o}/f/run_counter_collection.csv"))
           if "sk_mesh_kernel" in r["Kernel_Name"])
print(v, "avg_us", float(t["AverageNs"]) / 1e3, "min_us", float(t["MinNs"]) / 1e3, "fetch_MB", x[len(x) // 2] * 1024 / 1e6, flush=True)
PY
done
