# rocprofv3 kernel stats of the cost probe, current library and tools/alt/libotfuse_old.so
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp && cd - > /dev/null
LIB=ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd/otfuse/lib
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/cprof_new -o run -- python3 tools/cost_probe.py > gpurun_out/cprof_new.log 2>&1
rc=$?; echo "prof new rc=$rc"
if [ $rc -ne 0 ]; then tail -20 gpurun_out/cprof_new.log; exit $rc; fi
python3 - <<PYEOF
import sqlite3
for tag in ("new","old"):
    try: c=sqlite3.connect(f"gpurun_out/cprof_{tag}/run_results.db")
    except Exception: continue
    try: rows=list(c.execute("select name, grid_x, count(*), avg(end-start)/1000.0 from kernels where name like \"%cost%\" or name like \"%prep%\" group by name, grid_x order by name, grid_x"))
    except Exception: continue
    print(tag)
    for r in rows: print("  %-40s grid=%8d n=%3d avg=%8.2f" % (r[0][25:65], r[1], r[2], r[3]))
PYEOF
if [ -f tools/alt/libotfuse_old.so ]; then
  cp $LIB/libotfuse.so /tmp/libnew.so && cp tools/alt/libotfuse_old.so $LIB/libotfuse.so
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/cprof_old -o run -- python3 tools/cost_probe.py > gpurun_out/cprof_old.log 2>&1
  rc=$?; echo "prof old rc=$rc"
  cp /tmp/libnew.so $LIB/libotfuse.so
fi
exit $rc
