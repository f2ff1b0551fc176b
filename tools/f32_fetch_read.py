"""Counter rows of the float32 mesh launches of tools/f32_fetch_probe.py, by config."""
import csv
import sys

for path in sys.argv[1:]:
    rows = [r for r in csv.DictReader(open(path)) if "sk_mesh_kernel" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    cfg = [(it, pl) for it in (1, 10, 100) for pl in ("plan", "noplan") for _ in range(3)]
    ctr = rows[0]["Counter_Name"]
    for i in range(0, len(rows), 3):
        vals = [float(r["Counter_Value"]) * 1024 / 1e6 for r in rows[i:i + 3]]
        print(ctr, "iters %d %s" % cfg[i], "raw MB", " ".join("%.2f" % v for v in vals))
