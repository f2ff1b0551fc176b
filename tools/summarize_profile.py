"""Summarise a gpu_session.sh run (gpurun_out/) into tracked files under profiles/.

Writes, for round tag T (argv[1], e.g. r01):
  profiles/T_kernel_stats.csv      rocprofv3 --kernel-trace --stats summary (copied)
  profiles/T_summary.json          per-kernel median durations + PMC HBM bytes per launch
  profiles/pass_traffic.json       HBM bytes per launch of the Sinkhorn pass (read by bench.py)
PMC correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE / WRITE_SIZE are KiB;
on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced stream, so it is
doubled; WRITE_SIZE is exact for 16-B streaming stores and float atomics.
"""
import collections
import csv
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "gpurun_out")
PROF = os.path.join(REPO, "profiles")


def medians(path, value=None):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        v = float(r[value]) if value else int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        d[name.split("(")[0]].append(v)
    return {k: sorted(v)[len(v) // 2] for k, v in d.items()}, {k: len(v) for k, v in d.items()}


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    os.makedirs(PROF, exist_ok=True)
    shutil.copy(os.path.join(OUT, "prof", "run_kernel_stats.csv"),
                os.path.join(PROF, f"{tag}_kernel_stats.csv"))
    dur, cnt = medians(os.path.join(OUT, "prof", "run_kernel_trace.csv"))
    summary = {"kernels": {k: {"median_us": dur[k] / 1e3, "launches": cnt[k]} for k in dur}}
    pmc = {}
    for ctr, factor in (("FETCH_SIZE", 2.0), ("WRITE_SIZE", 1.0)):
        p = os.path.join(OUT, f"pmc_{ctr}", "run_counter_collection.csv")
        if os.path.exists(p):
            med, _ = medians(p, "Counter_Value")
            for k, v in med.items():
                pmc.setdefault(k, {})[ctr + "_bytes_corrected"] = v * 1024 * factor
    for k, v in pmc.items():
        summary["kernels"].setdefault(k, {}).update(v)
    bench = os.path.join(OUT, "bench.log")
    if os.path.exists(bench):
        lines = [ln for ln in open(bench).read().splitlines() if ln.startswith("{")]
        if lines:
            summary["bench"] = json.loads(lines[-1])
    json.dump(summary, open(os.path.join(PROF, f"{tag}_summary.json"), "w"), indent=1)
    pas = [k for k in summary["kernels"] if "sk_pass_kernel" in k]
    if pas and "FETCH_SIZE_bytes_corrected" in summary["kernels"][pas[0]]:
        kk = summary["kernels"][pas[0]]
        n = summary.get("bench", {}).get("config", {}).get("N", 4096)
        json.dump({"n": n, "kernel": pas[0], "round": tag,
                   "hbm_bytes_per_launch": kk["FETCH_SIZE_bytes_corrected"] + kk.get("WRITE_SIZE_bytes_corrected", 0.0),
                   "fetch_bytes_per_launch": kk["FETCH_SIZE_bytes_corrected"],
                   "write_bytes_per_launch": kk.get("WRITE_SIZE_bytes_corrected"),
                   "source": f"profiles/{tag}_summary.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, "
                             "separate passes, FETCH x2 gfx950 correction)"},
                  open(os.path.join(PROF, "pass_traffic.json"), "w"), indent=1)
    for k, v in summary["kernels"].items():
        print(f"{k[:70]:70s} {v}")


if __name__ == "__main__":
    main()
