"""Summarise a tools/gpu_run.sh session (gpurun_out/<TAG>/) into tracked files under profiles/.

Usage: python tools/summarize_profile.py <round tag, e.g. r06> [session dir, default gpurun_out]
Writes, for round tag T:
  profiles/T_kernel_stats.csv      rocprofv3 --kernel-trace --stats summary (copied)
  profiles/T_summary.json          per-kernel median durations + PMC HBM bytes per launch
  profiles/kernel_traffic.json     HBM bytes per launch of each hot kernel (read by bench.py)
PMC runs: <session dir>/pmc_<COUNTER>_<leg>/ (separate --pmc passes per counter, one per
Sinkhorn engine so both the resident kernel and the streaming pass are counted).
Correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE / WRITE_SIZE are KiB; on
gfx950 FETCH_SIZE reports half the bytes of a wide coalesced stream, so it is doubled;
WRITE_SIZE is exact for 16-B streaming stores and float atomics.
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "gpurun_out")
PROF = os.path.join(REPO, "profiles")
HOT = ("sk_mesh64_kernel", "dist_mfma_f64_kernel", "sqnorm_f64_kernel", "dist_scale_kernel",
       "sk_resident_kernel", "sk_tiled_kernel", "sk_mesh_kernel", "sk_gather_kernel", "sk_pass_kernel", "sk_sweep_kernel", "cost_8ph_kernel", "cost_big_kernel", "cost_big16_kernel", "cost_split16_kernel",
       "split16_prep2_kernel", "cost_f16_kernel", "sk_init_kernel", "sk_plan_kernel")
LIB = os.path.join(REPO, "ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd",
                   "otfuse", "lib", "libotfuse.so")


def lib_md5():
    import hashlib
    try:
        return hashlib.md5(open(LIB, "rb").read()).hexdigest()
    except OSError:
        return None


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return name.split("(")[0]


def medians(path, value=None):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        v = float(r[value]) if value else int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        d[short(r["Kernel_Name"])].append(v)
    return {k: sorted(v)[len(v) // 2] for k, v in d.items()}, {k: len(v) for k, v in d.items()}


def base_name(k):
    if k.startswith("_ZN"):  # mangled name (e.g. _Float16 arguments): last <len><id> component
        i, last = 3, k
        while i < len(k) and k[i].isdigit():
            j = i
            while k[j].isdigit():
                j += 1
            n = int(k[i:j])
            last, i = k[j:j + n], j + n
        return last
    k = k.split("<")[0]
    return k.split("::")[-1]


def main():
    global OUT
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    if len(sys.argv) > 2:
        OUT = os.path.abspath(sys.argv[2])
    os.makedirs(PROF, exist_ok=True)
    shutil.copy(os.path.join(OUT, "prof", "run_kernel_stats.csv"),
                os.path.join(PROF, f"{tag}_kernel_stats.csv"))
    dur, cnt = medians(os.path.join(OUT, "prof", "run_kernel_trace.csv"))
    summary = {"kernels": {k: {"median_us": dur[k] / 1e3, "launches": cnt[k]} for k in dur}}
    # config-5 passes (pmc_*_c5, bench.py --profile-config5: N = 8192 fp16, sweep engine)
    # go to their own section: same kernel names, different shapes
    summary["config5_kernels"] = {}
    c5trace = os.path.join(OUT, "prof_c5", "run_kernel_trace.csv")
    if os.path.exists(c5trace):
        d5, n5 = medians(c5trace)
        summary["config5_kernels"] = {k: {"median_us": d5[k] / 1e3, "launches": n5[k]} for k in d5}
    # the float32 metric leg (bench.py --profile-only --profile-f32: split-fp16 cost + float32
    # mesh); since r05 "prof" / pmc_*_auto are the float64 headline step
    summary["f32_kernels"] = {}
    f32trace = os.path.join(OUT, "prof_f32", "run_kernel_trace.csv")
    if os.path.exists(f32trace):
        d6, n6 = medians(f32trace)
        summary["f32_kernels"] = {k: {"median_us": d6[k] / 1e3, "launches": n6[k]} for k in d6}
        shutil.copy(os.path.join(OUT, "prof_f32", "run_kernel_stats.csv"),
                    os.path.join(PROF, f"{tag}_f32_kernel_stats.csv"))
    if os.path.exists(c5trace):
        shutil.copy(os.path.join(OUT, "prof_c5", "run_kernel_stats.csv"),
                    os.path.join(PROF, f"{tag}_config5_kernel_stats.csv"))
    for ctr, factor in (("FETCH_SIZE", 2.0), ("WRITE_SIZE", 1.0)):
        for p in glob.glob(os.path.join(OUT, f"pmc_{ctr}*", "run_counter_collection.csv")):
            med, _ = medians(p, "Counter_Value")
            leaf = os.path.basename(os.path.dirname(p))
            sect = "config5_kernels" if leaf.endswith("_c5") else "f32_kernels" if leaf.endswith("_f32") else "kernels"
            for k, v in med.items():
                summary[sect].setdefault(k, {})[ctr + "_bytes_corrected"] = v * 1024 * factor
    # MFMA utilisation pass: busy fraction = MFMA busy cycles / (1024 SIMDs x kernel
    # cycles), kernel cycles from GRBM_GUI_ACTIVE / 8 (summed over the 8 XCDs)
    mf = os.path.join(OUT, "pmc_MFMA_auto", "run_counter_collection.csv")
    if os.path.exists(mf):
        per = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(mf)):
            per[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, d in per.items():
            busy = sorted(d.get("SQ_VALU_MFMA_BUSY_CYCLES", [0]))[len(d.get("SQ_VALU_MFMA_BUSY_CYCLES", [0])) // 2]
            gui = sorted(d.get("GRBM_GUI_ACTIVE", [0]))[len(d.get("GRBM_GUI_ACTIVE", [0])) // 2]
            if busy > 0 and gui > 0:
                summary["kernels"].setdefault(k, {})["mfma_busy_frac"] = busy / 1024.0 / (gui / 8.0)
                summary["kernels"][k]["SQ_VALU_MFMA_BUSY_CYCLES"] = busy
                summary["kernels"][k]["GRBM_GUI_ACTIVE"] = gui
    bench = os.path.join(OUT, "bench.log")
    cfg = {}
    if os.path.exists(bench):
        lines = [ln for ln in open(bench).read().splitlines() if ln.startswith("{")]
        if lines:
            summary["bench"] = json.loads(lines[-1])
            cfg = summary["bench"].get("config", {})
    json.dump(summary, open(os.path.join(PROF, f"{tag}_summary.json"), "w"), indent=1)
    traffic = {}
    for k, v in list(summary["f32_kernels"].items()) + list(summary["kernels"].items()):
        b = base_name(k)
        if b in HOT and "FETCH_SIZE_bytes_corrected" in v:
            traffic[b] = {"kernel": k, "median_us": v.get("median_us"),
                          "fetch_bytes_per_launch": v["FETCH_SIZE_bytes_corrected"],
                          "write_bytes_per_launch": v.get("WRITE_SIZE_bytes_corrected"),
                          "hbm_bytes_per_launch": v["FETCH_SIZE_bytes_corrected"]
                          + v.get("WRITE_SIZE_bytes_corrected", 0.0)}
    if traffic:
        json.dump({"n": cfg.get("N", 4096), "iters": cfg.get("iters", 100), "round": tag,
                   "lib_md5": lib_md5(),
                   "source": f"profiles/{tag}_summary.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE "
                             "with --kernel-trace --stats only, separate passes; FETCH x2 gfx950 "
                             "correction)",
                   "kernels": traffic},
                  open(os.path.join(PROF, "kernel_traffic.json"), "w"), indent=1)
    for k, v in summary["kernels"].items():
        print(f"{k[:70]:70s} {v}")


if __name__ == "__main__":
    main()
