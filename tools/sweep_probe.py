"""Timing probe of the persistent sweep engine vs the streaming engine (GPU box).

Prints one JSON line per case: ms per solve without the plan (so per-iteration time
= ms / (iters + 1) sweeps incl. the prologue), with the plan, and the stream engine's
mean pass time, plus the implied GB/s of one cost read per sweep.
    python tools/sweep_probe.py [--cases c5,n16k,n4k]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd")
for _p in (PKG, REPO):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def timed(fn, reps=3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return sorted(ts)[len(ts) // 2]


def case(name, N, d, iters, cost_dtype, engines):
    from otfuse import ops
    from otfuse.synthetic import paired_embeddings
    dev = torch.device("cuda", 0)
    X, Y, _ = paired_embeddings(N, d, seed=1234)
    if cost_dtype == torch.float16:
        C, cmax, _ = ops.pairwise_cost_ex(torch.from_numpy(X.astype(np.float16)).to(dev),
                                          torch.from_numpy(Y.astype(np.float16)).to(dev),
                                          out_dtype=torch.float16)
    else:
        C, cmax = ops.pairwise_cost(torch.from_numpy(X).to(dev), torch.from_numpy(Y).to(dev))
    a = torch.full((N,), 1.0 / N, device=dev)
    ws = ops.sinkhorn_workspace(N, N, torch.float32, iters, dev)
    esz = C.element_size()
    out = {"case": name, "N": N, "iters": iters, "cost_bytes": N * N * esz}
    for eng in engines:
        r = {}
        r["ms_no_plan"] = timed(lambda: ops.sinkhorn(a, a, C, 0.1, max_iter=iters, stop_thr=0.0,
                                                     cost_scale=cmax, workspace=ws, want_plan=False,
                                                     engine=eng))
        res = ops.sinkhorn(a, a, C, 0.1, max_iter=iters, stop_thr=0.0, cost_scale=cmax,
                           workspace=ws, want_plan=False, engine=eng)
        info = res.info()
        r["engine"] = info["engine_name"]
        r["status"] = info["status_name"]
        r["us_per_sweep"] = r["ms_no_plan"] * 1e3 / (iters + 1)
        r["gbs"] = N * N * esz / (r["us_per_sweep"] * 1e-6) / 1e9
        out[eng] = r
    out["stream_pass_ms"] = ops.sinkhorn_profile(a, a, C, 0.1, min(iters, 20), cost_scale=cmax)
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="c5,n16k,n4k")
    args = ap.parse_args()
    cases = args.cases.split(",")
    if "c5" in cases:
        case("config5", 8192, 1024, 200, torch.float16, ["sweep", "stream"])
    if "n4k" in cases:
        case("metric_N4096", 4096, 512, 100, torch.float32, ["sweep", "tiled", "stream"])
    if "n16k" in cases:
        case("hbm_N16384", 16384, 512, 20, torch.float32, ["sweep", "stream"])


if __name__ == "__main__":
    main()
