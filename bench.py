"""Benchmark of the Sinkhorn OT fusion hot path (BASELINE.json metric).

Workload (one "step" = one solve): seeded paired MRI/PET embeddings
X, Y in HBM (N = 4096, d = 512, float32) -> pairwise squared-Euclidean cost on MFMA
(max-normalised) -> 100 POT-semantics Sinkhorn iterations (eps = 0.1, stopThr = 0,
so every iteration runs) -> N x N transport plan written to HBM.

  value            = MRI+PET pairs aligned per second, whole job (N x ranks / step time)
  sinkhorn_iters_per_sec = iterations / time of the Sinkhorn call (incl. plan write)
  roofline         = dominant kernel (the resident Sinkhorn kernel: one launch runs
                     all iterations): algorithmic bytes iters * N*N*4 per launch / its
                     duration from HIP events on its stream; traffic = PMC HBM bytes
                     per launch from profiles/kernel_traffic.json (same kernel)
  cost_roofline    = the split-fp16 MFMA cost kernel: 2*N*N*d flops / event time
  hbm_probe        = streaming engine at N = 16384 (1 GiB cost, past the 256 MiB
                     Infinity Cache): true-HBM rate of one fused pass
  cpu_baseline     = the float64 C/OpenMP restatement (oracle/, POT semantics) on the
                     host cores, same workload, rank 0 at N = 1 only (+ 1-core run)

Multi-GPU: one process per GPU (torchrun); every rank solves its own independent
N = 4096 problem (per-rank minibatch) — "weak" scaling, no collective on the data
path; barrier + max-over-ranks timing as the driver requires.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd")
for _p in (PKG, REPO):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "MRI+PET pairs/sec + Sinkhorn iters/sec, N=4096 d=512 100 iters"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--n", type=int, default=4096)
    p.add_argument("--d", type=int, default=512)
    p.add_argument("--iters", type=int, default=100)
    p.add_argument("--eps", type=float, default=0.1)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-threads", type=int, default=0)
    p.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "kernel_traffic.json"))
    p.add_argument("--no-hbm-probe", action="store_true")
    p.add_argument("--hbm-probe-n", type=int, default=16384)
    p.add_argument("--profile-only", action="store_true",
                   help="run warmup + steps only (for rocprofv3 runs); no probes, no JSON")
    p.add_argument("--no-gw", action="store_true", help="skip the per-epoch GW latency leg")
    p.add_argument("--no-config5", action="store_true",
                   help="skip the N=8192 d=1024 fp16 200-iteration single-GPU leg")
    p.add_argument("--no-batch-ot", action="store_true",
                   help="skip the per-training-step OT block leg (config 2)")
    p.add_argument("--engine", default="auto", choices=("auto", "stream", "resident", "tiled"),
                   help="Sinkhorn engine (auto = resident when the cost fits the register file)")
    return p.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from otfuse import ops
    from otfuse.synthetic import paired_embeddings

    N, d, iters, eps = args.n, args.d, args.iters, args.eps
    X_np, Y_np, _ = paired_embeddings(N, d, seed=1234 + rank)
    X = torch.from_numpy(X_np).to(dev)
    Y = torch.from_numpy(Y_np).to(dev)
    a = torch.full((N,), 1.0 / N, device=dev)
    ws = ops.sinkhorn_workspace(N, N, torch.float32, iters, dev)
    P = torch.empty((N, N), dtype=torch.float32, device=dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    MFMA_F32_PEAK_TFLOPS = 157.3   # dense fp32 MFMA (MI355X_MICROARCH.md chip table)

    def step(record):
        if record:
            ev[0].record()
        C, cmax = ops.pairwise_cost(X, Y)
        if record:
            ev[1].record()
        ops.sinkhorn(a, a, C, eps, max_iter=iters, stop_thr=0.0, cost_scale=cmax, workspace=ws,
                     plan_out=P, engine=args.engine)
        if record:
            ev[2].record()
        return C, cmax

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if args.profile_only:
        if world > 1:
            dist.destroy_process_group()
        return

    # per-phase split of extra steps (events on the current stream = the kernels' stream)
    cost_l, sk_l = [], []
    for _ in range(5):
        step(True)
        torch.cuda.synchronize()
        cost_l.append(ev[0].elapsed_time(ev[1]))
        sk_l.append(ev[1].elapsed_time(ev[2]))
    cost_ms = sorted(cost_l)[2]
    sk_ms = sorted(sk_l)[2]
    C, cmax = ops.pairwise_cost(X, Y)
    res = ops.sinkhorn(a, a, C, eps, max_iter=iters, stop_thr=0.0, cost_scale=cmax, workspace=ws,
                       plan_out=P, engine=args.engine)
    engine = res.info()["engine_name"]

    # roofline of the dominant kernel.  Algorithmic bytes: one compulsory
    # read of the N x N fp32 cost per Sinkhorn iteration.  resident engine: ONE launch
    # does all iterations (+ the plan write) with the cost held in registers, so its
    # algorithmic rate can exceed the HBM peak — the PMC traffic shows the real bytes.
    iter_bytes = N * N * 4
    kernel_name = {"resident": "sk_resident_kernel", "tiled": "sk_tiled_kernel"}.get(engine, "sk_pass_kernel")

    def pmc_traffic(kname):
        try:
            tj = json.load(open(args.traffic_json))
        except (OSError, ValueError):
            return None
        if int(tj.get("n", 0)) != N or int(tj.get("iters", 0)) != iters:
            return None
        return tj.get("kernels", {}).get(kname, {}).get("hbm_bytes_per_launch")
    traffic = pmc_traffic(kernel_name)
    # streaming engine for reference: HIP event pair around every fused pass
    pass_ms = ops.sinkhorn_profile(a, a, C, eps, iters, cost_scale=cmax, workspace=ws)
    if engine in ("resident", "tiled"):
        launch_bytes = iter_bytes * iters
        achieved = launch_bytes / (sk_ms * 1e-3) / 1e9
    else:
        launch_bytes = iter_bytes
        achieved = iter_bytes / (pass_ms * 1e-3) / 1e9
    cost_flops = 2.0 * N * N * d
    cost_tflops = cost_flops / (cost_ms * 1e-3) / 1e12

    ms_per_step = elapsed * 1e3 / args.steps
    value = world * N * args.steps / elapsed
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic: seeded paired structured embeddings (SURVEY.md 8d), resident in HBM",
        "config": {"workload": f"sinkhorn_pairwise_N{N}_d{d}_it{iters}", "N": N, "d": d,
                   "iters": iters, "eps": eps, "cost": "sqeuclidean / max (split-fp16 MFMA, fp32-accurate)",
                   "sinkhorn": "POT sinkhorn_knopp semantics, stopThr=0",
                   "plan": "N x N float32 written per step", "global_batch": N * world,
                   "parallelism": f"replicas x{world} (independent problems)"},
        "sinkhorn_iters_per_sec": iters / (sk_ms * 1e-3),
        "engine": engine,
        "breakdown_ms": {"cost": cost_ms, "sinkhorn_incl_plan": sk_ms,
                         "stream_engine_pass_mean": pass_ms},
        "roofline": {"bound": "hbm", "kernel": kernel_name, "achieved": achieved,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                     "traffic": traffic, "algorithmic_bytes_per_launch": launch_bytes,
                     "note": ("resident: all iterations in one launch, cost held in registers; "
                              "algorithmic bytes = iters x N*N*4" if engine in ("resident", "tiled") else
                              "one launch per iteration; C (64 MiB) fits the 256 MiB Infinity Cache")},
        "cost_roofline": {"bound": "mfma", "kernel": "cost_split16_kernel", "achieved": cost_tflops,
                          "peak": MFMA_F32_PEAK_TFLOPS, "unit": "TFLOP/s",
                          "frac": cost_tflops / MFMA_F32_PEAK_TFLOPS,
                          "traffic": pmc_traffic("cost_split16_kernel"),
                          "note": "2*N*N*d fp32-equivalent flops (3 f16 MFMAs per product) incl. "
                                  "the split/prep kernel, vs the dense fp32 MFMA peak"},
        "stream_engine": {"pass_ms": pass_ms, "achieved": iter_bytes / (pass_ms * 1e-3) / 1e9,
                          "frac": iter_bytes / (pass_ms * 1e-3) / 1e9 / HBM_PEAK_GBS},
    }
    if not args.no_hbm_probe:
        out["hbm_probe"] = hbm_probe(ops, paired_embeddings, args.hbm_probe_n, d, eps, dev)
    if rank == 0 and not args.no_gw:
        out["gw_per_epoch"] = gw_leg(dev, world == 1 and not args.no_cpu_baseline)
    if rank == 0 and not args.no_config5:
        out["config5_single_gpu"] = config5_leg(dev)
    if rank == 0 and not args.no_batch_ot:
        out["batch_ot_per_step"] = batch_ot_leg(dev, world == 1 and not args.no_cpu_baseline)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(X_np, Y_np, N, iters, eps, args.cpu_threads)
        out["vs_cpu"] = value / out["cpu_baseline"]["value"]
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def batch_ot_leg(dev, with_cpu, B=8, d=512, eps=1e-2):
    """Config 2: the OT block of forward in every training
    step (MRI_PET_OT_nojax.py:679-725) -- feature cost with Ts = I/B, POT Sinkhorn in
    float64 to stopThr 1e-9 (<= 2000 iterations), NaN guard + row normalisation,
    pet_fused @ T^T, cosine loss -- forward AND backward through the plan apply, all
    on the device (the reference: D2H copy, POT on the host, H2D copy).  Latency-bound,
    reported as ms per step.  CPU: the oracle's float64 C restatement of the same
    forward (feature cost + sinkhorn_knopp + post-processing + apply), host cores."""
    import numpy as np
    from otfuse import fusion
    from otfuse.synthetic import paired_embeddings
    X, Y, _ = paired_embeddings(B, d, seed=321)
    mri = torch.from_numpy(X).to(dev).requires_grad_(True)
    pet = torch.from_numpy(Y).to(dev).requires_grad_(True)

    def step():
        loss, _, T = fusion.ot_alignment_loss(mri, pet, eps=eps)
        loss.backward()
        return loss

    step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(7):
        e0.record()
        loss = step()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    _, res = fusion.batch_feature_plan(mri, pet, eps)
    info = res.info()
    out = {"B": B, "d": d, "eps": eps, "unit": "ms per training step (OT block forward + backward)",
           "device_ms": sorted(ts)[3], "sinkhorn_iters": info["niter"],
           "status": info["status_name"], "engine": info["engine_name"], "loss": float(loss.detach())}
    if with_cpu:
        from oracle import oracle as orc
        t0 = time.perf_counter()
        for _ in range(3):
            M = orc.feature_cost(X, Y, np.eye(B) / B)
            u = np.full(d, 1.0 / d)
            P, *_ = orc.sinkhorn_knopp(u, u, M, eps, 2000, 1e-9)
            T = np.nan_to_num(P.astype(np.float32), nan=1e-8)
            rs = T.sum(1, keepdims=True)
            T = T / np.where(rs == 0, 1e-8, rs)
            Z = Y @ T.T
            cos = (X * Z).sum(1) / (np.linalg.norm(X, axis=1) * np.linalg.norm(Z, axis=1))
            _ = 1.0 - cos.mean()
        out["cpu_ms"] = (time.perf_counter() - t0) * 1e3 / 3
        out["cpu_note"] = ("oracle C/OpenMP restatement of the forward only (no backward), "
                           f"{os.environ.get('OMP_NUM_THREADS', 'default')} OpenMP threads")
    return out


def config5_leg(dev, N=8192, d=1024, iters=200, eps=0.1):
    """BASELINE config 5 on ONE GPU (the 8-GPU form is the row-sharded solve of
    otfuse.distributed): N = 8192, d = 1024, fp16 embeddings, fp16 cost storage (power-
    of-two scaled), fp32 accumulation, 200 iterations, stopThr = 0.  1024 row blocks do
    not fit the resident / tiled engines, so the streaming engine runs: one read of the
    128 MiB fp16 cost per iteration -> HBM-bound pass, reported against 8 TB/s."""
    import numpy as np
    from otfuse import ops
    from otfuse.synthetic import paired_embeddings
    X, Y, _ = paired_embeddings(N, d, seed=1234)
    Xd = torch.from_numpy(X.astype(np.float16)).to(dev)
    Yd = torch.from_numpy(Y.astype(np.float16)).to(dev)
    a = torch.full((N,), 1.0 / N, device=dev)
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    tc, ts = [], []
    res = None
    for _ in range(4):
        e[0].record()
        C, cmax, _ = ops.pairwise_cost_ex(Xd, Yd, out_dtype=torch.float16)
        e[1].record()
        res = ops.sinkhorn(a, a, C, eps, max_iter=iters, stop_thr=0.0, cost_scale=cmax)
        e[2].record()
        torch.cuda.synchronize()
        tc.append(e[0].elapsed_time(e[1]))
        ts.append(e[1].elapsed_time(e[2]))
        del C
    tc, ts = sorted(tc[1:])[1], sorted(ts[1:])[1]
    info = res.info()
    iter_bytes = N * N * 2
    gbs = iter_bytes * iters / (ts * 1e-3) / 1e9
    return {"N": N, "d": d, "iters": iters, "eps": eps, "dtype": "f16 storage, f32 accumulate",
            "engine": info["engine_name"], "status": info["status_name"],
            "cost_ms": tc, "sinkhorn_incl_plan_ms": ts, "pairs_per_s": N / ((tc + ts) * 1e-3),
            "sinkhorn_iters_per_s": iters / (ts * 1e-3),
            "cost_tflops": 2.0 * N * N * d / (tc * 1e-3) / 1e12,
            "sinkhorn_hbm": {"achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": gbs / HBM_PEAK_GBS,
                             "note": "N*N*2 B per iteration (one read of the fp16 cost) incl. "
                                     "the plan write; the cost (128 MiB) fits the 256 MiB MALL"}}


def gw_leg(dev, with_cpu, labels=2, per_label=64, d=512, eps=5e-3):
    """Per-epoch sample coupling: `labels` label groups of
    `per_label` paired samples (the reference's --max-jax-samples 64), d = 512.
    Device: the three GW solvers, all labels in one launch (float64 costs built on the
    device first, inside the timing); latency-bound, so reported as ms per epoch
    call.  CPU: the oracle's float64 C restatements, one core, same problems."""
    from otfuse import gw
    from otfuse.synthetic import paired_embeddings
    Xs, Ys = [], []
    for k in range(labels):
        X, Y, _ = paired_embeddings(per_label, d, seed=500 + k)
        Xs.append(torch.from_numpy(X).to(dev))
        Ys.append(torch.from_numpy(Y).to(dev))

    def run(solver):
        # POT callers use cdist / max (Euclidean), OTT PointCloud the squared distance
        euc = solver in (gw.GW_CG, gw.GW_PGD)
        metric = "euclidean" if euc else "sqeuclidean"
        C1s = [gw.pairwise_cost_f64(x, None, metric=metric, zero_diag=euc,
                                    scale_max=True)[0] for x in Xs]
        C2s = [gw.pairwise_cost_f64(y, None, metric=metric, zero_diag=euc,
                                    scale_max=True)[0] for y in Ys]
        if solver == gw.GW_CG:
            return gw.solve_batched(C1s, C2s, gw.GW_CG, max_iter=10000, log_len=1), C1s, C2s
        if solver == gw.GW_PGD:
            return gw.solve_batched(C1s, C2s, gw.GW_PGD, max_iter=1000, tol_abs=1e-9, eps=eps,
                                    sk_max_iter=1000, sk_inner=10, sk_threshold=1e-9,
                                    log_len=1), C1s, C2s
        return gw.solve_batched(C1s, C2s, gw.GW_ENTROPIC, max_iter=2000, eps=eps,
                                sk_max_iter=2000, log_len=1), C1s, C2s

    out = {"labels": labels, "samples_per_label": per_label, "d": d, "eps": eps,
           "unit": "ms per epoch call (all labels)"}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for name, solver in (("pot_cg", gw.GW_CG), ("ott_entropic", gw.GW_ENTROPIC),
                         ("pot_entropic_pgd", gw.GW_PGD)):
        run(solver)
        ts = []
        for _ in range(5):
            e0.record()
            res, C1s, C2s = run(solver)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        info = res.infos()
        out[name] = {"device_ms": sorted(ts)[2], "outer_iters": [i["n_iter"] for i in info],
                     "inner_iters": [i["inner_iters"] for i in info]}
        if with_cpu:
            from oracle import oracle as orc
            c1 = [c.cpu().numpy() for c in C1s]
            c2 = [c.cpu().numpy() for c in C2s]
            t0 = time.perf_counter()
            for a_, b_ in zip(c1, c2):
                if solver == gw.GW_CG:
                    orc.gw_cg(a_, b_)
                elif solver == gw.GW_PGD:
                    orc.gw_pgd(a_, b_, eps)
                else:
                    orc.gw_entropic(a_, b_, eps)
            cpu_ms = (time.perf_counter() - t0) * 1e3
            out[name]["cpu_ms"] = cpu_ms
            out[name]["cpu_note"] = "oracle C restatement, 1 core, solve only (costs given)"
    return out


def hbm_probe(ops, paired_embeddings, n, d, eps, dev):
    """Streaming engine on an n x n fp32 cost (1 GiB at n = 16384, 4x the Infinity
    Cache): mean HIP-event time of one fused pass -> true-HBM GB/s."""
    Xn, Yn, _ = paired_embeddings(n, d, seed=99)
    X = torch.from_numpy(Xn).to(dev)
    Y = torch.from_numpy(Yn).to(dev)
    C, cmax = ops.pairwise_cost(X, Y)
    del X, Y
    a = torch.full((n,), 1.0 / n, device=dev)
    ws = ops.sinkhorn_workspace(n, n, torch.float32, 10, dev)
    ms = ops.sinkhorn_profile(a, a, C, eps, 10, cost_scale=cmax, workspace=ws)
    gbs = n * n * 4 / (ms * 1e-3) / 1e9
    del C, ws
    torch.cuda.empty_cache()
    return {"kernel": "sk_pass_kernel", "N": n, "pass_ms": ms, "achieved": gbs,
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
            "note": "streaming engine, 10 passes, cost 4x the Infinity Cache"}


def cpu_baseline(X, Y, N, iters, eps, threads):
    """float64 POT-semantics restatement (oracle/otoracle.c, OpenMP) on the host cores:
    full workload once (cost build + iterations + plan), after a small warm-up."""
    from oracle import oracle as orc
    n_threads = threads or min(16, os.cpu_count() or 1)
    used = orc.set_threads(n_threads)
    a = np.full(N, 1.0 / N)
    orc.sinkhorn_knopp(a[:256], a[:256] * (N / 256), np.zeros((256, 256)), eps, 2, 0.0)
    runs = []
    for _ in range(3):
        t0 = time.perf_counter()
        C, _ = orc.pairwise_cost(X, Y, scale_max=True)
        t1 = time.perf_counter()
        orc.sinkhorn_knopp(a, a, C, eps, iters, 0.0, want_plan=True)
        t2 = time.perf_counter()
        runs.append((t2 - t0, t1 - t0, t2 - t1))
    tot, tc, tl = sorted(runs)[1]  # median run
    # one core: the same workload with 10 iterations, loop time scaled to `iters`
    orc.set_threads(1)
    t0 = time.perf_counter()
    C, _ = orc.pairwise_cost(X, Y, scale_max=True)
    t1 = time.perf_counter()
    orc.sinkhorn_knopp(a, a, C, eps, 10, 0.0, want_plan=True)
    t2 = time.perf_counter()
    orc.set_threads(n_threads)
    one = (t1 - t0) + (t2 - t1) * iters / 10.0
    return {"value": N / tot, "unit": "pairs/s", "cores": used, "kind": "port",
            "sinkhorn_iters_per_sec": iters / tl, "seconds": tot,
            "sample": f"full workload, median of 3: N={N} d={X.shape[1]} {iters} iters float64 "
                      f"(cost {tc:.2f}s + loop/plan {tl:.2f}s)",
            "single_core": {"value": N / one, "unit": "pairs/s", "cores": 1,
                            "sinkhorn_iters_per_sec": 10.0 / (t2 - t1),
                            "sample": f"cost {t1 - t0:.2f}s + 10 iters {t2 - t1:.2f}s, scaled to {iters}"}}


if __name__ == "__main__":
    main()
