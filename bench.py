"""Benchmark of the Sinkhorn OT fusion hot path (BASELINE.json metric).

Workload (one "step" = one solve): seeded paired MRI/PET embeddings
X, Y in HBM (N = 4096, d = 512, float32) -> pairwise squared-Euclidean cost in float64
(POT euclidean_distances order, divided by its max) -> 100 POT-semantics Sinkhorn
iterations in float64 (eps = 0.1, stopThr = 0, so every iteration runs) -> N x N float64
transport plan written to HBM.  float64 is the reference's own precision (POT on NumPy
float64, MRI_PET_OT_nojax.py:70-75, 121-143), so the headline is like-for-like with the
CPU path; parity: tests/test_gpu_pairwise.py, tests/test_gpu_precision.py (1e-9 of the
oracle).  The step is ONE solve launch (ops.sinkhorn_pairwise -> otf_sinkhorn_pairwise_f64):
the cost is built inside it, tile by tile, on the float64 matrix cores (--two-call: the
cost kernel, then the solve on the stored cost).

  value            = MRI+PET pairs aligned per second, whole job (N x ranks / step time)
  sinkhorn_iters_per_sec = iterations / time of the solve call (incl. the cost build and
                     the plan write for the fused step)
  roofline         = the dominant kernel, sk_mesh64_kernel (the fused launch: cost tiles on
                     v_mfma_f64_16x16x4_f64, then all 100 iterations with the float64
                     K = exp(-C/eps) held in the register files and LDS): the step's float64
                     FLOP (2 N^2 d for the cost + 4 N^2 per iteration) per second of the call
                     against the float64 peak (78.6 TFLOP/s, matrix and vector alike); the
                     per-iteration slope (latency-bound: three in-launch granule hops) and
                     the intercept beside it; the PMC traffic (profiles/kernel_traffic.json,
                     only when measured on this exact library build)
  cost_roofline    = the two-call path's float64 cost kernel vs the float64 matrix peak
  metric_f32       = the same workload at float32 compute (split-fp16 cost, float32 mesh):
                     faster, within 1e-4 of the float64 oracle, NOT the reference's precision
  sweep_config5    = BASELINE config 5 on one GPU (N = 8192, d = 1024, fp16 cost, 200
                     iterations): the sweep engine streams the 128 MiB cost from the
                     Infinity Cache once per iteration -> an HBM-class roofline
  hbm_probe        = the sweep engine on an N = 16384 fp32 cost (1 GiB, 4x the Infinity
                     Cache): true-HBM rate per iteration
  cpu_baseline     = the float64 C/OpenMP restatement (oracle/, POT semantics) on this
                     process's host CPU share, same workload, rank 0 at N = 1 only; also the
                     1-core run and the NumPy restatement (reference-equivalent: POT's NumPy
                     loop); vs_cpu = float64 GPU / float64 CPU

Multi-GPU: one process per GPU (torchrun); every rank solves its own independent
N = 4096 problem (per-rank minibatch) — "weak" scaling, no collective on the headline
path; barrier + max-over-ranks timing as the driver requires.  At world > 1 two more
legs time the north star's sharded path (config 5 as ONE row-sharded solve with the
column sums exchanged in-kernel over xGMI or by RCCL, and config 3's per-epoch chain).
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
HBM_PEAK_GBS = 8000.0         # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
MFMA_F16_PEAK_TFLOPS = 2500.0  # dense fp16 / bf16 MFMA (same table; 2:1 sparsity excluded)
VALU_F32_PEAK_TFMA = 78.6     # 157.3 TFLOP/s fp32 vector = 78.6 T FMA/s
F64_VALU_TFLOPS = 78.6        # float64 vector peak (39.3 T FMA/s)
LIB = os.path.join(PKG, "otfuse", "lib", "libotfuse.so")


def lib_md5():
    import hashlib
    try:
        return hashlib.md5(open(LIB, "rb").read()).hexdigest()
    except OSError:
        return None


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--n", type=int, default=4096)
    p.add_argument("--d", type=int, default=512)
    p.add_argument("--iters", type=int, default=100)
    p.add_argument("--eps", type=float, default=0.1)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-threads", type=int, default=0, help="0 = all host cores (nproc)")
    p.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "kernel_traffic.json"))
    p.add_argument("--no-hbm-probe", action="store_true")
    p.add_argument("--hbm-probe-n", type=int, default=16384)
    p.add_argument("--profile-only", action="store_true",
                   help="run warmup + steps only (for rocprofv3 runs); no probes, no JSON")
    p.add_argument("--profile-config5", action="store_true",
                   help="with --profile-only: run the config-5 sweep workload instead")
    p.add_argument("--profile-f32", action="store_true",
                   help="with --profile-only: run the float32 metric leg instead")
    p.add_argument("--no-gw", action="store_true", help="skip the per-epoch GW latency leg")
    p.add_argument("--no-f32", action="store_true",
                   help="skip the float32 (split-fp16 cost, float32 solve) leg of the metric config")
    p.add_argument("--no-config5", action="store_true",
                   help="skip the N=8192 d=1024 fp16 200-iteration single-GPU leg")
    p.add_argument("--no-batch-ot", action="store_true",
                   help="skip the per-training-step OT block leg (config 2)")
    p.add_argument("--multi-legs", action="store_true",
                   help="run the sharded RCCL legs also at world = 1 (they always run at world > 1)")
    p.add_argument("--two-call", action="store_true",
                   help="headline step as two calls (gw.pairwise_cost_f64 + ops.sinkhorn) instead of "
                        "the fused ops.sinkhorn_pairwise")
    p.add_argument("--engine", default="auto",
                   choices=("auto", "stream", "resident", "tiled", "sweep", "gather", "mesh"),
                   help="Sinkhorn engine (auto = mesh / tiled / resident when the cost fits the "
                        "register files)")
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

    from otfuse import gw, ops
    from otfuse.synthetic import paired_embeddings

    if args.profile_only and args.profile_config5:
        config5_leg(dev, reps=args.steps)
        return
    if args.profile_only and args.profile_f32:
        Xp, Yp, _ = paired_embeddings(args.n, args.d, seed=1234)
        metric_f32_leg(dev, torch.from_numpy(Xp).to(dev), torch.from_numpy(Yp).to(dev), args.n, args.d,
                       args.iters, args.eps, args.engine, None, steps=args.steps, warmup=args.warmup,
                       profile_only=True)
        return

    N, d, iters, eps = args.n, args.d, args.iters, args.eps
    X_np, Y_np, _ = paired_embeddings(N, d, seed=1234 + rank)
    X = torch.from_numpy(X_np).to(dev)
    Y = torch.from_numpy(Y_np).to(dev)
    # the headline step in the reference's own precision (POT runs NumPy float64,
    # MRI_PET_OT_nojax.py:121-143): float64 cost from the float32 embeddings, float64 POT
    # Sinkhorn, float64 plan
    a64 = torch.full((N,), 1.0 / N, device=dev, dtype=torch.float64)
    ws64 = ops.sinkhorn_workspace(N, N, torch.float64, iters, dev)
    wsp = ops.sinkhorn_pairwise_workspace(N, N, iters, dev)
    P64 = torch.empty((N, N), dtype=torch.float64, device=dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]

    def step_two_call(record, it=iters):
        if record:
            ev[0].record()
        # the max-normalisation (MRI_PET_OT_nojax.py:75) is applied inside the solve through
        # cost_scale (no separate C /= max pass)
        C, cmax = gw.pairwise_cost_f64(X, Y, scale_max=False)
        if record:
            ev[1].record()
        res = ops.sinkhorn(a64, a64, C, eps, max_iter=it, stop_thr=0.0, cost_scale=cmax,
                           workspace=ws64, plan_out=P64, engine=args.engine)
        if record:
            ev[2].record()
        return res

    def step_fused(record, it=iters):
        # MRI_PET_OT_nojax.py:70-75 + :143 as ONE solve launch: every workgroup builds its
        # tile of the float64 cost on the matrix cores, the grid agrees on max(C), then the
        # float64 mesh runs the 100 iterations on K held on chip (otf_sinkhorn_pairwise_f64)
        if record:
            ev[0].record()
            ev[1].record()
        res = ops.sinkhorn_pairwise(X, Y, eps, max_iter=it, stop_thr=0.0, workspace=wsp, plan_out=P64,
                                    engine=args.engine)
        if record:
            ev[2].record()
        return res

    step = step_two_call if args.two_call else step_fused

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

    # per-phase split of extra steps (events on the current stream = the kernels' stream),
    # the steps enqueued back to back as in the timed loop and synchronised once: a sync per
    # step would leave the GPU idle while the host enqueues the next call, and the events
    # would time the host's Python overhead instead of the device
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(6)]
    res = None
    for k in range(6):
        ev[:] = evs[k]
        res = step(True)
    torch.cuda.synchronize()
    cost_ms = sorted(e[0].elapsed_time(e[1]) for e in evs[1:])[2]
    sk_ms = sorted(e[1].elapsed_time(e[2]) for e in evs[1:])[2]
    info = res.info()
    # the solve launch split by iteration count: the same step at iters / 5 iterations, the
    # per-iteration slope and the intercept (registration, the in-launch cost build for the
    # fused step, K = exp, the plan write, the small launches)
    it_lo = max(1, iters // 5)
    evl = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(6)]
    for k in range(6):
        ev[:] = evl[k]
        step(True, it_lo)
    torch.cuda.synchronize()
    sk_lo_ms = sorted(e[1].elapsed_time(e[2]) for e in evl[1:])[2]
    slope_us = (sk_ms - sk_lo_ms) * 1e3 / (iters - it_lo)
    intercept_us = sk_ms * 1e3 - iters * slope_us
    two_call_ms = None
    if not args.two_call:
        # the same step as two calls (cost kernel, then the solve on the stored cost)
        evt = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(6)]
        for k in range(6):
            ev[:] = evt[k]
            step_two_call(True)
        torch.cuda.synchronize()
        two_call_ms = sorted(e[0].elapsed_time(e[2]) for e in evt[1:])[2]
        cost_ms = sorted(e[0].elapsed_time(e[1]) for e in evt[1:])[2]
    engine = info["engine_name"]
    kernel_name = {"mesh": "sk_mesh64_kernel", "sweep": "sk_sweep_kernel", "tiled": "sk_tiled_kernel",
                   "resident": "sk_resident_kernel"}.get(engine, "sk_pass_kernel")

    # PMC traffic: only when profiles/kernel_traffic.json was measured on THIS library
    # build and shape (a stale profile is reported as null, not reused)
    try:
        tj = json.load(open(args.traffic_json))
    except (OSError, ValueError):
        tj = {}
    fresh = (tj.get("lib_md5") == lib_md5() and int(tj.get("n", 0)) == N
             and int(tj.get("iters", 0)) == iters)

    def pmc_traffic(kname):
        if not fresh:
            return None
        return tj.get("kernels", {}).get(kname, {}).get("hbm_bytes_per_launch")

    iter_bytes = N * N * 8
    traffic = pmc_traffic(kernel_name)
    sk_s = sk_ms * 1e-3
    us_per_iter = sk_ms * 1e3 / iters
    # VALU floor of one iteration: 2 N^2 float64 FMAs (row sums K v, column sums K^T u) at
    # the float64 vector peak (78.6 TFLOP/s = 39.3 T FMA/s)
    floor_us = 2.0 * N * N / (F64_VALU_TFLOPS / 2 * 1e12) * 1e6
    algo_gbs = iter_bytes * iters / sk_s / 1e9
    cost_flops = 2.0 * N * N * d
    iter_flops = 4.0 * N * N  # K v and K^T u: 2 N^2 FMAs
    if not args.two_call and engine == "mesh":
        # the fused launch does all the step's arithmetic: the cost on the float64 matrix
        # cores, then the iterations on the float64 vector units -- both at 78.6 TFLOP/s
        flops = cost_flops + iters * iter_flops
        tf = flops / sk_s / 1e12
        roofline = {"bound": "mfma", "kernel": kernel_name, "achieved": tf, "peak": F64_VALU_TFLOPS,
                    "unit": "TFLOP/s", "frac": tf / F64_VALU_TFLOPS, "traffic": traffic,
                    "flops_per_launch": flops, "launch_us": sk_ms * 1e3,
                    "floor_us": flops / (F64_VALU_TFLOPS * 1e12) * 1e6,
                    "per_iteration_us": slope_us, "per_iteration_floor_us": floor_us,
                    "intercept_us": intercept_us,
                    "note": ("ONE launch per step (otf_sinkhorn_pairwise_f64, csrc/otf_mesh64.hip PW): "
                             "every workgroup builds its 128 x 512 tile of the float64 cost on "
                             "v_mfma_f64_16x16x4_f64, the grid agrees on max(C), K = exp(-C/(eps max)) "
                             "stays on chip (register files + LDS) for the 100 iterations (three "
                             "in-launch granule hops each), then the N x N float64 plan; achieved = "
                             "(2 N^2 d + iters 4 N^2) FLOP / the call's device time (incl. the norm and "
                             "init launches); per_iteration_us / intercept_us: slope and intercept of "
                             "the call's time at iters and iters / 5 iterations")}
    elif engine in ("mesh", "tiled", "resident"):
        roofline = {"bound": "latency", "kernel": kernel_name, "achieved": us_per_iter,
                    "peak": floor_us, "unit": "us per iteration", "frac": floor_us / us_per_iter,
                    "traffic": traffic,
                    "traffic_GBs": (traffic / sk_s / 1e9) if traffic else None,
                    "algorithmic_bytes_per_launch": iter_bytes * iters,
                    "algorithmic_GBs": algo_gbs,
                    "note": ("float64 K = exp(-C/eps) held on chip (register files + LDS) for the "
                             "whole solve, C read once: per iteration three in-launch granule hops "
                             "(row partials within the row block, column partials to the reducers, "
                             "sums back; csrc/otf_mesh64.hip) against a VALU floor (peak) of 2 N^2 "
                             "float64 FMAs at 39.3 T FMA/s; achieved = the Sinkhorn call's device "
                             "time / iterations (incl. prologue and the N x N float64 plan write); "
                             "the HBM-bound engine is measured in sweep_config5 / hbm_probe")}
    else:
        roofline = {"bound": "hbm", "kernel": kernel_name, "achieved": algo_gbs,
                    "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": algo_gbs / HBM_PEAK_GBS,
                    "traffic": traffic, "algorithmic_bytes_per_launch": iter_bytes * iters,
                    "note": "N*N*8 B per sweep"}
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
        "dtype": "f64",
        "data": "synthetic: seeded paired structured embeddings (SURVEY.md 8d), resident in HBM",
        "config": {"workload": f"sinkhorn_pairwise_N{N}_d{d}_it{iters}", "N": N, "d": d,
                   "iters": iters, "eps": eps,
                   "cost": "sqeuclidean float64 from the float32 embeddings (POT euclidean_distances "
                           "order), max applied in the solve" + ("" if args.two_call else
                                                                 ", built inside the solve launch"),
                   "sinkhorn": "POT sinkhorn_knopp semantics in float64, stopThr=0",
                   "plan": "N x N float64 written per step", "global_batch": N * world,
                   "parallelism": f"replicas x{world} (independent problems)"},
        "sinkhorn_iters_per_sec": iters / sk_s,
        "engine": engine,
        "status": info["status_name"],
        "breakdown_ms": ({"cost": cost_ms, "sinkhorn_incl_plan": sk_ms} if args.two_call else
                         {"fused_call": sk_ms, "per_iteration": slope_us * 1e-3,
                          "intercept": intercept_us * 1e-3, "two_call_step": two_call_ms,
                          "two_call_cost": cost_ms}),
        "roofline": roofline,
        "cost_roofline": {"bound": "mfma", "kernel": "dist_mfma_f64_kernel",
                          "achieved": cost_tflops, "peak": F64_VALU_TFLOPS, "unit": "TFLOP/s",
                          "frac": cost_tflops / F64_VALU_TFLOPS, "op_us": cost_ms * 1e3,
                          "traffic": pmc_traffic("dist_mfma_f64_kernel"),
                          "note": ("the two-call path's cost (gw.pairwise_cost_f64: norm kernels, the "
                                   "128 x 128 tile kernel on v_mfma_f64_16x16x4_f64, max) against the "
                                   "float64 matrix peak (78.6 TFLOP/s); the headline step builds the "
                                   "cost inside its solve launch instead" if not args.two_call else
                                   "2 N^2 d float64 FLOP on v_mfma_f64_16x16x4_f64 over the whole "
                                   "host call (norm kernels, tile kernel, max) against the float64 "
                                   "matrix peak (78.6 TFLOP/s)")},
        "traffic_profile": {"fresh": fresh, "round": tj.get("round"), "lib_md5": lib_md5()},
    }
    del ws64, wsp, P64
    if rank == 0 and not args.no_f32:
        out["metric_f32"] = metric_f32_leg(dev, X, Y, N, d, iters, eps, args.engine, pmc_traffic)
    if not args.no_hbm_probe:
        out["hbm_probe"] = hbm_probe(ops, paired_embeddings, args.hbm_probe_n, d, eps, dev)
    if rank == 0 and not args.no_gw:
        out["gw_per_epoch"] = gw_leg(dev, world == 1 and not args.no_cpu_baseline)
    if rank == 0 and not args.no_config5:
        out["sweep_config5"] = config5_leg(dev)
    if rank == 0 and not args.no_batch_ot:
        out["batch_ot_per_step"] = batch_ot_leg(dev, world == 1 and not args.no_cpu_baseline)
    if world > 1 or args.multi_legs:
        # the sharded legs are extra evidence beside the headline: a failure that every
        # rank hits alike (same exception on every rank, so the collectives stay in step)
        # is recorded instead of costing the run its JSON line
        for key, leg in (("sharded_config5", sharded_config5_leg), ("config3_epoch_chain", config3_leg)):
            try:
                out[key] = leg(dev, world)
            except Exception as e:  # noqa: BLE001
                out[key] = {"error": f"{type(e).__name__}: {e}"[:300]}
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


def config5_leg(dev, N=8192, d=1024, iters=200, eps=0.1, reps=4):
    """BASELINE config 5 on ONE GPU (the multi-GPU form is sharded_config5_leg): N = 8192,
    d = 1024, fp16 embeddings, fp16 cost storage (power-of-two scaled), fp32 arithmetic,
    200 iterations, stopThr = 0.  The cost does not fit the register files, so the sweep
    engine runs: ONE persistent launch that streams the 128 MiB cost once per iteration
    (iters + 1 sweeps incl. the prologue K^T u0).  Its roofline is HBM-class: per sweep
    N*N*2 bytes are really read (from the Infinity Cache, which holds the 128 MiB cost).
    Reported: per-sweep time from a solve without the plan, the same with the plan, and
    the cost kernel on fp16 MFMA."""
    import numpy as np
    from otfuse import ops
    from otfuse.synthetic import paired_embeddings
    X, Y, _ = paired_embeddings(N, d, seed=1234)
    Xd = torch.from_numpy(X.astype(np.float16)).to(dev)
    Yd = torch.from_numpy(Y.astype(np.float16)).to(dev)
    a = torch.full((N,), 1.0 / N, device=dev)
    ws = ops.sinkhorn_workspace(N, N, torch.float32, iters, dev)
    P = torch.empty((N, N), dtype=torch.float32, device=dev)
    e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    tc, ts, tn = [], [], []
    res = None
    for _ in range(reps):
        e[0].record()
        C, cmax, _ = ops.pairwise_cost_ex(Xd, Yd, out_dtype=torch.float16)
        e[1].record()
        res = ops.sinkhorn(a, a, C, eps, max_iter=iters, stop_thr=0.0, cost_scale=cmax, workspace=ws,
                           plan_out=P)
        e[2].record()
        ops.sinkhorn(a, a, C, eps, max_iter=iters, stop_thr=0.0, cost_scale=cmax, workspace=ws,
                     want_plan=False)
        e[3].record()
        torch.cuda.synchronize()
        tc.append(e[0].elapsed_time(e[1]))
        ts.append(e[1].elapsed_time(e[2]))
        tn.append(e[2].elapsed_time(e[3]))
        del C
    k = len(tc) // 2
    tc, ts, tn = sorted(tc)[k], sorted(ts)[k], sorted(tn)[k]
    info = res.info()
    sweep_us = tn * 1e3 / (iters + 1)
    iter_bytes = N * N * 2
    gbs = iter_bytes / (sweep_us * 1e-6) / 1e9
    return {"N": N, "d": d, "iters": iters, "eps": eps, "dtype": "f16 storage, f32 arithmetic",
            "engine": info["engine_name"], "status": info["status_name"],
            "cost_ms": tc, "sinkhorn_incl_plan_ms": ts, "sinkhorn_no_plan_ms": tn,
            "us_per_sweep": sweep_us,
            "pairs_per_s": N / ((tc + ts) * 1e-3),
            "sinkhorn_iters_per_s": iters / (ts * 1e-3),
            "cost_roofline": {"bound": "mfma", "achieved": 2.0 * N * N * d / (tc * 1e-3) / 1e12,
                              "peak": MFMA_F16_PEAK_TFLOPS, "unit": "TFLOP/s",
                              "frac": 2.0 * N * N * d / (tc * 1e-3) / 1e12 / MFMA_F16_PEAK_TFLOPS},
            "roofline": {"bound": "hbm", "kernel": "sk_sweep_kernel", "achieved": gbs,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
                         "note": "N*N*2 B read per sweep (the fp16 cost, streamed every iteration "
                                 "from the Infinity Cache); per-sweep time = solve without the "
                                 "plan / (iters + 1); the plan write is timed separately"}}


def metric_f32_leg(dev, X, Y, N, d, iters, eps, engine, pmc_traffic, steps=20, warmup=3,
                   profile_only=False):
    """The metric config at float32 compute (not the reference's precision; reported beside
    the float64 headline): split-fp16 cost on fp16 MFMA (fp32-accurate: x.y = hi.hi + hi.lo
    + lo.hi), float32 POT Sinkhorn on the float32 mesh (csrc/otf_mesh.hip), float32 plan.
    The step is the two calls (pairwise_cost + sinkhorn); the r06 fused form
    (ops.sinkhorn_pairwise(precision="fp32", engine="mesh"), otf_sinkhorn_pairwise_f32: every
    workgroup builds its cost tile in the solve's prologue from the split-fp16 images, bitwise
    the two calls' results, tests/test_gpu_pairwise32.py) is timed beside it -- measured slower,
    so AUTO keeps the two calls.  Parity: within 1e-4 of the float64 oracle at eps 0.1 ... 5e-3
    (tests/test_gpu_precision.py, tests/test_gpu_pairwise32.py)."""
    from otfuse import ops
    a = torch.full((N,), 1.0 / N, device=dev)
    ws = ops.sinkhorn_workspace(N, N, torch.float32, iters, dev)
    ws32 = ops.sinkhorn_pairwise_workspace(N, N, iters, dev, d=d, precision="fp32")
    P = torch.empty((N, N), dtype=torch.float32, device=dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]

    def fused(it=iters):
        return ops.sinkhorn_pairwise(X, Y, eps, max_iter=it, stop_thr=0.0, workspace=ws32, plan_out=P,
                                     engine="mesh", precision="fp32")

    def two_call(record):
        if record:
            ev[0].record()
        C, cmax = ops.pairwise_cost(X, Y)
        if record:
            ev[1].record()
        r = ops.sinkhorn(a, a, C, eps, max_iter=iters, stop_thr=0.0, cost_scale=cmax, workspace=ws,
                         plan_out=P, engine=engine)
        if record:
            ev[2].record()
        return r

    for _ in range(warmup):
        two_call(False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        two_call(False)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if profile_only:
        return None

    def call_ms(fn, reps=7):
        ts = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        return sorted(ts)[reps // 2]

    fused_ms = call_ms(fused)
    short = max(iters // 5, 1)
    # the step's solve at iters and iters / 5 on one cost: slope and intercept of the mesh launch
    C0, cm0 = ops.pairwise_cost(X, Y)
    solve = lambda it: ops.sinkhorn(a, a, C0, eps, max_iter=it, stop_thr=0.0, cost_scale=cm0, workspace=ws,
                                    plan_out=P, engine=engine)
    sk_long_ms = call_ms(lambda: solve(iters))
    sk_short_ms = call_ms(lambda: solve(short))
    per_it_ms = (sk_long_ms - sk_short_ms) / (iters - short)
    intercept_ms = sk_long_ms - per_it_ms * iters
    del C0
    rf = fused()
    for _ in range(2):
        two_call(False)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(6)]
    res = None
    for k in range(6):
        ev[:] = evs[k]
        res = two_call(True)
    torch.cuda.synchronize()
    cost_ms = sorted(e[0].elapsed_time(e[1]) for e in evs[1:])[2]
    sk_ms = sorted(e[1].elapsed_time(e[2]) for e in evs[1:])[2]
    # the two-call cost op split into its prep (norms / scales) and the MFMA kernel (device
    # events recorded by the library around each, OTF_COST_PHASES)
    os.environ["OTF_COST_PHASES"] = "1"
    ph = []
    for _ in range(5):
        ops.pairwise_cost(X, Y)
        ph.append(ops.cost_last_phases())
    os.environ.pop("OTF_COST_PHASES", None)
    prep_ms = sorted(p for p, _ in ph)[2]
    kern_ms = sorted(k for _, k in ph)[2]
    info = res.info()
    eng = info["engine_name"]
    # the 256 x 256 cost kernel the library ran (OTF_COST_8PH=0: the register-staged one)
    cname = "cost_big16_kernel" if os.environ.get("OTF_COST_8PH") == "0" else "cost_8ph_kernel"
    kname = {"mesh": "sk_mesh_kernel", "tiled": "sk_tiled_kernel", "sweep": "sk_sweep_kernel",
             "resident": "sk_resident_kernel", "gather": "sk_gather_kernel"}.get(eng, "sk_pass_kernel")
    floor_us = 2.0 * N * N / (VALU_F32_PEAK_TFMA * 1e12) * 1e6
    it_us = per_it_ms * 1e3
    traffic = pmc_traffic(kname) if pmc_traffic else None
    cost_flops = 2.0 * N * N * d
    ms_per_step = elapsed * 1e3 / steps
    return {"dtype": "f32", "N": N, "d": d, "iters": iters, "eps": eps, "engine": eng,
            "status": info["status_name"], "ms_per_step": ms_per_step,
            "pairs_per_s": N / (ms_per_step * 1e-3), "sinkhorn_iters_per_s": iters / (sk_ms * 1e-3),
            "step": "two calls: pairwise_cost (split-fp16 prep + %s) + sinkhorn (float32 mesh)" % cname,
            "breakdown_ms": {"cost": cost_ms, "sinkhorn_incl_plan": sk_ms,
                             "fused_call": fused_ms, "fused_engine": rf.info()["engine_name"],
                             "fused_fallback": rf.info()["fallback"], "sinkhorn_per_iteration": per_it_ms,
                             "sinkhorn_intercept": intercept_ms},
            "roofline": {"bound": "latency", "kernel": kname, "achieved": it_us, "peak": floor_us,
                         "unit": "us per iteration", "frac": floor_us / it_us, "traffic": traffic,
                         "note": "K in registers for the whole solve; the solve's per-iteration slope "
                                 "(between iters / 5 and iters) against the VALU floor of 2 N^2 float32 "
                                 "FMAs at 78.6 T FMA/s"},
            "cost_roofline": {"bound": "mfma", "kernel": cname,
                              "achieved": 3.0 * cost_flops / (kern_ms * 1e-3) / 1e12,
                              "peak": MFMA_F16_PEAK_TFLOPS, "unit": "TFLOP/s",
                              "frac": 3.0 * cost_flops / (kern_ms * 1e-3) / 1e12 / MFMA_F16_PEAK_TFLOPS,
                              "kernel_us": kern_ms * 1e3, "prep_us": prep_ms * 1e3,
                              "op_us": cost_ms * 1e3, "traffic": pmc_traffic(cname) if pmc_traffic else None,
                              "note": "the fp32-accurate product x.y = hi.hi + hi.lo + lo.hi runs as "
                                      "three fp16 MFMA contractions: achieved = 3 x 2*N*N*d / the MFMA "
                                      "kernel's device time vs the dense fp16 MFMA peak"},
            "note": "float32 compute: within 1e-4 of the float64 oracle (tests/test_gpu_precision.py, "
                    "tests/test_gpu_pairwise32.py), not the reference's precision -- the headline is the "
                    "float64 step"}


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


def hbm_probe(ops, paired_embeddings, n, d, eps, dev, iters=10):
    """Sweep engine on an n x n fp32 cost (1 GiB at n = 16384, 4x the Infinity Cache):
    per-sweep time of a solve without the plan -> true-HBM GB/s (nt loads)."""
    Xn, Yn, _ = paired_embeddings(n, d, seed=99)
    X = torch.from_numpy(Xn).to(dev)
    Y = torch.from_numpy(Yn).to(dev)
    C, cmax = ops.pairwise_cost(X, Y)
    del X, Y
    a = torch.full((n,), 1.0 / n, device=dev)
    ws = ops.sinkhorn_workspace(n, n, torch.float32, iters, dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    res = None
    for _ in range(3):
        e0.record()
        res = ops.sinkhorn(a, a, C, eps, max_iter=iters, stop_thr=0.0, cost_scale=cmax, workspace=ws,
                           want_plan=False)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ms = sorted(ts)[1]
    us = ms * 1e3 / (iters + 1)
    gbs = n * n * 4 / (us * 1e-6) / 1e9
    engine = res.info()["engine_name"]
    del C, ws
    torch.cuda.empty_cache()
    return {"kernel": "sk_sweep_kernel" if engine == "sweep" else "sk_pass_kernel", "engine": engine,
            "N": n, "us_per_sweep": us, "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": gbs / HBM_PEAK_GBS,
            "note": f"{iters} iterations + prologue in one launch, no plan; cost 4x the Infinity Cache"}


def _cpu_port_run(orc, X, Y, N, iters, eps, threads, reps=3):
    """float64 POT-semantics C/OpenMP restatement: full workload (cost + iterations +
    plan), median of `reps` after a small warm-up."""
    import numpy as np
    used = orc.set_threads(threads)
    a = np.full(N, 1.0 / N)
    orc.sinkhorn_knopp(a[:256], a[:256] * (N / 256), np.zeros((256, 256)), eps, 2, 0.0)
    runs = []
    for _ in range(reps):
        t0 = time.perf_counter()
        C, _ = orc.pairwise_cost(X, Y, scale_max=True)
        t1 = time.perf_counter()
        orc.sinkhorn_knopp(a, a, C, eps, iters, 0.0, want_plan=True)
        t2 = time.perf_counter()
        runs.append((t2 - t0, t1 - t0, t2 - t1))
    tot, tc, tl = sorted(runs)[len(runs) // 2]
    return used, tot, tc, tl


def cpu_baseline(X, Y, N, iters, eps, threads):
    """The CPU path on the GPU box's host: the float64 C/OpenMP
    restatement of POT sinkhorn_knopp (oracle/otoracle.c) on ALL host cores (nproc),
    the full workload; the headline value is the fastest of the all-core run and the run
    at this process's CPU share (OMP_NUM_THREADS / affinity, set by the box), so the GPU
    is compared against the CPU's best.  Also: 1 core (10 iterations, scaled) and the
    NumPy restatement (POT's own NumPy loop, reference-equivalent, BLAS threads = cores,
    10 iterations scaled)."""
    import numpy as np
    from oracle import oracle as orc
    nproc = os.cpu_count() or 1
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = nproc
    share = int(os.environ.get("OMP_NUM_THREADS") or 0) or affinity
    all_threads = threads or nproc
    runs = {}
    # the share first (the box pins OMP_NUM_THREADS to this process's CPU share); all
    # host cores (nproc) next -- oversubscribed when the share is smaller, so that run
    # times 10 iterations and scales the loop to `iters` to stay within the bench budget
    used, tot, tc, tl = _cpu_port_run(orc, X, Y, N, iters, eps, share)
    runs["cpu_share"] = {"threads": used, "seconds": tot, "cost_s": tc, "loop_plan_s": tl}
    # the box grants this process `share` CPUs (OMP_NUM_THREADS) of the host's nproc: an
    # all-core run is oversubscribed there (r03: 33 s on 256 threads against 0.52 s on 16),
    # so it runs only when asked for (--cpu-threads) or when the share is the whole host
    if all_threads != share and (threads or share >= nproc):
        used, tot, tc, tl = _cpu_port_run(orc, X, Y, N, 10, eps, all_threads, reps=1)
        tl *= iters / 10.0
        runs["all_cores"] = {"threads": used, "seconds": tc + tl, "cost_s": tc, "loop_plan_s": tl,
                             "note": "10 iterations, loop scaled to %d" % iters}
    best_key = min(runs, key=lambda k: runs[k]["seconds"])
    best = runs[best_key]
    # one core: the same workload with 10 iterations, loop time scaled to `iters`
    orc.set_threads(1)
    a = np.full(N, 1.0 / N)
    t0 = time.perf_counter()
    C, _ = orc.pairwise_cost(X, Y, scale_max=True)
    t1 = time.perf_counter()
    orc.sinkhorn_knopp(a, a, C, eps, 10, 0.0, want_plan=True)
    t2 = time.perf_counter()
    one = (t1 - t0) + (t2 - t1) * iters / 10.0
    one_cost, one_loop = t1 - t0, t2 - t1
    # NumPy restatement (POT's loop: K = exp(-M/reg), Kp, K^T u, Kp v), BLAS on all cores
    npy = None
    try:
        from threadpoolctl import threadpool_limits
        with threadpool_limits(limits=best["threads"]):
            t0 = time.perf_counter()
            Cn = orc.pairwise_cost_np(X, Y)
            Cn /= Cn.max()
            t1 = time.perf_counter()
            orc.sinkhorn_knopp_np(a, a, Cn, eps, 10, 0.0)
            t2 = time.perf_counter()
        npy_s = (t1 - t0) + (t2 - t1) * iters / 10.0
        npy = {"value": N / npy_s, "unit": "pairs/s", "cores": best["threads"],
               "sinkhorn_iters_per_sec": 10.0 / (t2 - t1),
               "sample": f"NumPy float64 (oracle.pairwise_cost_np + sinkhorn_knopp_np, the POT "
                         f"sinkhorn_knopp loop): cost {t1 - t0:.2f}s + 10 iterations incl. plan "
                         f"{t2 - t1:.2f}s, scaled to {iters}"}
        del Cn
    except Exception as e:  # noqa: BLE001 - a missing threadpoolctl only drops this line
        npy = {"error": repr(e)}
    orc.set_threads(best["threads"])
    return {"value": N / best["seconds"], "unit": "pairs/s", "cores": best["threads"], "kind": "port",
            "nproc": nproc, "affinity_cpus": affinity, "omp_share": share, "chosen": best_key,
            "host_cpu_quota": {"granted_cpus": share, "nproc": nproc,
                               "note": f"the GPU box grants this process {share} of the host's "
                                       f"{nproc} CPUs (OMP_NUM_THREADS); the baseline runs on "
                                       f"that share"},
            "sinkhorn_iters_per_sec": iters / best["loop_plan_s"], "seconds": best["seconds"],
            "sample": f"full workload, median of 3: N={N} d={X.shape[1]} {iters} iters float64 "
                      f"(cost {best['cost_s']:.2f}s + loop/plan {best['loop_plan_s']:.2f}s) with "
                      f"{best['threads']} threads; the fastest of {sorted(runs)}",
            "runs": runs,
            "single_core": {"value": N / one, "unit": "pairs/s", "cores": 1,
                            "sinkhorn_iters_per_sec": 10.0 / one_loop,
                            "sample": f"cost {one_cost:.2f}s + 10 iters {one_loop:.2f}s, scaled to {iters}"},
            "numpy_reference_equivalent": npy}


def sharded_config5_leg(dev, world, N=8192, d=1024, iters=200, eps=0.1):
    """The north star's sharded path for BASELINE config 5: ONE N = 8192 problem over the
    ranks.  Rank r holds N / world MRI rows; the PET shards are all-gathered (RCCL), the
    rank builds its fp16 cost rows, the global max is agreed (all-reduce MAX), then the
    solve runs as ONE persistent launch per rank whose column sums are exchanged inside
    the launch through the peers' exchange buffers over xGMI (otf_sinkhorn_xsweep): the
    "xmesh" leg keeps the rank's slab of K in the register files (from 4 ranks on), the
    "xsweep" leg streams it.  For comparison the previous form: the row-sharded solve with one RCCL
    all-reduce(SUM) of m + 1 sums per iteration (otf_sinkhorn_row_sharded, "rccl").
    Reported per solve and per iteration, max over ranks.  Scaling 'strong'."""
    import numpy as np
    from otfuse.comm import Communicator
    from otfuse.distributed import XPeer, coupled_solve_sharded
    from otfuse.synthetic import paired_embeddings
    out = {"N": N, "d": d, "iters": iters, "eps": eps, "ranks": world, "scaling": "strong"}
    try:
        rank = dist.get_rank() if world > 1 else 0
        comm = Communicator(device=dev)
        X, Y, _ = paired_embeddings(N, d, seed=1234)
        rows = N // world
        Xl = torch.from_numpy(X[rank * rows:(rank + 1) * rows].astype(np.float16)).to(dev)
        Yl = torch.from_numpy(Y[rank * rows:(rank + 1) * rows].astype(np.float16)).to(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

        def timed(**kw):
            ts, res = [], None
            for _ in range(3):
                if world > 1:
                    dist.barrier()
                torch.cuda.synchronize()
                e0.record()
                res, _ = coupled_solve_sharded(Xl, Yl, eps, max_iter=iters, want_plan=False, comm=comm, **kw)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            t = torch.tensor([sorted(ts)[1]], dtype=torch.float64, device=dev)
            if world > 1:
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
            return float(t[0]), res

        legs = {}
        # the in-kernel cross-rank engines on the peers' exchange buffers: "xmesh" (this
        # rank's slab of K in the register files, where it fits: 8192 / world x 8192 needs
        # world >= 4) and "xsweep" (the slab streamed every iteration)
        for leg, eng in (("xmesh", "mesh"), ("xsweep", "sweep")):
            try:
                xp = XPeer(N)
                ms, res = timed(xpeer=xp, engine=eng)
                legs[leg] = {"status": res.info()["status_name"], "engine": res.info()["engine_name"],
                             "ms_per_solve": ms, "us_per_iteration": ms * 1e3 / (iters + 1)}
                xp.close()
            except Exception as e:  # noqa: BLE001 - the other forms still report
                legs[leg] = {"error": repr(e)[:300]}
        ms, res = timed()
        legs["rccl"] = {"status": res.info()["status_name"], "ms_per_solve": ms,
                        "us_per_iteration": ms * 1e3 / (iters + 1)}
        best = min((k for k in legs if "ms_per_solve" in legs[k]), key=lambda k: legs[k]["ms_per_solve"])
        ms = legs[best]["ms_per_solve"]
        out.update({"engine": best, "status": legs[best]["status"], "ms_per_solve": ms,
                    "us_per_iteration": ms * 1e3 / (iters + 1), "legs": legs,
                    "pairs_per_s": N / (ms * 1e-3), "sinkhorn_iters_per_s": iters / (ms * 1e-3),
                    "note": "max over ranks; includes the all-gather, the cost rows and the max "
                            "all-reduce; per iteration each rank sweeps N/world x N fp16 cost rows"})
        comm.close()
    except Exception as e:  # noqa: BLE001 - report, never take the headline bench down
        out["error"] = repr(e)
    return out


def config3_leg(dev, world, B=32, d=2048, labels=2, per_label=64, eps=5e-3):
    """BASELINE config 3's per-epoch chain (MRI_PET_OT_OT_per_epoch_attn.py:940-960) over
    the ranks: every rank extracts B backbone features per minibatch (synthetic here),
    one RCCL all-gather gives every rank the whole set (B x world rows of d = 2048, MRI
    and PET) and labels; the per-label entropic GW on <= 64 samples
    (get_coupling_egw_ott_fixed) is split over the ranks by label, and get_coupling_fot on
    the 2048 x 2048 float64 feature cost at eps = 5e-3 runs on every rank.  Reported per
    epoch call."""
    import numpy as np
    from otfuse.comm import Communicator
    from otfuse.synthetic import paired_embeddings
    out = {"B_per_rank": B, "d": d, "labels": labels, "samples_per_label": per_label, "eps": eps,
           "ranks": world}
    try:
        from otfuse import perturbot
        rank = dist.get_rank() if world > 1 else 0
        comm = Communicator(device=dev)
        X, Y, lab = paired_embeddings(B, d, seed=700 + rank)
        Xl = torch.from_numpy(X).to(dev)
        Yl = torch.from_numpy(Y).to(dev)
        Ll = torch.from_numpy(lab.astype(np.float32)).to(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ts, tg = [], []
        for _ in range(3):
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e0.record()
            Xa, Ya, La = comm.all_gather(Xl), comm.all_gather(Yl), comm.all_gather(Ll)
            e1.record()
            # the whole chain stays on the device (one host read: the labels); at world > 1
            # the per-label entropic GW is split over the ranks (one all-reduce of the plans)
            Tv, _ = perturbot.per_epoch_coupling_device(Xa, Ya, La, eps=eps,
                                                        max_per_label=per_label,
                                                        comm=comm if world > 1 else None)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
            tg.append(e0.elapsed_time(e1))
        t = torch.tensor([sorted(ts)[1], sorted(tg)[1]], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        out.update({"ms_per_epoch_call": float(t[0]), "allgather_ms": float(t[1]),
                    "plan_shape": list(Tv.shape),
                    "note": ("max over ranks; after the all-gather the per-label entropic GW is "
                             "split over the ranks (labels round-robin, one all-reduce of the "
                             "plans, otfuse.distributed.split_label_plans) and the 2048^2 feature "
                             "solve is replicated (one latency-bound resident launch); "
                             "device-resident (otfuse.perturbot.per_epoch_coupling_device)")})
        comm.close()
    except Exception as e:  # noqa: BLE001
        out["error"] = repr(e)
    return out


if __name__ == "__main__":
    main()
