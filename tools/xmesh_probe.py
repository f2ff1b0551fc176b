"""Cross-rank mesh probe on ONE device: two processes share cuda:0 (gloo for the IPC
handles), each solves its slab of one problem with the in-kernel exchange (xmesh), and
the same slab alone (the single-rank mesh, no exchange).  The per-iteration difference is
the exchange hop measured through this device's memory (not xGMI: the 8-GPU node's
cross-device latency comes on top -- DESIGN.md 6).  Slopes from two iteration counts.

  python tools/xmesh_probe.py [rows_per_rank] [m] [fp16]
"""
import json
import os
import socket
import sys

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd")


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, rows, m, f16, out):
    for p in (PKG, REPO):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import otfuse.distributed as D
    from otfuse import ops
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(100 + rank)
    C = torch.rand(rows, m, device=dev, generator=g)
    if f16:
        C = C.half()
    n = rows * world
    a = torch.full((rows,), 1.0 / n, device=dev)
    b = torch.full((m,), 1.0 / m, device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    xp = D.XPeer(m)
    res = {}
    for iters in (100, 400):
        ts = []
        for _ in range(5):
            dist.barrier()
            torch.cuda.synchronize()
            e0.record()
            r = D.sinkhorn_xsweep(a, b, C, 0.1, xp, n_total=n, max_iter=iters, stop_thr=0.0,
                                  want_plan=False, engine="mesh")
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        res[f"xmesh_{iters}"] = sorted(ts)[2]
        res["engine"] = r.info()["engine_name"]
    xp.close()
    dist.barrier()
    # the same slab alone: the single-rank mesh (one rank at a time, the other waits)
    for turn in range(world):
        if turn == rank:
            a1 = torch.full((rows,), 1.0 / rows, device=dev)
            for iters in (100, 400):
                ts = []
                for _ in range(5):
                    torch.cuda.synchronize()
                    e0.record()
                    ops.sinkhorn(a1, b, C, 0.1, max_iter=iters, stop_thr=0.0, want_plan=False, engine="mesh")
                    e1.record()
                    torch.cuda.synchronize()
                    ts.append(e0.elapsed_time(e1))
                res[f"mesh_{iters}"] = sorted(ts)[2]
        dist.barrier()
    res["xmesh_us_per_iter"] = (res["xmesh_400"] - res["xmesh_100"]) * 1e3 / 300
    res["mesh_us_per_iter"] = (res["mesh_400"] - res["mesh_100"]) * 1e3 / 300
    res["exchange_us_per_iter"] = res["xmesh_us_per_iter"] - res["mesh_us_per_iter"]
    json.dump(res, open(os.path.join(out, f"xmesh_probe_r{rank}.json"), "w"))
    dist.destroy_process_group()


if __name__ == "__main__":
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    m = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
    f16 = len(sys.argv) > 3 and sys.argv[3] == "fp16"
    out = os.path.join(REPO, "gpurun_out")
    os.makedirs(out, exist_ok=True)
    mp.spawn(_worker, args=(2, _port(), rows, m, f16, out), nprocs=2, join=True)
    for r in range(2):
        print(json.dumps({"rank": r, "rows_per_rank": rows, "m": m, "fp16": f16,
                          **json.load(open(os.path.join(out, f"xmesh_probe_r{r}.json")))}))
