"""Where the float32 mesh's FETCH_SIZE comes from: the same 4096 x 4096 float32 solve at
1, 10 and 100 iterations, with and without the plan (3 runs each, dispatch order fixed).
Run under rocprofv3 --pmc FETCH_SIZE (or WRITE_SIZE) --kernel-trace; tools/f32_fetch_read.py
splits the counter rows by config."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd"))
from otfuse import ops  # noqa: E402

dev = torch.device("cuda:0")
n = 4096
g = torch.Generator(device=dev).manual_seed(5)
C = torch.rand(n, n, device=dev, generator=g, dtype=torch.float32)
a = torch.full((n,), 1.0 / n, device=dev, dtype=torch.float32)
ws = ops.sinkhorn_workspace(n, n, torch.float32, 100, dev)
P = torch.empty(n, n, device=dev, dtype=torch.float32)
for it in (1, 10, 100):
    for plan in (True, False):
        for _ in range(3):
            r = ops.sinkhorn(a, a, C, 0.1, max_iter=it, stop_thr=0.0, workspace=ws, engine="mesh",
                             want_plan=plan, plan_out=P if plan else None)
            assert r.info()["engine_name"] == "mesh", r.info()
torch.cuda.synchronize()
print("configs: iters (1, 10, 100) x plan (yes, no) x 3", flush=True)
