"""Fused Sinkhorn pass time vs problem size (fp32, d = 512 costs, POT flavour).
Prints mean pass time (HIP events around each pass) and the algorithmic HBM rate."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd"))

import torch  # noqa: E402

from otfuse import ops  # noqa: E402

dev = torch.device("cuda", 0)
sizes = [int(x) for x in sys.argv[1:]] or [1024, 2048, 4096, 8192, 16384]
for N in sizes:
    g = torch.Generator(device=dev).manual_seed(0)
    C = torch.rand((N, N), device=dev, generator=g)
    a = torch.full((N,), 1.0 / N, device=dev)
    ws = ops.sinkhorn_workspace(N, N, torch.float32, 30, dev)
    ms = min(ops.sinkhorn_profile(a, a, C, 0.1, 30, workspace=ws) for _ in range(3))
    print(f"N={N:6d}  pass {ms * 1e3:8.2f} us  {N * N * 4 / (ms * 1e-3) / 1e9:7.0f} GB/s", flush=True)
