"""Pairwise-cost kernel probe: event time of ops.pairwise_cost (split-fp16 MFMA, fp32 out)
and pairwise_cost_ex variants at the metric shape, plus max error vs float64 on a row
sample.  python tools/bench_cost.py [N] [d]   (OTF_COST_RING=0/1 picks the 256 x 256 kernel)"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from otfuse import ops  # noqa: E402
from otfuse.synthetic import paired_embeddings  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
d = int(sys.argv[2]) if len(sys.argv) > 2 else 512
dev = torch.device("cuda", 0)
X, Y, _ = paired_embeddings(N, d, seed=1234)
Xd, Yd = torch.from_numpy(X).to(dev), torch.from_numpy(Y).to(dev)


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


rows = np.arange(0, N, max(1, N // 64))
ref = ((X[rows].astype(np.float64) ** 2).sum(1)[:, None] + (Y.astype(np.float64) ** 2).sum(1)[None]
       - 2.0 * X[rows].astype(np.float64) @ Y.astype(np.float64).T)
for algo in ("split16", "f32"):
    ms = timeit(lambda: ops.pairwise_cost(Xd, Yd, algo=algo))
    C, _ = ops.pairwise_cost(Xd, Yd, algo=algo)
    err = np.abs(C.cpu().numpy()[rows] - ref).max() / np.abs(ref).max()
    print(f"{algo:8s} {ms * 1e3:8.1f} us  {2.0 * N * N * d / ms / 1e9:7.1f} TFLOP/s fp32-eq  "
          f"max err / max C {err:.2e}", flush=True)
Xh, Yh = Xd.half(), Yd.half()
C0, _, _ = ops.pairwise_cost_ex(Xh, Yh, out_dtype=torch.float16)
ms = timeit(lambda: ops.pairwise_cost_ex(Xh, Yh, out_dtype=torch.float16))
print(f"f16-in f16-out {ms * 1e3:8.1f} us  {2.0 * N * N * d / ms / 1e9:7.1f} TFLOP/s", flush=True)
