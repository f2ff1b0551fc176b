"""GW kernel latency probe: per-epoch shapes (labels x samples), costs precomputed.
Run under rocprofv3 --kernel-trace --stats for per-kernel device time."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from otfuse import gw  # noqa: E402
from otfuse.synthetic import paired_embeddings  # noqa: E402

dev = torch.device("cuda", 0)
for labels, per, d in [(2, 64, 512), (2, 130, 512), (8, 64, 512)]:
    C1s, C2s, C1e, C2e = [], [], [], []
    for k in range(labels):
        X, Y, _ = paired_embeddings(per, d, seed=500 + k)
        X, Y = torch.from_numpy(X).to(dev), torch.from_numpy(Y).to(dev)
        C1s.append(gw.pairwise_cost_f64(X, None, metric="euclidean", scale_max=True)[0])
        C2s.append(gw.pairwise_cost_f64(Y, None, metric="euclidean", scale_max=True)[0])
        C1e.append(gw.pairwise_cost_f64(X, None, metric="sqeuclidean", zero_diag=False, scale_max=True)[0])
        C2e.append(gw.pairwise_cost_f64(Y, None, metric="sqeuclidean", zero_diag=False, scale_max=True)[0])
    for name, fn in [("cg", lambda: gw.solve_batched(C1s, C2s, gw.GW_CG, max_iter=10000, log_len=1)),
                     ("entropic", lambda: gw.solve_batched(C1e, C2e, gw.GW_ENTROPIC, max_iter=2000,
                                                           eps=5e-3, log_len=1))]:
        r = fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            r = fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 5 * 1e3
        info = r.infos()
        print(f"{labels}x{per} {name}: {dt:.3f} ms/call wall, outer {[i['n_iter'] for i in info]}, "
              f"inner {[i['inner_iters'] for i in info]}", flush=True)
