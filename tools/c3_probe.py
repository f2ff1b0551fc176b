"""Config-3 chain split (GPU box): per-label EGW, then get_coupling_fot's parts -- feature
cost, the OTT-flavour solve (iterations, engine), and the host-side tail (numpy copy)."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, "ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd")
sys.path.insert(0, ".")
from otfuse import ops, perturbot  # noqa: E402

dev = torch.device("cuda", 0)
rng = np.random.default_rng(0)
d, ns = 2048, 64
xd = {0: rng.standard_normal((ns, d)).astype(np.float32), 1: rng.standard_normal((ns, d)).astype(np.float32)}
yd = {0: rng.standard_normal((ns, d)).astype(np.float32), 1: rng.standard_normal((ns, d)).astype(np.float32)}
for rep in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    Ts, _ = perturbot.get_coupling_egw_ott_fixed((xd, yd), eps=5e-3)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    Tv, log = perturbot.get_coupling_fot((xd, yd), Ts, eps=5e-3)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    # the same solve, timed alone
    X = np.concatenate([xd[k] for k in xd]); Y = np.concatenate([yd[k] for k in xd])
    Tsm = perturbot.mdict_to_matrix(Ts, np.repeat([0, 1], ns), np.repeat([0, 1], ns)) if isinstance(Ts, dict) else Ts
    Tsm = np.asarray(Tsm, dtype=np.float64); Tsm = Tsm / Tsm.sum()
    M = ops.feature_cost(torch.as_tensor(X, device=dev), torch.as_tensor(Y, device=dev),
                         Ts=torch.as_tensor(Tsm, device=dev), weights="fot")
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    for se in (50, 0):
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        res, _ = perturbot.solve_ott(M, 5e-3, sync_every=se)
        info = res.info()
        t5 = time.perf_counter()
        print(f"rep {rep}: egw {1e3*(t1-t0):.2f} ms, fot {1e3*(t2-t1):.2f} ms, solve(sync_every={se}) "
              f"{1e3*(t5-t4):.2f} ms, niter {info['niter']} status {info['status_name']} engine {info['engine_name']}",
              flush=True)
