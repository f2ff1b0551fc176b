"""Timing + accuracy probe of the MFMA cost kernel (GPU box).

Per case: median ms of ops.pairwise_cost / pairwise_cost_ex over reps (HIP events on
the current stream), the implied fp16-MFMA TF/s (3 products for the split path), and
the max relative error against an fp64 torch reference on a row sample.
    python tools/cost_probe.py
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd")
for _p in (PKG, REPO):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402


def timed(fn, reps=10):
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


def case(name, n, m, d, in_dt, out_dt):
    from otfuse import ops
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(5)
    X = torch.randn(n, d, generator=g).to(dev, in_dt)
    Y = torch.randn(m, d, generator=g).to(dev, in_dt)
    if in_dt == torch.float32 and out_dt == torch.float32:
        fn = lambda: ops.pairwise_cost(X, Y)  # noqa: E731
    else:
        fn = lambda: ops.pairwise_cost_ex(X, Y, out_dtype=out_dt)  # noqa: E731
    ms = timed(fn)
    out = fn()
    C = out[0]
    unit = out[2] if len(out) > 2 else None
    rows = torch.arange(0, n, max(1, n // 64), device=dev)
    ref = torch.cdist(X[rows].double(), Y.double()) ** 2
    got = C[rows].double() * (unit.double() if unit is not None else 1.0)
    err = ((got - ref).abs().max() / ref.abs().max()).item()
    nprod = 3 if in_dt == torch.float32 else 1
    tf = nprod * 2.0 * n * m * d / (ms * 1e-3) / 1e12
    print(json.dumps({"case": name, "n": n, "m": m, "d": d, "ms": ms, "fp16_tflops": tf,
                      "max_rel_err": err}), flush=True)


def main():
    case("metric_f32", 4096, 4096, 512, torch.float32, torch.float32)
    case("config5_f16", 8192, 8192, 1024, torch.float16, torch.float16)
    case("ragged_f32", 1000, 777, 300, torch.float32, torch.float32)
    case("ragged_big_f32", 4100, 3999, 300, torch.float32, torch.float32)
    case("ragged_f16", 999, 1025, 130, torch.float16, torch.float16)


if __name__ == "__main__":
    main()
