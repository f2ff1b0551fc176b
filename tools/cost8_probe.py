"""A/B of the 256 x 256 cost kernels in one process (GPU box): the 8-phase LDS-DMA kernel
(OTF_COST_8PH=1, the default) against the register-staged kernels (OTF_COST_8PH=0:
cost_big16_kernel / cost_big_kernel), interleaved rounds; per case the median prep and
kernel times from the library's own events (OTF_COST_PHASES=1) and the kernel's fraction
of the dense fp16 MFMA peak (2.5 PFLOP/s; 3 products per split-fp16 dot).
    python tools/cost8_probe.py [rounds]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd"))
import torch  # noqa: E402
from otfuse import ops  # noqa: E402

dev = torch.device("cuda", 0)
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
os.environ["OTF_COST_PHASES"] = "1"
cases = [("metric_f32", 4096, 4096, 512, torch.float32, torch.float32),
         ("config5_f16", 8192, 8192, 1024, torch.float16, torch.float16),
         ("f16_in_f32_out", 4096, 4096, 512, torch.float16, torch.float32),
         ("f32_in_f16_out", 8192, 8192, 1024, torch.float32, torch.float16)]
g = torch.Generator(device="cpu").manual_seed(5)
data = {c[0]: (torch.randn(c[1], c[3], generator=g).to(dev, c[4]), torch.randn(c[2], c[3], generator=g).to(dev, c[4]))
        for c in cases}
res = {}
for r in range(rounds):
    for name, n, m, d, idt, odt in cases:
        X, Y = data[name]
        for v in ("1", "0"):
            os.environ["OTF_COST_8PH"] = v
            ks, ps = [], []
            for _ in range(6):
                ops.pairwise_cost_ex(X, Y, out_dtype=odt)
                p, k = ops.cost_last_phases()
                ks.append(k)
                ps.append(p)
            res.setdefault((name, v), []).append((sorted(ks)[3], sorted(ps)[3]))
for name, n, m, d, idt, odt in cases:
    nprod = 3 if idt == torch.float32 else 1
    for v in ("1", "0"):
        k = min(x[0] for x in res[(name, v)])
        p = min(x[1] for x in res[(name, v)])
        frac = nprod * 2.0 * n * m * d / (k * 1e-3) / 2.5e15
        print("%-16s 8ph=%s kernel %.1f us (rounds %s) prep %.1f us, %.3f of fp16 peak" % (
            name, v, 1e3 * k, " ".join("%.1f" % (1e3 * x[0]) for x in res[(name, v)]), 1e3 * p, frac), flush=True)
