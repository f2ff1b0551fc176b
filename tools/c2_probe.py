"""Config-2 probe: ms per training step of the OT block (forward + backward, bench.py
batch_ot_leg) and the engine that ran, under the environment given (A/B of gather forms).
Usage: python tools/c2_probe.py [reps]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from otfuse import fusion  # noqa: E402
from otfuse.synthetic import paired_embeddings  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda", 0)
X, Y, _ = paired_embeddings(8, 512, seed=321)
mri = torch.from_numpy(X).to(dev).requires_grad_(True)
pet = torch.from_numpy(Y).to(dev).requires_grad_(True)


def step():
    loss, _, T = fusion.ot_alignment_loss(mri, pet, eps=1e-2)
    loss.backward()
    return loss


for _ in range(3):
    step()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps):
    loss = step()
e1.record()
torch.cuda.synchronize()
env = {k: v for k, v in os.environ.items() if k.startswith("OTF_")}
print(f"{env} config-2 step {e0.elapsed_time(e1) / reps:.3f} ms, loss {float(loss):.8f}")
