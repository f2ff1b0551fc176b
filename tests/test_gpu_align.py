"""The training step's fused alignment kernels against torch's autograd of the reference
formula (cosine_loss, MRI_PET_OT_nojax.py:552-560, applied at :718-725):
otf_cosine_align (loss + both gradients, one launch) and otf_ot_align_backward
(g_pet = (g_loss gy + g_ot) @ Tn, g_mri = g_loss gx, one launch).  The torch fp32
reference is the numerics oracle here (floating point, 1e-5 relative)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref_loss_grads(X, Y):
    from otfuse.fusion import cosine_loss
    x = X.detach().float().requires_grad_(True)
    y = Y.detach().float().requires_grad_(True)
    L = cosine_loss(x, y)
    gx, gy = torch.autograd.grad(L, (x, y))
    return L.detach(), gx, gy


def _rel(a, b):
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


@pytest.mark.parametrize("B,d,dt", [(8, 512, torch.float32), (1, 64, torch.float32),
                                    (32, 2048, torch.float32), (8, 512, torch.bfloat16),
                                    (5, 300, torch.float16), (70, 33, torch.float32)])
def test_cosine_align_vs_torch_autograd(dev, B, d, dt):
    from otfuse import ops
    g = torch.Generator(device=dev).manual_seed(B * 1000 + d)
    X = torch.randn(B, d, device=dev, generator=g).to(dt)
    Y = torch.randn(B, d, device=dev, generator=g) * 3 + 0.5
    L, gx, gy, keep = ops.cosine_align(X, Y)
    Lr, gxr, gyr = _ref_loss_grads(X, Y)
    assert int(keep) == 1
    assert abs(float(L) - float(Lr)) < 1e-5
    assert _rel(gx, gxr) < 1e-5 and _rel(gy, gyr) < 1e-5


def test_cosine_align_zeroes_nonfinite_and_not_ok(dev):
    from otfuse import ops
    X = torch.randn(8, 64, device=dev)
    Y = torch.randn(8, 64, device=dev)
    Y[3, 5] = float("nan")
    L, gx, gy, keep = ops.cosine_align(X, Y)
    assert int(keep) == 0 and float(L) == 0.0
    assert torch.count_nonzero(gx) == 0 and torch.count_nonzero(gy) == 0
    L, gx, gy, keep = ops.cosine_align(X, torch.randn(8, 64, device=dev),
                                       ok=torch.zeros((), dtype=torch.bool, device=dev))
    assert int(keep) == 0 and float(L) == 0.0 and torch.count_nonzero(gx) == 0


@pytest.mark.parametrize("status,stop,stalled,keep", [
    ("SK_MAX_ITER", 1, 0, 1), ("SK_CONVERGED", 1, 0, 1), ("SK_NUMERICAL_BREAK", 1, 0, 1),
    ("SK_TIMEOUT", 1, 1, 0), ("SK_RUNNING", 0, 0, 0), ("SK_MAX_ITER", 0, 0, 0), ("SK_MAX_ITER", 1, 1, 0)])
def test_cosine_align_checks_the_solve_info(dev, status, stop, stalled, keep):
    """The loss kernel reads the solve's info words (sk_info): only a finished solve --
    final status, stop set, no stalled workgroup -- keeps the loss and its gradients."""
    from otfuse import _lib as L
    from otfuse import ops
    info = torch.zeros(L.INFO_INT32S, dtype=torch.int32)
    info[L.INFO_FIELDS.index("status")] = getattr(L, status)
    info[L.INFO_FIELDS.index("stop")] = stop
    info[L.INFO_FIELDS.index("stalled")] = stalled
    X = torch.randn(8, 64, device=dev)
    Y = torch.randn(8, 64, device=dev)
    L0, gx0, gy0, _ = ops.cosine_align(X, Y)
    L1, gx1, gy1, k1 = ops.cosine_align(X, Y, sk_info=info.to(dev))
    assert int(k1) == keep
    if keep:
        assert torch.equal(L0, L1) and torch.equal(gx0, gx1) and torch.equal(gy0, gy1)
    else:
        assert float(L1) == 0.0 and torch.count_nonzero(gx1) == 0 and torch.count_nonzero(gy1) == 0


@pytest.mark.parametrize("B,d,d2", [(8, 512, 512), (3, 100, 77), (20, 2048, 2048), (9, 64, 130)])
def test_ot_align_backward_vs_torch(dev, B, d, d2):
    from otfuse import ops
    g = torch.Generator(device=dev).manual_seed(d + d2)
    gx = torch.randn(B, d, device=dev, generator=g)
    gy = torch.randn(B, d, device=dev, generator=g)
    g_ot = torch.randn(B, d, device=dev, generator=g)
    Tn = torch.rand(d, d2, device=dev, generator=g)
    gl = torch.tensor(0.7, device=dev)
    g_mri, g_pet = ops.ot_align_backward(gx, gy, Tn, g_loss=gl, g_ot=g_ot)
    ref = (0.7 * gy.double() + g_ot.double()) @ Tn.double()
    assert _rel(g_pet.double(), ref) < 1e-5
    assert torch.allclose(g_mri, 0.7 * gx, rtol=1e-6, atol=0)
    # loss-only backward: no g_ot; keep = 0 and a NaN plan give exact zeros
    Tn[2, 3] = float("nan")
    keep = torch.zeros((), dtype=torch.uint8, device=dev)
    _, g_pet = ops.ot_align_backward(gx, gy, Tn, g_loss=gl, keep=keep)
    assert torch.count_nonzero(g_pet) == 0


def test_ot_alignment_loss_end_to_end_matches_autograd_form(dev):
    """The whole OT block (solve -> fused apply -> fused loss -> fused backward) against
    the same plan applied and differentiated by torch."""
    from otfuse.fusion import cosine_loss, ot_alignment_loss
    g = torch.Generator(device=dev).manual_seed(5)
    X = torch.randn(8, 512, device=dev, generator=g).requires_grad_(True)
    Y = torch.randn(8, 512, device=dev, generator=g).requires_grad_(True)
    loss, ot_mri, T = ot_alignment_loss(X, Y, eps=1e-2)
    (loss + 0.1 * ot_mri.square().sum()).backward()
    X2 = X.detach().clone().requires_grad_(True)
    Y2 = Y.detach().clone().requires_grad_(True)
    ot2 = Y2 @ T.t()
    (cosine_loss(X2, ot2) + 0.1 * ot2.square().sum()).backward()
    assert abs(float(loss) - float(cosine_loss(X2, ot2))) < 1e-5
    assert _rel(X.grad, X2.grad) < 1e-4 and _rel(Y.grad, Y2.grad) < 1e-4
