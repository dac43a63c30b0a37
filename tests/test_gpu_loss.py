"""GPU: the fused compute_loss (dadmm_loss / dadmm_loss_grad) against the torch formula of the
reference (gnn_dlasso_utils.py:27-88): values, the NaN/Inf fallback, and dL/dY."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _torch_loss(Y, label):
    import gnn_dlasso_utils as U
    losses = U.layer_losses(Y, label)
    return losses.mean() + 1e-8, losses[-1] + 1e-8


@pytest.mark.parametrize("K,B,P,n,ns", [(25, 64, 5, 256, 256), (7, 33, 3, 62, 64), (1, 5, 1, 4, 4),
                                        (12, 300, 16, 512, 512)])
def test_fused_loss_and_gradient_match_torch(cuda, K, B, P, n, ns):
    from dadmm_hip.loss import fused_compute_loss
    g = torch.Generator(cuda).manual_seed(K * 1000 + n)
    base = torch.randn(K, B, P, ns, device=cuda, generator=g)
    label = torch.randn(B, n, 1, device=cuda, generator=g)
    Y = base[..., :n].unsqueeze(-1).requires_grad_(False)
    Yf = Y.detach().clone().requires_grad_(True)          # torch path (contiguous copy)
    Yk = base.clone().requires_grad_(True)
    Yv = Yk[..., :n].unsqueeze(-1)
    lm, lf = fused_compute_loss(Yv, label)
    rm, rf = _torch_loss(Yf, label)
    torch.testing.assert_close(lm, rm, rtol=1e-5, atol=0)
    torch.testing.assert_close(lf, rf, rtol=1e-5, atol=0)
    (0.3 * lm + 1.7 * lf).backward()
    (0.3 * rm + 1.7 * rf).backward()
    torch.testing.assert_close(Yk.grad[..., :n].unsqueeze(-1), Yf.grad, rtol=1e-5, atol=1e-12)
    assert bool((Yk.grad[..., n:] == 0).all())


def test_fused_loss_fallback_on_nonfinite(cuda):
    from dadmm_hip.loss import fused_compute_loss
    Y = torch.randn(4, 8, 2, 16, 1, device=cuda).requires_grad_(True)
    label = torch.randn(8, 16, 1, device=cuda)
    with torch.no_grad():
        Y[2, 3, 1, 5, 0] = float("nan")
    lm, lf = fused_compute_loss(Y, label)
    assert float(lm) == 1.0 and float(lf) == 1.0
    (lm + lf).backward()
    assert bool((Y.grad == 0).all())
    label2 = label.clone()
    label2[0, 0, 0] = float("inf")
    lm, lf = fused_compute_loss(torch.randn(4, 8, 2, 16, 1, device=cuda), label2)
    assert float(lm) == 1.0 and float(lf) == 1.0


def test_compute_loss_uses_the_fused_kernels_for_module_output(cuda):
    import gnn_dlasso_utils as U
    from dadmm_hip import loss as L
    Y = torch.randn(3, 4, 2, 8, device=cuda)[..., None]
    assert L._layout(Y) is not None
    assert L._layout(Y.cpu()) is None
    assert L._layout(Y.transpose(1, 2)) is None
    lm, lf = U.compute_loss(Y, torch.randn(4, 8, 1, device=cuda))
    assert lm.grad_fn is None or "LossFn" in type(lm.grad_fn).__name__
