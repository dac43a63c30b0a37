"""Drop-in ``gnn_dlasso_utils``: the input generator and the loss the drivers call.

``set_A``         reference gnn_dlasso_utils.py:4-16   (per-agent A_p = U clamp(S, 0.1, 10) V^T)
``compute_loss``  reference gnn_dlasso_utils.py:27-88  (per-layer MSE, NaN/Inf -> (1, 1))
``compute_loss2`` reference gnn_dlasso_utils.py:18-25  (weighted variant; unused by the drivers)

``compute_loss`` is vectorised (one reduction instead of K*P ``mse_loss`` calls) and keeps the
reference's NaN/Inf fallback without the host synchronisations: the fallback value is selected on
the device with ``torch.where``.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

_EPS = 1e-8


def set_A(args):
    """[1, P, m, n] float32 on the CPU: each A_p is a Gaussian m x n matrix whose singular values
    are clamped into [0.1, 10]."""
    P, m, n = args.P, args.m, args.n
    blocks = []
    for _ in range(P):
        g = torch.randn((m, n))
        u, s, v = torch.svd(g)
        blocks.append(u @ torch.diag(s.clamp(min=0.1, max=10.0)) @ v.T)
    return torch.stack(blocks).unsqueeze(0)


def layer_losses(Y, label):
    """losses[k] = (1/P) sum_p mean_{b,n} (Y[k,b,p,n] - label[b,n])^2  -> [K]."""
    K, B, P, n = Y.shape[:4]
    diff = Y.reshape(K, B, P, n) - label.reshape(1, B, 1, n)
    per_agent = diff.pow(2).mean(dim=(1, 3))          # [K, P]
    return per_agent.sum(dim=1) / P


def compute_loss(Y, label):
    """Y [K,B,P,n,1], label [B,n,1] -> (loss_mean, loss_final) as 0-dim tensors.

    Returns (1.0, 1.0) if Y, the label or any layer loss is non-finite (reference :36-43,
    :69-71, :83-86). Iterates in the HIP forward's layout go through the fused loss kernels
    (dadmm_hip.loss: one pass forward, one pass for dL/dY); anything else (e.g. CPU tensors)
    through the same formula in torch.

    Iterates returned by the HIP forwards carry their device status word. If the forward's
    guarded recomputation timed out (its Y is NaN-poisoned, a case the reference cannot reach)
    both losses are NaN instead of the fallback (1, 1), selected on the device: no host
    synchronisation is added. The returned losses carry the same status word, so
    ``dadmm_hip.autograd.raise_if_timed_out(loss)`` raises GuardTimeoutError wherever the caller
    synchronises anyway, and ``loss.backward()`` raises it in the adjoint."""
    from dadmm_hip.loss import fused_compute_loss
    fused = fused_compute_loss(Y, label)
    if fused is not None:
        return _poison_timed_out(Y, *fused)
    losses = layer_losses(Y, label)
    ok = torch.isfinite(Y).all() & torch.isfinite(label).all() & torch.isfinite(losses).all()
    one = torch.ones((), dtype=losses.dtype, device=losses.device)
    loss_mean = torch.where(ok, losses.mean() + _EPS, one)
    loss_final = torch.where(ok, losses[-1] + _EPS, one)
    loss_mean = torch.where(torch.isfinite(loss_mean), loss_mean, one)
    loss_final = torch.where(torch.isfinite(loss_final), loss_final, one)
    return _poison_timed_out(Y, loss_mean, loss_final)


def _poison_timed_out(Y, loss_mean, loss_final):
    """NaN losses when Y's forward reported a guard-recomputation timeout (device-side select,
    no sync); the losses inherit Y's status word."""
    status = getattr(Y, "_dadmm_status", None)
    if status is None:
        return loss_mean, loss_final
    from dadmm_hip import _lib
    from dadmm_hip.autograd import tag_status
    bad = (status.reshape(-1)[0] & _lib.STATUS_BARRIER_TIMEOUT) != 0
    if bad.device != loss_mean.device:
        bad = bad.to(loss_mean.device)
    nan = torch.full((), float("nan"), dtype=loss_mean.dtype, device=loss_mean.device)
    return (tag_status(torch.where(bad, nan, loss_mean), status),
            tag_status(torch.where(bad, nan, loss_final), status))


def compute_loss2(Y, label):
    """Weighted loss on the agent-averaged iterates (reference :18-25)."""
    w = label.abs() + 0.0001
    w = w / w.sum(dim=1).unsqueeze(-1)
    y_mean = Y.mean(dim=2)
    loss_final = (F.mse_loss(y_mean[-1], label, reduction="none") * w).sum(dim=1)
    loss_mean = (F.mse_loss(y_mean.mean(dim=0), label, reduction="none") * w).sum(dim=1)
    return loss_mean.mean(), loss_final.mean()
