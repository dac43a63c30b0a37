"""Fused compute_loss on the device (C ABI dadmm_loss / dadmm_loss_grad) with its autograd rule.

Reference: gnn_dlasso_utils.compute_loss (gnn_dlasso_utils.py:27-88). One pass over the iterates
for (loss_mean, loss_final) and one pass for dL/dY, deterministic, no host synchronisation.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from .ops import _ptr, _stream


def _layout(Y):
    """(K, B, P, n, n_store) when Y [K,B,P,n,1] (or [K,B,P,n]) is a float32 CUDA view of rows of
    length n_store >= n (the layout the HIP forward returns), else None."""
    if Y.device.type != "cuda" or Y.dtype != torch.float32:
        return None
    if Y.dim() == 5 and Y.shape[-1] == 1:
        Y4 = Y[..., 0]
    elif Y.dim() == 4:
        Y4 = Y
    else:
        return None
    K, B, P, n = Y4.shape
    st = Y4.stride()
    ns = st[2]
    if st[3] != 1 or ns < n or st[1] != P * ns or st[0] != B * P * ns:
        return None
    return K, B, P, n, ns


class LossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, Y, label, lay):
        K, B, P, n, ns = lay
        dev = Y.device
        L = _lib.load()
        label = label.reshape(B, n).contiguous().float()
        scratch = torch.empty(L.dadmm_loss_scratch_bytes(K, B * P, n) // 4 + 1, device=dev)
        losses = torch.empty(K, device=dev)
        out = torch.empty(2, device=dev)
        flags = torch.empty(2, dtype=torch.int32, device=dev)
        with torch.cuda.device(dev):
            _lib.check("dadmm_loss", L.dadmm_loss(K, B, P, n, ns, _ptr(Y), _ptr(label),
                                                  _ptr(losses), _ptr(out), _ptr(flags),
                                                  _ptr(scratch), _stream(dev)))
        ctx.save_for_backward(Y, label, flags)
        ctx.lay = lay
        ctx.shape = Y.shape
        return out[0], out[1]

    @staticmethod
    def backward(ctx, g_mean, g_final):
        Y, label, flags = ctx.saved_tensors
        K, B, P, n, ns = ctx.lay
        dev = Y.device
        gout = torch.stack([g_mean if g_mean is not None else torch.zeros((), device=dev),
                            g_final if g_final is not None else torch.zeros((), device=dev)])
        gout = gout.float().contiguous()
        dY = torch.empty((K, B, P, ns), device=dev)
        with torch.cuda.device(dev):
            _lib.check("dadmm_loss_grad", _lib.load().dadmm_loss_grad(
                K, B, P, n, ns, _ptr(Y), _ptr(label), _ptr(flags), _ptr(gout), _ptr(dY),
                _stream(dev)))
        dY = dY if ns == n else dY[..., :n]
        return dY.reshape(ctx.shape) if ns == n else dY.unsqueeze(-1).reshape(ctx.shape), None, None


def fused_compute_loss(Y, label):
    """(loss_mean, loss_final) by the fused kernels, or None when Y's layout does not qualify."""
    lay = _layout(Y)
    if lay is None or label.requires_grad or label.device != Y.device:
        return None
    if label.numel() != lay[1] * lay[3]:
        return None
    return LossFn.apply(Y, label, lay)
