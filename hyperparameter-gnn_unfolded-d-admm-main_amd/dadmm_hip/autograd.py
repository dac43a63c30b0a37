"""autograd plumbing for the fused forward (the drivers call ``loss.backward()`` through it)."""
from __future__ import annotations

import torch

from . import _lib
from .ops import forward_raw


class NonFiniteError(RuntimeError):
    """A non-finite value reached one of the reference's NaN/Inf guards."""


class _UnfoldedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, table, op, b, graphs, y0, U0, d0, variant):
        Y, _, status = forward_raw(op, b, graphs, table.detach(), y0, U0, d0, variant=variant)
        st = int(status.item())
        if st != 0:
            raise NonFiniteError(
                f"non-finite values reached the reference's NaN/Inf guards (status bits {st:#x}: "
                "1 y0, 2 U0, 4 gradient, 8 hyper-parameters); the guarded path is not built yet")
        ctx.mark_non_differentiable()
        return Y

    @staticmethod
    def backward(ctx, gY):
        raise NotImplementedError(
            "the adjoint (backward) kernel of the fused D-ADMM forward is not built yet")


def dadmm_unfolded_apply(op, b, graphs, table, y0, U0, d0, variant=_lib.VARIANT_UNFOLDED):
    """Y [K,B,P,n] = the K-step recurrence; differentiable w.r.t. ``table`` once the adjoint
    kernel exists."""
    return _UnfoldedFn.apply(table, op, b, graphs, y0, U0, d0, variant)
