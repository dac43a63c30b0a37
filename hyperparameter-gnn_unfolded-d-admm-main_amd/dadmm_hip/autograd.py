"""autograd plumbing for the fused forward (the drivers call ``loss.backward()`` through it)."""
from __future__ import annotations

import os

import torch

from . import _lib
from .ops import describe_status, forward_raw

# DADMM_GUARD_WARNINGS=1: synchronise after every forward and print the reference's guard
# warnings (unfolded_DLASSO.py:56-104). Off by default: the guards themselves are applied on the
# device either way; only the printing needs the host round trip.
_WARN = os.environ.get("DADMM_GUARD_WARNINGS", "0") not in ("", "0")


class GuardTimeoutError(RuntimeError):
    """The gated stepwise recomputation could not synchronise its grid (Y is invalid)."""


def check_status(status: torch.Tensor) -> int:
    """Synchronise on ``status`` and return its bits; raise if the guarded recomputation failed."""
    st = int(status.item())
    if st & _lib.STATUS_BARRIER_TIMEOUT:
        raise GuardTimeoutError("; ".join(describe_status(st)))
    return st


class _UnfoldedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, table, op, b, graphs, y0, U0, d0, variant):
        Y, _, status = forward_raw(op, b, graphs, table.detach(), y0, U0, d0, variant=variant)
        if _WARN:
            for msg in describe_status(check_status(status)):
                print(f"Warning: {msg}")
        ctx.mark_non_differentiable(status)
        return Y, status

    @staticmethod
    def backward(ctx, gY, gstatus):
        raise NotImplementedError(
            "the adjoint (backward) kernel of the fused D-ADMM forward is not built yet")


def dadmm_unfolded_apply(op, b, graphs, table, y0, U0, d0, variant=_lib.VARIANT_UNFOLDED):
    """(Y [K,B,P,n], status [1] int32 device tensor) = the K-step recurrence with the reference's
    guards; Y is differentiable w.r.t. ``table`` once the adjoint kernel exists."""
    return _UnfoldedFn.apply(table, op, b, graphs, y0, U0, d0, variant)
