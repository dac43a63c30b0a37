"""autograd plumbing for the HIP forward (the drivers call ``loss.backward()`` through it).

Training-mode forwards (the hyper-parameter table requires grad) run the recording forward
(``dadmm_forward_record``) and keep the trajectory; ``backward`` runs the adjoint kernel
(``dadmm_backward``) and returns d loss / d table, from which torch autograd continues into
``seq_hyp.param`` (cumsum / sigmoid / penalty / clamp of ``seq_hyperparam.table``).
"""
from __future__ import annotations

import os

import torch

from . import _lib
from .ops import backward_raw, describe_status, forward_raw

# DADMM_GUARD_WARNINGS=1: synchronise after every forward and print the reference's guard
# warnings (unfolded_DLASSO.py:56-104). Off by default: the guards themselves are applied on the
# device either way; only the printing needs the host round trip.
_WARN = os.environ.get("DADMM_GUARD_WARNINGS", "0") not in ("", "0")


class GuardTimeoutError(RuntimeError):
    """The gated stepwise recomputation could not synchronise its grid (Y is invalid)."""


class GuardAdjointError(NotImplementedError):
    """backward through a forward in which one of the reference's NaN/Inf guards fired."""


def check_status(status: torch.Tensor) -> int:
    """Synchronise on ``status`` and return its bits; raise if the guarded recomputation failed."""
    st = int(status.item())
    if st & _lib.STATUS_BARRIER_TIMEOUT:
        raise GuardTimeoutError("; ".join(describe_status(st)))
    return st


class _UnfoldedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, table, op, b, graphs, y0, U0, d0, variant):
        record = ctx.needs_input_grad[0]
        out = forward_raw(op, b, graphs, table.detach(), y0, U0, d0, variant=variant,
                          record=record)
        Y, _, status = out[:3]
        if _WARN:   # the reference's warnings (bit 16 is internal: the exact recomputation ran)
            for msg in describe_status(check_status(status) & ~_lib.STATUS_RECOMPUTE):
                print(f"Warning: {msg}")
        ctx.mark_non_differentiable(status)
        if record:
            ctx.op, ctx.graphs, ctx.traj, ctx.status = op, graphs, out[3], status
        return Y, status

    @staticmethod
    def backward(ctx, gY, gstatus):
        # one host sync per backward. Bit 16 (an asymmetric shared adjacency sent the batch
        # through the exact recomputation, which records the trajectory itself) is no guard event:
        # the adjoints follow any adjacency
        st = check_status(ctx.status) & ~_lib.STATUS_RECOMPUTE
        if st:
            raise GuardAdjointError(
                "backward through a forward in which the reference's NaN/Inf guards fired ("
                + "; ".join(describe_status(st)) + ") is not supported by the adjoint kernel")
        dtable = backward_raw(ctx.op, ctx.graphs, ctx.traj, gY)
        ctx.traj = None
        return dtable, None, None, None, None, None, None, None


def tag_status(Y: torch.Tensor, status: torch.Tensor) -> torch.Tensor:
    """Attach the forward's device status word to the returned iterates: compute_loss turns a
    guard-recomputation timeout into NaN losses on the device (not the reference's silent (1, 1)
    fallback) and passes the word on, so a caller that synchronises anyway can raise
    GuardTimeoutError (raise_if_timed_out); the adjoints raise it in backward."""
    Y._dadmm_status = status
    return Y


def timed_out(Y: torch.Tensor) -> bool:
    """True if ``Y`` (iterates, or the losses compute_loss made from them) came from a forward
    whose guarded recomputation could not synchronise its grid (one host synchronisation; False
    when the tensor carries no status). Multi-rank callers pass it through the collective that
    follows (dist.global_losses(..., timed_out=...)) so every rank raises together."""
    status = getattr(Y, "_dadmm_status", None)
    if status is None:
        return False
    return bool(int(status.item()) & _lib.STATUS_BARRIER_TIMEOUT)


def raise_if_timed_out(Y: torch.Tensor) -> None:
    """GuardTimeoutError if ``Y`` (iterates, or the losses compute_loss made from them) came from
    a forward whose guarded recomputation could not synchronise its grid (one host
    synchronisation; nothing when the tensor carries no status)."""
    status = getattr(Y, "_dadmm_status", None)
    if status is not None:
        check_status(status)


def dadmm_unfolded_apply(op, b, graphs, table, y0, U0, d0, variant=_lib.VARIANT_UNFOLDED):
    """(Y [K,B,P,n], status [1] int32 device tensor) = the K-step recurrence with the reference's
    guards; Y is differentiable w.r.t. ``table`` (adjoint kernel)."""
    return _UnfoldedFn.apply(table, op, b, graphs, y0, U0, d0, variant)
