"""Torch-facing wrappers over the C ABI (device memory, streams and autograd plumbing only).

All arithmetic of the D-ADMM recurrence runs in ``libdadmm.so``; this module validates tensors,
allocates outputs with the torch caching allocator and passes raw device pointers plus the
current HIP stream.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from .graph import GraphBatch


def _dev_check(*tensors):
    for t in tensors:
        if t is None:
            continue
        if t.device.type != "cuda":
            raise RuntimeError(
                "dadmm_hip runs on a ROCm GPU only (tensors must be on a cuda/hip device); "
                f"got a tensor on {t.device}")


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


class PreparedOperator:
    """The per-agent operator prepared once per A (replaces ``self.AtA = compute_Atx(self.A)``,
    unfolded_DLASSO.py:16): padded A and A^T in one device workspace."""

    def __init__(self, A: torch.Tensor):
        if A.dim() == 4:
            if A.shape[0] != 1:
                raise ValueError(f"A must be [1, P, m, n], got {tuple(A.shape)}")
            A = A[0]
        if A.dim() != 3:
            raise ValueError(f"A must be [1, P, m, n] or [P, m, n], got {tuple(A.shape)}")
        _dev_check(A)
        self.P, self.m, self.n = (int(x) for x in A.shape)
        self.n_store = (self.n + 3) & ~3          # kernel needs n % 4 == 0: zero-pad columns
        A = A.detach().to(torch.float32)
        if self.n_store != self.n:
            A = torch.nn.functional.pad(A, (0, self.n_store - self.n))
        A = A.contiguous()
        self.device = A.device
        L = _lib.load()
        d = self.dims(B=0, K=0)
        nbytes = L.dadmm_operator_bytes(ctypes.byref(d))
        if nbytes == 0:
            _lib.check("dadmm_operator_bytes", _lib.DADMM_EINVAL)
        self.workspace = torch.empty(nbytes // 4, dtype=torch.float32, device=self.device)
        with torch.cuda.device(self.device):
            _lib.check("dadmm_prepare_operator",
                       L.dadmm_prepare_operator(ctypes.byref(d), _ptr(A), _ptr(self.workspace),
                                                _stream(self.device)))

    def dims(self, B, K, variant=_lib.VARIANT_UNFOLDED, hyp_rows=1, graph_shared=0):
        return _lib.Dims(B=B, P=self.P, m=self.m, n=self.n_store, K=K, variant=variant,
                         hyp_rows=hyp_rows, graph_shared=int(graph_shared))


def _pad_n(t, n_store):
    if t.shape[-1] == n_store:
        return t
    return torch.nn.functional.pad(t, (0, n_store - t.shape[-1]))


def forward_raw(op: PreparedOperator, b: torch.Tensor, graphs: GraphBatch, hyp: torch.Tensor,
                y0: torch.Tensor, U0: torch.Tensor, d0: torch.Tensor, *,
                variant: int = _lib.VARIANT_UNFOLDED, want_U: bool = False, path: str = "auto"):
    """The K-step forward with the reference's NaN/Inf guards, enqueued on the current stream
    (no host synchronisation). Shapes: b [B,P,m], hyp [K,H,4], y0/U0/d0 [B,P,n].

    path "auto": the fused kernel when the shape is compiled, followed by the device-gated
    stepwise recomputation (runs only if the fused kernel flagged a guard event); otherwise the
    stepwise kernels. "fused" / "stepwise" force one path ("fused" alone does NOT apply the
    guards: its status only flags them).

    Returns (Y [K,B,P,n], U_K [B,P,n] or None, status int32 device tensor [1])."""
    _dev_check(b, hyp, y0, U0, d0, graphs.nbr, graphs.deg)
    if path not in ("auto", "fused", "stepwise"):
        raise ValueError(f"unknown path {path!r}")
    B, P, m = b.shape
    if P != op.P or m != op.m:
        raise ValueError(f"b is [B,{P},{m}], operator is P={op.P}, m={op.m}")
    K, H = int(hyp.shape[0]), int(hyp.shape[1])
    ns = op.n_store
    b = b.contiguous().float()
    hyp = hyp.contiguous().float()
    y0, U0, d0 = (_pad_n(x, ns).contiguous().float() for x in (y0, U0, d0))
    Y = torch.empty((K, B, P, ns), dtype=torch.float32, device=b.device)
    U = torch.empty((B, P, ns), dtype=torch.float32, device=b.device) if want_U else None
    status = torch.zeros(1, dtype=torch.int32, device=b.device)
    d = op.dims(B=B, K=K, variant=variant, hyp_rows=H, graph_shared=graphs.shared)
    L = _lib.load()
    with torch.cuda.device(b.device):
        stream = _stream(b.device)
        if path == "fused" and not graphs.fused_ok:
            raise ValueError("the fused kernel follows non-ascending adjacency orders only for "
                             "P <= 8; use path='auto' or 'stepwise'")
        fused = path != "stepwise" and graphs.fused_ok
        if fused:
            rc = L.dadmm_forward(ctypes.byref(d), _ptr(op.workspace), _ptr(b), _ptr(graphs.nbr),
                                 _ptr(graphs.order), _ptr(graphs.deg), _ptr(hyp), _ptr(y0),
                                 _ptr(U0), _ptr(d0), _ptr(Y), _ptr(U), _ptr(status), stream)
            if rc == _lib.DADMM_EUNSUPPORTED and path == "auto":
                fused = False
            else:
                _lib.check("dadmm_forward", rc)
        if path != "fused":
            nbytes = L.dadmm_stepwise_scratch_bytes(ctypes.byref(d))
            scratch = torch.empty(max(nbytes, 256), dtype=torch.uint8, device=b.device)
            _lib.check("dadmm_forward_stepwise", L.dadmm_forward_stepwise(
                ctypes.byref(d), _ptr(op.workspace), _ptr(b), _ptr(graphs.vptr), _ptr(graphs.vq),
                _ptr(graphs.deg), _ptr(hyp), _ptr(y0), _ptr(U0), _ptr(d0), _ptr(Y), _ptr(U),
                _ptr(status), 1 if fused else 0, _ptr(scratch), stream))
    if ns != op.n:
        Y = Y[..., : op.n]
        U = U[..., : op.n] if U is not None else None
    return Y, U, status


def describe_status(st: int) -> list:
    """The reference's warnings (unfolded_DLASSO.py:56-104) for the guard bits in ``st``."""
    out = []
    if st & _lib.STATUS_Y_NONFINITE:
        out.append("NaN/Inf detected in y_k, reset to zeros")
    if st & _lib.STATUS_U_NONFINITE:
        out.append("NaN/Inf detected in U_k, reset to zeros")
    if st & _lib.STATUS_GRAD_NAN:
        out.append("NaN/Inf in gradient, update skipped")
    if st & _lib.STATUS_YNEXT_NAN:
        out.append("NaN/Inf in y_next, previous value kept")
    if st & _lib.STATUS_BARRIER_TIMEOUT:
        out.append("stepwise grid barrier timed out: Y is invalid (device shared with other work)")
    return out
