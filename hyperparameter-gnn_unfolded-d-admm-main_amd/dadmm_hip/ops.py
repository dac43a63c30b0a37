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


def _sw_flag_bytes(K):
    return 4 * (8 + 4 * K)   # SW_FLAG_WORDS(K) of csrc/dadmm_internal.h


def draw_inits(shape, device, n_store=None, zero=None, nzero=0):
    """(y0, U0, d0) = torch.randn(shape) * 1e-2 x 3 in that order (unfolded_DLASSO.py:49-51),
    bit-identical to torch's own draws, from the device's default generator (advanced exactly as
    the three torch calls would), in ONE launch that also zeroes ``nzero`` int32 words at
    ``zero``. shape = (B, P, n); outputs are [B, P, n_store] (padding columns zero)."""
    B, P, n = shape
    ns = n if n_store is None else n_store
    L = _lib.load()
    alloc = torch.zeros if ns != n else torch.empty
    y0, U0, d0 = (alloc((B, P, ns), dtype=torch.float32, device=device) for _ in range(3))
    numel = B * P * n
    gen = torch.cuda.default_generators[device.index if device.index is not None
                                        else torch.cuda.current_device()]
    seed, off = gen.initial_seed(), gen.get_offset()
    if numel > 0:
        step = L.dadmm_normal_offset_step(numel)
        if step == 0:
            _lib.check("dadmm_normal_offset_step", _lib.DADMM_EHIP)
        gen.set_offset(off + 3 * step)
    with torch.cuda.device(device):
        _lib.check("dadmm_prologue", L.dadmm_prologue(
            seed, off, numel, n, ns, 0.0, 1e-2, _ptr(y0), _ptr(U0), _ptr(d0),
            _ptr(zero), nzero, _stream(device)))
    return y0, U0, d0


def forward_raw(op: PreparedOperator, b: torch.Tensor, graphs: GraphBatch, hyp: torch.Tensor,
                y0: torch.Tensor = None, U0: torch.Tensor = None, d0: torch.Tensor = None, *,
                variant: int = _lib.VARIANT_UNFOLDED, want_U: bool = False, path: str = "auto",
                record: bool = False):
    """The K-step forward with the reference's NaN/Inf guards, enqueued on the current stream
    (no host synchronisation). Shapes: b [B,P,m], hyp [K,H,4], y0/U0/d0 [B,P,n].

    path "auto": the fused kernel when the shape is compiled (its column-split form,
    dadmm_forward_split, for batches that fill at most half the CUs: GEMM1 in the split order,
    ``split_cols``), otherwise the tiled kernel (one launch per iteration); either is followed by
    the device-gated stepwise recomputation (runs only if a guard event was flagged). Training (record) outside the fused shapes: the stepwise
    kernels, or the streamed single launch where it applies (P <= 16, m <= 64). "fused" / "split" / "tiled" / "stepwise" force one path ("fused" / "split" / "tiled"
    alone do NOT apply the guards: their status only flags them).

    record: also store the trajectory the adjoint consumes (training; dadmm_forward_record).

    y0 = U0 = d0 = None: the reference's random inits are drawn by the prologue launch
    (draw_inits; bit-identical to torch.randn * 1e-2 from the device's default generator).

    Returns (Y [K,B,P,n], U_K [B,P,n] or None, status int32 device tensor [1]), plus, with
    ``record``, a ``Trajectory`` as a fourth element."""
    _dev_check(b, hyp, y0, U0, d0, graphs.nbr, graphs.deg)
    draw = y0 is None
    if draw != (U0 is None) or draw != (d0 is None):
        raise ValueError("pass all of y0, U0, d0 or none of them")
    if path not in ("auto", "fused", "split", "tiled", "stepwise"):
        raise ValueError(f"unknown path {path!r}")
    B, P, m = b.shape
    if P != op.P or m != op.m:
        raise ValueError(f"b is [B,{P},{m}], operator is P={op.P}, m={op.m}")
    K, H = int(hyp.shape[0]), int(hyp.shape[1])
    ns = op.n_store
    b = b.contiguous().float()
    hyp = hyp.contiguous().float()
    if not draw:
        y0, U0, d0 = (_pad_n(x, ns).contiguous().float() for x in (y0, U0, d0))
    Y = torch.empty((K, B, P, ns), dtype=torch.float32, device=b.device)
    U = torch.empty((B, P, ns), dtype=torch.float32, device=b.device) if want_U else None
    Grec = Urec = None
    if record:
        Grec = torch.empty((K, B, P, ns), dtype=torch.float32, device=b.device)
        Urec = torch.empty((K, B, P, ns), dtype=torch.float32, device=b.device)
    d = op.dims(B=B, K=K, variant=variant, hyp_rows=H, graph_shared=graphs.shared)
    L = _lib.load()
    if path in ("fused", "split") and not graphs.fused_ok:
        raise ValueError("the fused kernel follows non-ascending adjacency orders only for "
                         "P <= 8; use path='auto' or 'stepwise'")
    # small batches (the fused tiles would fill at most half the CUs): the column-split forward
    split_b = 0
    if path in ("auto", "split") and not record and graphs.fused_ok:
        split_b = L.dadmm_split_scratch_bytes(ctypes.byref(d))
    if path == "split" and split_b == 0:
        raise ValueError(f"the column-split forward does not serve B={B} P={P} n={ns} "
                         "(n_pad 128 or 256, P <= 6, m <= 64, ceil(B/16) <= CUs/2)")
    flag_b = L.dadmm_split_flag_bytes(ctypes.byref(d)) if split_b else 0
    # one device allocation: [status word | 252 B pad | split epoch words | stepwise scratch
    # (guard flags first)]; the prologue zeroes the status word, the epoch words and the guard
    # flags in the same launch as the draws
    gated = path in ("auto", "stepwise")
    nbytes = L.dadmm_stepwise_scratch_bytes(ctypes.byref(d)) if gated else 0
    words = torch.empty(256 + flag_b + max(nbytes, 256), dtype=torch.uint8, device=b.device)
    status = words[:4].view(torch.int32)
    sflags = words[256:256 + flag_b]
    scratch = words[256 + flag_b:]
    nzero = (256 + flag_b + (_sw_flag_bytes(K) if gated else 0)) // 4
    if draw:
        y0, U0, d0 = draw_inits((B, P, op.n), b.device, ns, zero=words, nzero=nzero)
    else:
        with torch.cuda.device(b.device):
            _lib.check("dadmm_prologue", L.dadmm_prologue(
                0, 0, 0, 1, 1, 0.0, 0.0, None, None, None, _ptr(words), nzero, _stream(b.device)))
    with torch.cuda.device(b.device):
        stream = _stream(b.device)
        fused = path in ("auto", "fused", "split") and graphs.fused_ok
        if split_b:
            xbuf = torch.empty(split_b, dtype=torch.uint8, device=b.device)
            _lib.check("dadmm_forward_split", L.dadmm_forward_split(
                ctypes.byref(d), _ptr(op.workspace), _ptr(b), _ptr(graphs.nbr), _ptr(graphs.order),
                _ptr(graphs.deg), _ptr(hyp), _ptr(y0), _ptr(U0), _ptr(d0), _ptr(Y), _ptr(U),
                _ptr(status), _ptr(sflags), _ptr(xbuf), stream))
        elif fused:
            if record:
                rc = L.dadmm_forward_record(
                    ctypes.byref(d), _ptr(op.workspace), _ptr(b), _ptr(graphs.nbr),
                    _ptr(graphs.order), _ptr(graphs.deg), _ptr(hyp), _ptr(y0), _ptr(U0), _ptr(d0),
                    _ptr(Y), _ptr(Grec), _ptr(Urec), _ptr(U), _ptr(status), stream)
            else:
                rc = L.dadmm_forward(ctypes.byref(d), _ptr(op.workspace), _ptr(b),
                                     _ptr(graphs.nbr), _ptr(graphs.order), _ptr(graphs.deg),
                                     _ptr(hyp), _ptr(y0), _ptr(U0), _ptr(d0), _ptr(Y), _ptr(U),
                                     _ptr(status), stream)
            if rc == _lib.DADMM_EUNSUPPORTED and path == "auto":
                fused = False
            else:
                _lib.check("dadmm_forward_record" if record else "dadmm_forward", rc)
        tiled = path == "tiled" or (path == "auto" and not fused and not record)
        if record and not fused and path in ("auto", "tiled"):
            # the streamed single launch records the trajectory (P <= 16, m <= 64); otherwise the
            # stepwise kernels below record it
            tb = L.dadmm_tiled_scratch_bytes(ctypes.byref(d))
            tscratch = torch.empty(max(tb, 256), dtype=torch.uint8, device=b.device)
            rc = L.dadmm_forward_tiled_record(
                ctypes.byref(d), _ptr(op.workspace), _ptr(b), _ptr(graphs.vptr), _ptr(graphs.vq),
                _ptr(graphs.deg), _ptr(hyp), _ptr(y0), _ptr(U0), _ptr(d0), _ptr(Y), _ptr(Grec),
                _ptr(Urec), _ptr(U), _ptr(status), _ptr(tscratch), stream)
            if rc == _lib.DADMM_EUNSUPPORTED and path == "auto":
                tiled = False
            else:
                _lib.check("dadmm_forward_tiled_record", rc)
                tiled = True
        elif tiled:
            tb = L.dadmm_tiled_scratch_bytes(ctypes.byref(d))
            tscratch = torch.empty(max(tb, 256), dtype=torch.uint8, device=b.device)
            rc = L.dadmm_forward_tiled(
                ctypes.byref(d), _ptr(op.workspace), _ptr(b), _ptr(graphs.vptr), _ptr(graphs.vq),
                _ptr(graphs.deg), _ptr(hyp), _ptr(y0), _ptr(U0), _ptr(d0), _ptr(Y), _ptr(U),
                _ptr(status), _ptr(tscratch), stream)
            if rc == _lib.DADMM_EUNSUPPORTED and path == "auto":
                tiled = False
            else:
                _lib.check("dadmm_forward_tiled", rc)
        if gated:
            gate = _lib.FLAGS_ZEROED | (_lib.GATE_ON if (fused or tiled) else 0)
            _lib.check("dadmm_forward_stepwise", L.dadmm_forward_stepwise(
                ctypes.byref(d), _ptr(op.workspace), _ptr(b), _ptr(graphs.vptr), _ptr(graphs.vq),
                _ptr(graphs.deg), _ptr(hyp), _ptr(y0), _ptr(U0), _ptr(d0), _ptr(Y), _ptr(U),
                _ptr(Grec), _ptr(Urec), _ptr(status), gate, _ptr(scratch), stream))
    traj = Trajectory(Y, Grec, Urec, y0, d0, hyp, variant, fused) if record else None
    if ns != op.n:
        Y = Y[..., : op.n]
        U = U[..., : op.n] if U is not None else None
    if record:
        return Y, U, status, traj
    return Y, U, status


def split_cols(op: PreparedOperator, B: int, K: int, graphs: GraphBatch = None, hyp_rows: int = 1,
               record: bool = False) -> int:
    """The GEMM1 slice width forward_raw's "auto" path uses for this batch: 64 when it runs the
    column-split forward (dadmm_forward_split), else 0 (the oracle's ``split_cols`` argument)."""
    if record or (graphs is not None and not graphs.fused_ok):
        return 0
    shared = graphs.shared if graphs is not None else 1
    d = op.dims(B=B, K=K, hyp_rows=hyp_rows, graph_shared=shared)
    return 64 if _lib.load().dadmm_split_scratch_bytes(ctypes.byref(d)) else 0


class Trajectory:
    """What the adjoint consumes: the n-padded iterates Y, pre-clamp gradients Grec and dual
    states Urec ([K,B,P,n_store] each), the inits y0 / d0 and the hyper-parameter table;
    ``fused``: recorded by the fused kernel (its on-chip adjoint applies), else by the stepwise
    path (the general adjoint)."""

    __slots__ = ("Y", "Grec", "Urec", "y0", "d0", "hyp", "variant", "fused")

    def __init__(self, Y, Grec, Urec, y0, d0, hyp, variant, fused=False):
        self.Y, self.Grec, self.Urec = Y, Grec, Urec
        self.y0, self.d0, self.hyp, self.variant, self.fused = y0, d0, hyp, variant, fused


def backward_raw(op: PreparedOperator, graphs: GraphBatch, traj: Trajectory,
                 gY: torch.Tensor, path: str = "auto") -> torch.Tensor:
    """dL/dhyp [K,H,4] for L = sum_k <gY[k], Y[k]> along ``traj``, enqueued on the current
    stream. gY: [K,B,P,n] (n or n_store columns).

    path "auto": the fused adjoint (dadmm_backward: one launch, state on chip) for a fused
    trajectory, otherwise the general adjoint (dadmm_adjoint: any P <= 64, any m, n); "fused" /
    "general" force one."""
    _dev_check(gY)
    if path not in ("auto", "fused", "general"):
        raise ValueError(f"unknown path {path!r}")
    # compute_delta is the sum over its visits (p, q) of (e_p - e_q)(e_p - e_q)^T: symmetric for
    # ANY adjacency, so every adjoint applies it through the forward's own visit order. The fused
    # adjoint's shared-graph consensus (consensus_fma) reads one edge multiplier per unordered
    # pair, i.e. assumes a symmetric adjacency: a directed SHARED graph takes the general adjoint
    # (its visit lists follow the successor lists); per-sample graphs use the direction-aware
    # consensus_lane / consensus_ordered in either adjoint.
    directed_shared = graphs.shared and not getattr(graphs, "symmetric", True)
    K, B, P, ns = traj.Y.shape
    H = int(traj.hyp.shape[1])
    gY = _pad_n(gY.float(), ns).contiguous()
    if tuple(gY.shape) != (K, B, P, ns):
        raise ValueError(f"gY must be [{K},{B},{P},{op.n}], got {tuple(gY.shape)}")
    d = op.dims(B=B, K=K, variant=traj.variant, hyp_rows=H, graph_shared=graphs.shared)
    L = _lib.load()
    dhyp = torch.empty((K, H, 4), dtype=torch.float32, device=gY.device)
    if path == "fused" and directed_shared:
        raise ValueError("the fused adjoint assumes a symmetric shared adjacency; use 'auto' or "
                         "'general' for a directed shared graph")
    use_fused = path == "fused" or (path == "auto" and traj.fused and graphs.fused_ok
                                    and not directed_shared)
    with torch.cuda.device(gY.device):
        stream = _stream(gY.device)
        if use_fused:
            if not graphs.fused_ok:
                raise ValueError("the fused adjoint follows non-ascending adjacency orders only "
                                 "for P <= 8; use path='auto' or 'general'")
            nbytes = L.dadmm_backward_scratch_bytes(ctypes.byref(d))
            scratch = torch.empty(max(nbytes, 16) // 4 + 4, dtype=torch.float32, device=gY.device)
            rc = L.dadmm_backward(ctypes.byref(d), _ptr(op.workspace), _ptr(graphs.nbr),
                                  _ptr(graphs.order), _ptr(graphs.deg), _ptr(traj.hyp),
                                  _ptr(traj.y0), _ptr(traj.d0), _ptr(traj.Y), _ptr(traj.Grec),
                                  _ptr(traj.Urec), _ptr(gY), _ptr(dhyp), _ptr(scratch), stream)
            if rc != _lib.DADMM_EUNSUPPORTED or path == "fused":
                _lib.check("dadmm_backward", rc)
                return dhyp
        nbytes = L.dadmm_adjoint_scratch_bytes(ctypes.byref(d))
        scratch = torch.empty(max(nbytes, 256), dtype=torch.uint8, device=gY.device)
        _lib.check("dadmm_adjoint", L.dadmm_adjoint(
            ctypes.byref(d), _ptr(op.workspace), _ptr(graphs.vptr), _ptr(graphs.vq),
            _ptr(graphs.deg), _ptr(traj.hyp), _ptr(traj.y0), _ptr(traj.d0), _ptr(traj.Y),
            _ptr(traj.Grec), _ptr(traj.Urec), _ptr(gY), _ptr(dhyp), _ptr(scratch), stream))
    return dhyp


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
    if st & _lib.STATUS_RECOMPUTE:
        out.append("fused kernel: asymmetric shared adjacency, batch needs the guarded recomputation")
    if st & _lib.STATUS_BARRIER_TIMEOUT:
        out.append("stepwise grid barrier timed out: Y is invalid (device shared with other work)")
    return out
