"""CPU tensors: the drop-in modules' K-step recurrence in torch eager ops.

The reference runs on any torch device and defaults to ``--device cpu``
(configurations.py:108). Here CUDA tensors go to the HIP library (``dadmm_hip``; a missing or
broken library raises, it is never replaced by this code), and CPU tensors run this module: the
reference's own op sequence, vectorised over the batch, differentiable by torch autograd.

* ``unfolded_forward`` — ``DLASSO_unfolded.forward``'s loop (unfolded_DLASSO.py:53-107): the Gram
  form A_p^T A_p y_p (:69-71), the gradient ((((AtAy - Atb) + sign(y) tau) + U deg) + delta rho)
  (:73-77), its clamp to +-max(1, 30 - k) (:80-81) and batch-global NaN zeroing (:84-86), the
  primal update and its clamp (:89-93), delta = compute_delta(y_next) (:95), the dual update and
  clamp (:98-99), and the y / U / y_next guards (:55-61, :102-104), in that order.
* ``gnn_step`` — one iteration of ``DLASSO_GNNHyp3_Progressive.forward`` (gnn_dlasso_models_
  progressive.py:197-237): fixed clamps (+-10, +-100, delta +-20, U +-100).
* ``visit_laplacian`` — compute_delta's linear map (unfolded_DLASSO.py:127-140) per sample from
  the ingested visit lists: delta_p = sum over p's visit row of (y_p - y_q), so delta = L y with
  L[p] = |row p| e_p - sum_t e_{q_t}. The visit rows follow the reference's loops (a one-graph
  list of a B-sample batch gives delta to sample 0 only, as the reference's loop over
  len(graph_list) does). delta is formed as a matrix product, so it rounds differently from the
  reference's sequential adds (fp32 rounding, not bit-for-bit).

The returned status word has the HIP path's bits (include/dadmm.h DADMM_STATUS_*): 1 the y_k
guard, 2 the U_k guard, 4 the NaN gradient, 8 the y_next guard.
"""
from __future__ import annotations

import torch

from dadmm_hip import _lib


def visit_laplacian(graphs, P: int, batch_size: int, dtype=torch.float32) -> torch.Tensor:
    """[G, P, P] with G = 1 (one shared graph) or the batch size: delta = L @ y per sample."""
    vptr = graphs.vptr.to("cpu", torch.int64)
    G = 1 if graphs.shared else batch_size
    rows = G * P
    vptr = vptr[:rows + 1]
    counts = vptr[1:] - vptr[:-1]
    total = int(vptr[-1])
    q = graphs.vq.to("cpu", torch.int64)[:total]
    rid = torch.repeat_interleave(torch.arange(rows), counts)
    L = torch.zeros(rows, P, dtype=torch.float64)
    L[torch.arange(rows), torch.arange(rows) % P] = counts.to(torch.float64)
    L.index_put_((rid, q), torch.full((total,), -1.0, dtype=torch.float64), accumulate=True)
    return L.reshape(G, P, P).to(dtype)


def _bad(x: torch.Tensor) -> bool:
    return bool(torch.isnan(x).any() or torch.isinf(x).any())


def _setup(A, bb, graphs, batch_size):
    """AtA [P, n, n] (the reference's self.AtA, :16), Atb [B, P, n, 1] (:45), deg [G, P, 1, 1]
    (:46), the consensus maps [G, P, P]."""
    P = A.shape[1]
    A0 = A[0]
    AtA = torch.matmul(A0.transpose(-1, -2), A0)
    Atb = torch.matmul(A0.transpose(-1, -2)[None], bb[..., None])            # [B, P, n, 1]
    deg = graphs.deg.to("cpu", torch.float32)
    deg = deg.reshape(1 if graphs.shared else -1, P, 1, 1)
    return AtA, Atb, deg, visit_laplacian(graphs, P, batch_size)


def _delta(L, y):
    """compute_delta(y) = L y per sample; y [B, P, n, 1]."""
    B, P = y.shape[:2]
    return torch.matmul(L, y.reshape(B, P, -1)).reshape(y.shape)   # L [1 | B, P, P] broadcasts


def unfolded_forward(A, bb, graphs, table, K, inits):
    """A [1, P, m, n], bb [B, P, m], table [K, H, 4] (seq_hyp rows, differentiable), inits
    (y0, U0, d0) each [B, P, n] -> (Y [K, B, P, n], status int)."""
    B, P = bb.shape[:2]
    AtA, Atb, deg, L = _setup(A, bb, graphs, B)
    y, U, delta = (x.reshape(B, P, -1, 1) for x in inits)
    status = 0
    Y = []
    for k in range(K):
        if _bad(y):                                                  # :55-58
            status |= _lib.STATUS_Y_NONFINITE
            y = torch.zeros_like(y)
        if _bad(U):                                                  # :59-61
            status |= _lib.STATUS_U_NONFINITE
            U = torch.zeros_like(U)
        h = table[k]                                                 # seq_hyp(k): [H, 4]
        alpha, tau, rho, eta = (h[:, c].reshape(1, -1, 1, 1) for c in range(4))
        AtAy = torch.matmul(AtA[None], y)                             # :69-71 (Gram form)
        grad = AtAy - Atb + y.sign() * tau + U * deg + delta * rho   # :73-77
        gmax = max(1.0, 30.0 - k)
        grad = torch.clamp(grad, -gmax, gmax)                        # :80-81
        if _bad(grad):                                               # :84-86
            status |= _lib.STATUS_GRAD_NAN
            grad = torch.zeros_like(grad)
        y_next = y - alpha * grad                                    # :89
        vmax = max(10.0, 200.0 - k * 3)
        y_next = torch.clamp(y_next, -vmax, vmax)                    # :92-93
        delta = _delta(L, y_next)                                    # :95
        U = torch.clamp(U + delta * eta, -vmax, vmax)                # :98-99
        if _bad(y_next):                                             # :102-104
            status |= _lib.STATUS_YNEXT_NAN
            y_next = y
        y = y_next
        Y.append(y)
    return torch.stack(Y)[..., 0], status


def gnn_prepare(A, bb, graphs, batch_size):
    """The loop-invariant operands of the GNN recurrence (AtA, Atb, deg, L)."""
    return _setup(A, bb, graphs, batch_size)


def gnn_step(prep, y, U, delta, AtAy, alpha, tau, rho, eta):
    """One GNN-model iteration after the hypernetwork (gnn_dlasso_models_progressive.py:199-237);
    alpha..eta [B, H, 1, 1] (tau, rho, eta already clamped <= 0.9999, :194-196). Returns
    (y_next, U, delta, status bits)."""
    _, Atb, deg, L = prep
    status = 0
    grad = AtAy - Atb + y.sign() * tau + U * deg + delta * rho       # :205-210
    grad = torch.clamp(grad, -10.0, 10.0)                             # :212-213
    if _bad(grad):                                                    # :216-218
        status |= _lib.STATUS_GRAD_NAN
        grad = torch.zeros_like(grad)
    y_next = torch.clamp(y - alpha * grad, -100.0, 100.0)             # :221-225
    delta = torch.clamp(_delta(L, y_next), -20.0, 20.0)               # :228-229
    U = torch.clamp(U + delta * eta, -100.0, 100.0)                   # :231-232
    if _bad(y_next):                                                  # :235-237
        status |= _lib.STATUS_YNEXT_NAN
        y_next = y
    return y_next, U, delta, status
