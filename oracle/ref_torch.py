"""Literal torch restatement of the reference forward (TEST INFRASTRUCTURE ONLY).

Replays the reference's exact op sequence with torch eager ops on the CPU — compute_Atx via
per-agent ``torch.matmul(A[0,p].T, x[:,p])`` (unfolded_DLASSO.py:120-124), the Gram matrix AtA
(:16), the per-agent ``AtA[0,p] @ y[:,p]`` GEMVs (:69-71), the gradient/clamp/update expressions
(:73-99), the Python edge loop of compute_delta (:127-140) and the guards (:55-61, :84-86,
:102-104) — so, with the same torch build, it computes what the reference's own fp32 CPU forward
computes. It is the "reference-form fp32" control for the tolerance tests and the CPU-baseline
leg that reproduces the reference's cost profile. It never imports the reference.
"""
from __future__ import annotations

import numpy as np
import torch


def _atx(A, x):
    # compute_Atx: [B,P,n,c] = A_p^T x_p, one matmul per agent
    P, n = A.shape[1], A.shape[3]
    out = torch.zeros((x.shape[0], P, n, x.shape[3]), dtype=x.dtype)
    for p in range(P):
        out[:, p] = torch.matmul(A[0, p].T, x[:, p])
    return out


def _delta(graph_list, y, P):
    d = torch.zeros_like(y)
    for s in range(len(graph_list)):
        G = graph_list[s]
        for p in range(P):
            yp = y[s, p]
            for q in G.neighbors(p):
                diff = yp - y[s, q]
                d[s, p] += diff
                d[s, q] -= diff
    return d


def forward(A, b, graph_list, hyp, y0, U0, d0, variant=0, dtype=torch.float32):
    """A [P,m,n] or [1,P,m,n]; b [B,P,m]; hyp [K,H,4] (rows of seq_hyp); y0/U0/d0 [B,P,n].

    Returns Y [K,B,P,n] as numpy (dtype of the computation)."""
    A = torch.as_tensor(np.asarray(A), dtype=dtype)
    if A.dim() == 3:
        A = A[None]
    _, P, m, n = A.shape
    B = y0.shape[0]
    b = torch.as_tensor(np.asarray(b), dtype=dtype).reshape(B, P, m, 1)
    hyp = torch.as_tensor(np.asarray(hyp), dtype=dtype)
    AtA = torch.zeros((1, P, n, n), dtype=dtype)
    for p in range(P):
        AtA[0, p] = torch.matmul(A[0, p].T, A[0, p])
    Atb = _atx(A, b)
    deg = torch.zeros((B, P, 1, 1), dtype=dtype)
    for s in range(B):
        for p in range(P):
            deg[s, p] = len(list(graph_list[s].neighbors(p)))
    y = torch.as_tensor(np.asarray(y0), dtype=dtype).reshape(B, P, n, 1).clone()
    U = torch.as_tensor(np.asarray(U0), dtype=dtype).reshape(B, P, n, 1).clone()
    d = torch.as_tensor(np.asarray(d0), dtype=dtype).reshape(B, P, n, 1).clone()
    Y = []
    for k in range(hyp.shape[0]):
        if torch.isnan(y).any() or torch.isinf(y).any():
            y = torch.zeros_like(y)
        if torch.isnan(U).any() or torch.isinf(U).any():
            U = torch.zeros_like(U)
        h = hyp[k]
        al, ta, rh, et = (h[:, c].reshape(1, -1, 1, 1) for c in range(4))
        AtAy = torch.zeros((B, P, n, 1), dtype=dtype)
        for p in range(P):
            AtAy[:, p] = torch.matmul(AtA[0, p], y[:, p])
        grad = AtAy - Atb + y.sign() * ta + U * deg + d * rh
        gclip = max(1.0, 30.0 - k) if variant == 0 else 10.0
        vclip = max(10.0, 200.0 - k * 3) if variant == 0 else 100.0
        grad = torch.clamp(grad, -gclip, gclip)
        if torch.isnan(grad).any() or torch.isinf(grad).any():
            grad = torch.zeros_like(grad)
        yn = torch.clamp(y - al * grad, -vclip, vclip)
        d = _delta(graph_list, yn, P)
        if variant != 0:
            d = torch.clamp(d, -20.0, 20.0)
        U = torch.clamp(U + d * et, -vclip, vclip)
        if torch.isnan(yn).any() or torch.isinf(yn).any():
            yn = y
        y = yn
        Y.append(y)
    return torch.stack(Y)[..., 0].numpy()


def forward_vectorized(A, b, graph_list, hyp, y0, U0, d0, variant=0, dtype=torch.float32):
    """The reference forward vectorised for the CPU (SURVEY.md §7 item 1, §8(d) CPU baseline (i)):
    the same algorithm as ``forward`` — Gram form AtA @ y (unfolded_DLASSO.py:16, :69-71), the
    guards, the clamps — with the P per-agent GEMVs as one batched matmul and compute_delta's
    edge loop (:127-140) as the Laplacian product delta = 2 (D - Adj) y (one bmm per forward
    iteration). fp32 results differ from the loop form only by summation order. Timing leg of the
    CPU baseline; never the product path."""
    A = torch.as_tensor(np.asarray(A), dtype=dtype)
    if A.dim() == 4:
        A = A[0]
    P, m, n = A.shape
    B = y0.shape[0]
    b = torch.as_tensor(np.asarray(b), dtype=dtype).reshape(B, P, m)
    hyp = torch.as_tensor(np.asarray(hyp), dtype=dtype)
    AtA = torch.matmul(A.transpose(1, 2), A)                       # [P, n, n]
    Atb = torch.einsum("pmn,bpm->bpn", A, b)                       # [B, P, n]
    adj = np.zeros((len(graph_list), P, P), np.float32)
    for s, G in enumerate(graph_list):
        for p in range(P):
            for q in G.neighbors(p):
                adj[s, p, q] += 1.0
    adj = torch.from_numpy(adj).to(dtype)
    deg = adj.sum(-1, keepdim=True)                                # [G, P, 1]
    lap2 = 2.0 * (torch.diag_embed(deg[..., 0]) - adj)             # 2 L, [G, P, P]
    y = torch.as_tensor(np.asarray(y0), dtype=dtype).reshape(B, P, n).clone()
    U = torch.as_tensor(np.asarray(U0), dtype=dtype).reshape(B, P, n).clone()
    d = torch.as_tensor(np.asarray(d0), dtype=dtype).reshape(B, P, n).clone()
    Y = torch.empty((hyp.shape[0], B, P, n), dtype=dtype)
    for k in range(hyp.shape[0]):
        if not torch.isfinite(y).all():
            y = torch.zeros_like(y)
        if not torch.isfinite(U).all():
            U = torch.zeros_like(U)
        h = hyp[k]
        al, ta, rh, et = (h[:, c].reshape(1, -1, 1) for c in range(4))
        AtAy = torch.bmm(AtA, y.permute(1, 2, 0)).permute(2, 0, 1)  # [B, P, n]
        grad = AtAy - Atb + y.sign() * ta + U * deg + d * rh
        gclip = max(1.0, 30.0 - k) if variant == 0 else 10.0
        vclip = max(10.0, 200.0 - k * 3) if variant == 0 else 100.0
        grad = torch.clamp(grad, -gclip, gclip)
        if not torch.isfinite(grad).all():
            grad = torch.zeros_like(grad)
        yn = torch.clamp(y - al * grad, -vclip, vclip)
        d = torch.matmul(lap2, yn)
        if variant != 0:
            d = torch.clamp(d, -20.0, 20.0)
        U = torch.clamp(U + d * et, -vclip, vclip)
        if not torch.isfinite(yn).all():
            yn = y
        y = yn
        Y[k] = y
    return Y.numpy()


def forward_autograd(A, b, graph_list, hyp, y0, U0, d0, variant=0, dtype=torch.float64):
    """The same op sequence as ``forward`` (no guards: finite inputs only) on torch tensors that keep
    the autograd graph, so ``torch.autograd.grad`` takes exactly the derivative the reference's
    ``loss.backward()`` takes (unfolded_train_new.py:78). ``hyp`` [K,H,4] is a
    tensor (may require grad). Returns (Y [K,B,P,n], Grec [K,B,P,n] pre-clamp gradients,
    Urec [K,B,P,n] U_k entering iteration k, U_K); Grec/Urec/U_K are detached."""
    A = torch.as_tensor(np.asarray(A), dtype=dtype)
    if A.dim() == 3:
        A = A[None]
    _, P, m, n = A.shape
    B = y0.shape[0]
    b = torch.as_tensor(np.asarray(b), dtype=dtype).reshape(B, P, m, 1)
    AtA = torch.stack([A[0, p].T @ A[0, p] for p in range(P)])[None]
    Atb = _atx(A, b)
    deg = torch.zeros((B, P, 1, 1), dtype=dtype)
    for s in range(B):
        for p in range(P):
            deg[s, p] = len(list(graph_list[s].neighbors(p)))
    y = torch.as_tensor(np.asarray(y0), dtype=dtype).reshape(B, P, n, 1)
    U = torch.as_tensor(np.asarray(U0), dtype=dtype).reshape(B, P, n, 1)
    d = torch.as_tensor(np.asarray(d0), dtype=dtype).reshape(B, P, n, 1)
    Y, G, Ur = [], [], []
    for k in range(hyp.shape[0]):
        h = hyp[k]
        al, ta, rh, et = (h[:, c].reshape(1, -1, 1, 1) for c in range(4))
        AtAy = torch.stack([AtA[0, p] @ y[:, p] for p in range(P)], dim=1)
        grad = AtAy - Atb + y.sign() * ta + U * deg + d * rh
        G.append(grad.detach())
        Ur.append(U.detach())
        gclip = max(1.0, 30.0 - k) if variant == 0 else 10.0
        vclip = max(10.0, 200.0 - k * 3) if variant == 0 else 100.0
        grad = torch.clamp(grad, -gclip, gclip)
        yn = torch.clamp(y - al * grad, -vclip, vclip)
        d = _delta_autograd(graph_list, yn, P)
        if variant != 0:
            d = torch.clamp(d, -20.0, 20.0)
        U = torch.clamp(U + d * et, -vclip, vclip)
        y = yn
        Y.append(y)
    sq = lambda L: torch.stack(L)[..., 0]
    return sq(Y), sq(G), sq(Ur), U.detach()[..., 0]


def _delta_autograd(graph_list, y, P):
    # compute_delta's edge loop (unfolded_DLASSO.py:127-140) without in-place writes, so autograd
    # can run through it: same terms, same per-agent accumulation order
    B = len(graph_list)
    rows = []
    for s in range(B):
        G = graph_list[s]
        acc = [torch.zeros_like(y[s, 0]) for _ in range(P)]
        for p in range(P):
            for q in G.neighbors(p):
                diff = y[s, p] - y[s, q]
                acc[p] = acc[p] + diff
                acc[q] = acc[q] - diff
        rows.append(torch.stack(acc))
    return torch.stack(rows)


def gnn_forward_autograd(model, A, b, graph_list, y0, U0, d0, K, a_hat, dtype=torch.float64):
    """DLASSO_GNNHyp3_Progressive.forward's loop (gnn_dlasso_models_progressive.py:148-240) in
    torch eager ops on the CPU, keeping the autograd graph (no guards: finite inputs only).
    ``model`` supplies the hypernetwork (its ``hypernetwork(AtAy, Atb, a_hat)``), already in
    ``dtype`` on the CPU. Returns (Y [K,B,P,n], (alpha, tau, rho, eta) of the last iteration)."""
    A = torch.as_tensor(np.asarray(A), dtype=dtype)
    if A.dim() == 3:
        A = A[None]
    _, P, m, n = A.shape
    B = y0.shape[0]
    b = torch.as_tensor(np.asarray(b), dtype=dtype).reshape(B, P, m, 1)
    AtA = torch.stack([A[0, p].T @ A[0, p] for p in range(P)])[None]
    Atb = _atx(A, b)
    deg = torch.zeros((B, P, 1, 1), dtype=dtype)
    for s in range(B):
        for p in range(P):
            deg[s, p] = len(list(graph_list[s].neighbors(p)))
    y = torch.as_tensor(np.asarray(y0), dtype=dtype).reshape(B, P, n, 1)
    U = torch.as_tensor(np.asarray(U0), dtype=dtype).reshape(B, P, n, 1)
    d = torch.as_tensor(np.asarray(d0), dtype=dtype).reshape(B, P, n, 1)
    Y = []
    for k in range(K):
        AtAy = torch.stack([AtA[0, p] @ y[:, p] for p in range(P)], dim=1)
        al, ta, rh, et = model.hypernetwork(AtAy[..., 0], Atb[..., 0], a_hat)
        grad = AtAy - Atb + y.sign() * ta + U * deg + d * rh
        grad = torch.clamp(grad, -10.0, 10.0)
        yn = torch.clamp(y - al * grad, -100.0, 100.0)
        d = torch.clamp(_delta_autograd(graph_list, yn, P), -20.0, 20.0)
        U = torch.clamp(U + d * et, -100.0, 100.0)
        y = yn
        Y.append(y)
    return torch.stack(Y)[..., 0], (al, ta, rh, et)
