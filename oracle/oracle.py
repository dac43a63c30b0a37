"""Python side of the CPU oracle (TEST INFRASTRUCTURE ONLY — see ``oracle/__init__.py``).

Restates, from the reference source text:
  * ``seq_hyperparam.forward``                       unfolded_DLASSO.py:156-168   -> hyp_table()
  * ``DLASSO_unfolded.compute_sum_neighbors``        unfolded_DLASSO.py:111-118   -> graph_arrays()
  * ``DLASSO_unfolded.forward`` + ``compute_delta``  unfolded_DLASSO.py:34-140    -> forward_f32/_f64
    (C: oracle/dadmm_oracle.c), and a vectorised numpy fp64 form (forward_np64) used as an
    independent second restatement
  * the reverse-mode derivative of that forward w.r.t. the hyper-parameter table, as torch autograd
    takes it through the reference's eager ops (clamp/sign/matmul backward rules)   -> backward_np64
  * ``gnn_dlasso_utils.compute_loss``                gnn_dlasso_utils.py:27-88    -> compute_loss()
  * ``gnn_dlasso_utils.set_A`` / ``gnn_data.set_Data`` (input distribution)       -> make_problem()
  * reading the reference's shipped fixtures (A.pt, model.pt) without unpickling  -> load_fixture()
"""
from __future__ import annotations

import ctypes
import os
import zipfile

import numpy as np

__all__ = [
    "lib", "hyp_table", "graph_arrays", "forward_f32", "forward_f64", "forward_np64",
    "forward_f32_rec", "forward_f32_gram", "laplacians", "backward_np64",
    "compute_loss", "make_problem", "load_fixture_tensor", "er_graph", "connected_er_graph",
    "set_threads",
]

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def lib() -> ctypes.CDLL:
    """Load (building if needed, in this container only) ``oracle/liboracle.so``."""
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            import subprocess
            subprocess.run(["make", "-C", _HERE], check=True, capture_output=True)
        L = ctypes.CDLL(path)
        fp = ctypes.c_void_p
        i = ctypes.c_int
        for name in ("oracle_forward_f32", "oracle_forward_f64", "oracle_forward_f32_gram"):
            f = getattr(L, name)
            f.restype = ctypes.c_int
            f.argtypes = [i, i, i, i, i, i, i, i] + [fp] * 12
        L.oracle_forward_f32_rec.restype = ctypes.c_int
        L.oracle_forward_f32_rec.argtypes = [i, i, i, i, i, i, i, i] + [fp] * 14
        L.oracle_forward_f32_split.argtypes = [i, i, i, i, i, i, i, i] + [fp] * 12 + [i]
        L.oracle_abi_version.restype = ctypes.c_int
        L.oracle_set_threads.restype = ctypes.c_int
        L.oracle_set_threads.argtypes = [i]
        _LIB = L
    return _LIB


def set_threads(t: int) -> int:
    """OpenMP threads of the C restatements (CPU-baseline legs); returns the team size now set."""
    return int(lib().oracle_set_threads(int(t)))


# --------------------------------------------------------------------------------------------
def hyp_table(param, max_param, training=False, threshold=0.8, factor=0.95, dtype=np.float32):
    """All K rows of seq_hyperparam(k) (unfolded_DLASSO.py:156-168) -> [K, H, 4].

    hyp_k = clamp(sigmoid(sum_{i<=k} param[i]) * max_param, 1e-4, 0.99); in training mode, if the
    mean of hyp_k over (H, 4) exceeds ``threshold`` the row is multiplied by ``factor`` first.
    """
    param = np.asarray(param, dtype=dtype)
    mx = np.asarray(max_param, dtype=dtype).reshape(1, 4)
    out = []
    for k in range(param.shape[0]):
        s = param[: k + 1].sum(axis=0, dtype=dtype)          # torch.sum(param[:k+1], dim=0)
        h = (1.0 / (1.0 + np.exp(-s))).astype(dtype) * mx     # sigmoid * max_param
        if training and h.sum() / (h.shape[0] * h.shape[1]) > threshold:
            h = h * dtype(factor)
        out.append(np.clip(h, dtype(1e-4), dtype(0.99)))
    return np.stack(out).astype(dtype)


def graph_arrays(graph_list, P):
    """Neighbour lists in adjacency order (CSR) and compute_sum_neighbors degrees.

    Returns (nbr_ptr int32 [B*P+1], nbr_idx int32 [E], deg float32 [B, P]); the lists follow
    ``graph.neighbors(p)`` order, exactly what compute_delta iterates (unfolded_DLASSO.py:136).
    """
    ptr, idx = [0], []
    deg = np.zeros((len(graph_list), P), np.float32)
    for s, G in enumerate(graph_list):
        for p in range(P):
            nb = list(G.neighbors(p))
            deg[s, p] = len(nb)
            idx.extend(nb)
            ptr.append(len(idx))
    return np.asarray(ptr, np.int32), np.asarray(idx if idx else [0], np.int32), deg


def _c(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def _run(fn, out_dt, A, b, graph_list, hyp, y0, U0, d0, variant, hyp_mode, rec=None, tail=()):
    A = _c(A, np.float32).reshape(A.shape[-3:]) if A.ndim == 4 else _c(A, np.float32)
    P, m, n = A.shape
    B = y0.shape[0]
    K = hyp.shape[0]
    H = hyp.shape[-1] if hyp_mode == 1 else hyp.shape[1]
    if isinstance(graph_list, tuple) and len(graph_list) == 3:   # precomputed CSR (goldens)
        nbr_ptr, nbr_idx, deg = (np.ascontiguousarray(v) for v in graph_list)
        nbr_ptr, nbr_idx = nbr_ptr.astype(np.int32), nbr_idx.astype(np.int32)
        deg = deg.astype(np.float32)
    else:
        nbr_ptr, nbr_idx, deg = graph_arrays(graph_list, P)
    b = _c(b, np.float32).reshape(B, P, m)
    y0, U0, d0 = (_c(x, np.float32).reshape(B, P, n) for x in (y0, U0, d0))
    hyp = _c(hyp, np.float32)
    Y = np.empty((K, B, P, n), out_dt)
    U = np.empty((B, P, n), out_dt)
    st = np.zeros(1, np.int32)
    extra = ()
    if rec is not None:
        rec[0] = np.empty((K, B, P, n), out_dt)
        rec[1] = np.empty((K, B, P, n), out_dt)
        extra = (_ptr(rec[0]), _ptr(rec[1]))
    rc = fn(B, P, m, n, K, variant, hyp_mode, H, _ptr(A), _ptr(b), _ptr(nbr_ptr), _ptr(nbr_idx),
            _ptr(deg), _ptr(hyp), _ptr(y0), _ptr(U0), _ptr(d0), _ptr(Y), _ptr(U), _ptr(st), *extra,
            *tail)
    if rc != 0:
        raise RuntimeError(f"oracle returned {rc}")
    return Y, U, int(st[0])


def forward_f32(A, b, graph_list, hyp, y0, U0, d0, variant=0, hyp_mode=0, split_cols=0):
    """Order-matched fp32 restatement (bit-exact target of the HIP kernel).

    ``graph_list``: B networkx graphs, or a (nbr_ptr, nbr_idx, deg) CSR tuple (graph_arrays).
    ``split_cols`` > 0: GEMM1 in the column-split order of the small-batch forward
    (dadmm_split.hip; the split the library chose is ``dadmm_hip.ops.split_cols``).

    Returns (Y [K,B,P,n] float32, U_K [B,P,n] float32, guard status bits)."""
    if split_cols:
        return _run(lib().oracle_forward_f32_split, np.float32, A, b, graph_list, hyp, y0, U0, d0,
                    variant, hyp_mode, tail=(int(split_cols),))
    return _run(lib().oracle_forward_f32, np.float32, A, b, graph_list, hyp, y0, U0, d0, variant,
                hyp_mode)


def forward_f32_rec(A, b, graph_list, hyp, y0, U0, d0, variant=0, hyp_mode=0):
    """forward_f32 that also records the adjoint's trajectory.

    Returns (Y, U_K, status, Grec, Urec): Grec[k] = the gradient of iteration k before its clamp
    (unfolded_DLASSO.py:73-77), Urec[k] = U_k entering iteration k; both [K,B,P,n] float32."""
    rec = [None, None]
    Y, U, st = _run(lib().oracle_forward_f32_rec, np.float32, A, b, graph_list, hyp, y0, U0, d0,
                    variant, hyp_mode, rec)
    return Y, U, st, rec[0], rec[1]


def forward_f32_gram(A, b, graph_list, hyp, y0, U0, d0, variant=1, hyp_mode=1):
    """The GNN model's recurrence (gnn_dlasso_models_progressive.py:148-240) in the exact order of
    the per-iteration HIP path: AtAy and Atb as separate chains, then AtAy - Atb. hyp_mode 1:
    hyp [K][B][4][H] (the hypernetwork output of every iteration)."""
    return _run(lib().oracle_forward_f32_gram, np.float32, A, b, graph_list, hyp, y0, U0, d0,
                variant, hyp_mode)


def forward_f64(A, b, graph_list, hyp, y0, U0, d0, variant=0, hyp_mode=0):
    """The reference's algorithm (Gram form) in double precision. Same return layout, float64."""
    return _run(lib().oracle_forward_f64, np.float64, A, b, graph_list, hyp, y0, U0, d0, variant,
                hyp_mode)


def forward_np64(A, b, graph_list, hyp, y0, U0, d0, variant=0):
    """Independent vectorised fp64 restatement (Gram form, Laplacian as a matrix, no guards).

    delta = 2 (D - Adj) y holds for every nx.Graph (each undirected edge is visited from both
    ends in compute_delta, unfolded_DLASSO.py:132-139)."""
    A = np.asarray(A, np.float64).reshape(np.shape(A)[-3:])
    P, m, n = A.shape
    B = y0.shape[0]
    AtA = np.einsum("pri,prj->pij", A, A)
    Atb = np.einsum("pri,bpr->bpi", A, np.asarray(b, np.float64).reshape(B, P, m))
    L = np.zeros((B, P, P))
    deg = np.zeros((B, P))
    for s, G in enumerate(graph_list):
        for p in range(P):
            for q in G.neighbors(p):
                L[s, p, q] -= 1.0
                deg[s, p] += 1.0
        L[s] += np.diag(deg[s])
    y = np.asarray(y0, np.float64).reshape(B, P, n)
    U = np.asarray(U0, np.float64).reshape(B, P, n)
    d = np.asarray(d0, np.float64).reshape(B, P, n)
    hyp = np.asarray(hyp, np.float64)
    Y = []
    for k in range(hyp.shape[0]):
        al, ta, rh, et = (hyp[k][:, c][None, :, None] for c in range(4))
        gclip = max(1.0, 30.0 - k) if variant == 0 else 10.0
        vclip = max(10.0, 200.0 - 3 * k) if variant == 0 else 100.0
        g = np.einsum("pij,bpj->bpi", AtA, y) - Atb + np.sign(y) * ta + U * deg[:, :, None] + d * rh
        g = np.clip(g, -gclip, gclip)
        yn = np.clip(y - al * g, -vclip, vclip)
        d = 2.0 * np.einsum("bpq,bqi->bpi", L, yn)
        if variant != 0:
            d = np.clip(d, -20.0, 20.0)
        U = np.clip(U + d * et, -vclip, vclip)
        y = yn
        Y.append(y)
    return np.stack(Y), U


def laplacians(graph_list, P):
    """(L [B,P,P] float64, deg [B,P]) with compute_delta(y) = 2 L y and deg = len(neighbors(p))
    (sum_neighbors, unfolded_DLASSO.py:112-118). compute_delta (:127-140) adds, for every visit
    (p, q) with q in neighbors(p), (y_p - y_q) to delta[p] and subtracts it from delta[q]: the map
    is the sum over visits of (e_p - e_q)(e_p - e_q)^T, SYMMETRIC for any adjacency (a directed
    graph's successor lists included; a self-loop contributes nothing). For an undirected graph
    every edge is visited twice and 2 L = 2 (D - Adj)."""
    B = len(graph_list)
    L = np.zeros((B, P, P))
    deg = np.zeros((B, P))
    for s, G in enumerate(graph_list):
        for p in range(P):
            for q in G.neighbors(p):
                deg[s, p] += 1.0
                if q == p:
                    continue
                L[s, p, p] += 0.5
                L[s, q, q] += 0.5
                L[s, p, q] -= 0.5
                L[s, q, p] -= 0.5
    return L, deg


def backward_np64(A, graph_list, hyp, y0, d0, Y, Grec, Urec, gY, variant=0):
    """d(sum_k <gY[k], Y[k]>) / d hyp  ->  [K, H, 4] float64, in reverse mode along a recorded
    trajectory (Y, Grec, Urec as forward_f32_rec / the HIP recording path return them).

    Follows the derivative torch autograd takes through the reference's forward
    (unfolded_DLASSO.py:53-107): sign() has zero derivative; clamp(x, lo, hi) passes the
    gradient where lo <= x <= hi; delta_{k+1} = compute_delta(y_{k+1}) = 2 (D - Adj) y_{k+1} is
    differentiated (its transpose is itself, for any adjacency: ``laplacians``), delta_0 is a
    random leaf; b, y0, U0 carry no
    gradient. Per iteration k (a = alpha_k, ...; g = clamp(gr_k); z = y_k - a g; w = U_k + d_{k+1} e):
        dEta_k   += sum(w_bar d_{k+1})            w_bar = U_bar [|w| <= vclip]
        d_bar    += w_bar e ;  y_bar += 2 L d_bar  (GNN variant: d_bar masked by |2Ly| <= 20)
        z_bar     = y_bar [|z| <= vclip] ;  dAlpha_k += sum(-z_bar g)
        gr_bar    = -a z_bar [|gr| <= gclip]
        dTau_k   += sum(gr_bar sign(y_k)) ;  dRho_k += sum(gr_bar d_k)
        U_bar     = w_bar + deg gr_bar ;  d_bar = rho gr_bar ;  y_bar = z_bar + AtA gr_bar
    z is re-evaluated in the trajectory's dtype (two roundings, as the kernels do); w and the
    consensus in float64, so a float32 trajectory can differ from the kernels' masks only where
    |w| or |2Ly| lies within rounding of its clip bound. Sums run over the batch and n; for
    H = 1 ('same' mode) also over the agents. No guard handling: finite trajectories only.
    """
    A = np.asarray(A, np.float64).reshape(np.shape(A)[-3:])
    P, m, n = A.shape
    K, B = Y.shape[0], Y.shape[1]
    tdt = np.asarray(Y).dtype
    AtA = np.einsum("pri,prj->pij", A, A)
    L, deg = laplacians(graph_list, P)
    hyp = np.asarray(hyp)
    H = hyp.shape[1]
    Yd = np.asarray(Y, np.float64).reshape(K, B, P, n)
    y0d = np.asarray(y0, np.float64).reshape(B, P, n)
    d0d = np.asarray(d0, np.float64).reshape(B, P, n)
    gY = np.asarray(gY, np.float64).reshape(K, B, P, n)
    dh = np.zeros((K, P, 4))
    yb = np.zeros((B, P, n))
    Ub = np.zeros((B, P, n))
    db = np.zeros((B, P, n))

    def cons(x):
        return 2.0 * np.einsum("bpq,bqi->bpi", L, x)

    for k in reversed(range(K)):
        hk = np.broadcast_to(hyp[k], (P, 4))
        al, ta, rh, et = (hk[:, c].astype(np.float64)[None, :, None] for c in range(4))
        gclip = max(1.0, 30.0 - k) if variant == 0 else 10.0
        vclip = max(10.0, 200.0 - 3 * k) if variant == 0 else 100.0
        y1 = Yd[k]
        yk = Yd[k - 1] if k > 0 else y0d
        d1 = cons(y1)
        md1 = None
        if variant != 0:
            md1 = np.abs(d1) <= 20.0
            d1 = np.clip(d1, -20.0, 20.0)
        if k > 0:
            dk = cons(yk)
            if variant != 0:
                dk = np.clip(dk, -20.0, 20.0)
        else:
            dk = d0d
        yb = yb + gY[k]
        w = np.asarray(Urec[k], np.float64) + d1 * et
        wb = Ub * (np.abs(w) <= vclip)
        dh[k, :, 3] += (wb * d1).sum(axis=(0, 2))
        d1b = db + wb * et
        if md1 is not None:
            d1b = d1b * md1
        yb = yb + cons(d1b)
        gr = np.asarray(Grec[k], np.float64)
        g = np.clip(gr, -gclip, gclip)
        z = (np.asarray(yk, tdt) - hk[:, 0].astype(tdt)[None, :, None] * g.astype(tdt)).astype(np.float64)
        zb = yb * (np.abs(z) <= vclip)
        dh[k, :, 0] += (-zb * g).sum(axis=(0, 2))
        grb = -al * zb * (np.abs(gr) <= gclip)
        dh[k, :, 1] += (grb * np.sign(yk)).sum(axis=(0, 2))
        dh[k, :, 2] += (grb * dk).sum(axis=(0, 2))
        Ub = wb + grb * deg[:, :, None]
        db = grb * rh
        yb = zb + np.einsum("pij,bpj->bpi", AtA, grb)
    if H == 1:
        dh = dh.sum(axis=1, keepdims=True)
    return dh


def compute_loss(Y, label):
    """gnn_dlasso_utils.compute_loss (:27-88) in float64: (mean_k loss_k + 1e-8, loss_{K-1} + 1e-8)
    with loss_k = mean_p mean_{b,n} (Y[k,b,p,n] - label[b,n])^2, and (1, 1) on any NaN/Inf."""
    Y = np.asarray(Y, np.float64)
    K, B, P, n = Y.shape[:4]
    Y = Y.reshape(K, B, P, n)
    label = np.asarray(label, np.float64).reshape(B, n)
    if not np.isfinite(Y).all() or not np.isfinite(label).all():
        return 1.0, 1.0
    losses = ((Y - label[None, :, None, :]) ** 2).mean(axis=(1, 3)).mean(axis=1)
    if not np.isfinite(losses).all():
        return 1.0, 1.0
    return float(losses.mean() + 1e-8), float(losses[-1] + 1e-8)


# --------------------------------------------------------------------------------------------
def er_graph(P, prob, seed):
    """nx.erdos_renyi_graph(P, prob, seed) (unfolded_train_new.py:56)."""
    import networkx as nx
    return nx.erdos_renyi_graph(P, prob, seed=seed)


def connected_er_graph(P, prob, seed):
    """The per-sample graph of gnn_dlasso_progressive.py:181-191 (ER with max(prob, 0.3), then
    components chained by one edge each)."""
    import networkx as nx
    G = nx.erdos_renyi_graph(P, max(prob, 0.3), seed=seed)
    if not nx.is_connected(G):
        comps = list(nx.connected_components(G))
        for i in range(len(comps) - 1):
            G.add_edge(list(comps[i])[0], list(comps[i + 1])[0])
    return G


def make_problem(P, m, n, B, seed=1234):
    """Synthetic inputs with the reference's distribution (gnn_dlasso_utils.py:4-16,
    gnn_data.py:6-15): per-agent A_p = U clamp(S, 0.1, 10) V^T of a Gaussian, x* = 2 N(0,1) *
    Bernoulli(0.25), b_p = A_p x* (noise-free: the noisy b is overwritten, gnn_data.py:13-14).
    Returns float32 arrays A [P,m,n], b [B,P,m], x [B,n]."""
    import torch
    g = torch.Generator().manual_seed(seed)
    A = torch.zeros(P, m, n)
    for p in range(P):
        T = torch.randn(m, n, generator=g)
        Us, S, V = torch.svd(T)
        A[p] = Us @ torch.diag(S.clamp(0.1, 10.0)) @ V.T
    x = 2 * torch.randn(B, n, generator=g) * (torch.rand(B, n, generator=g) <= 0.25)
    b = torch.einsum("pmn,bn->bpm", A, x)
    return A.numpy(), b.numpy(), x.numpy()


def load_fixture_tensor(path):
    """Read the single fp32 storage of a shipped reference ``.pt`` (A.pt / model.pt) as a flat
    float32 array, by reading the zip member ``*/data/0`` — nothing is unpickled."""
    with zipfile.ZipFile(path) as z:
        names = [x for x in z.namelist() if x.endswith("/data/0")]
        if len(names) != 1:
            raise ValueError(f"{path}: expected one storage, found {names}")
        return np.frombuffer(z.read(names[0]), dtype="<f4").copy()
