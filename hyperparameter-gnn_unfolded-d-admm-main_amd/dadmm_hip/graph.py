"""Graph ingestion: ``graph_list`` (networkx graphs) -> the device layouts the kernels read.

Replaces the Python loops of ``compute_sum_neighbors`` (unfolded_DLASSO.py:111-118) and the graph
walk of ``compute_delta`` (:127-140) with (include/dadmm.h):
  * fused kernel: ``nbr[s][p]`` bit q set <=> q in graph_list[s].neighbors(p) and, for adjacency
    lists that are not ascending, ``order`` (the adjacency order packed 4 bits per neighbour,
    P <= 8);
  * stepwise kernel: visit lists ``vptr``/``vq`` — for each agent p the neighbour ids in the
    order compute_delta accumulates delta[p] (its own ``neighbors(p)`` loop between the visits
    of lower and higher agents), any P <= MAX_P;
  * both: ``deg[s][p] = len(neighbors(p))``.

More than 64 agents (up to MAX_P = 255, the visit lists' uint8 ids) have no neighbour masks: the
batch is described by its degrees and visit lists (a CSR form of the adjacency in the reference's
accumulation order) plus a dense 0/1 adjacency ``adj`` [G, P, P] for the GNN model's GCN
normalisation, and takes the non-fused kernels (the fused ones serve P <= 6).

compute_delta sums each agent's own neighbour terms in ``graph.neighbors(p)`` order. For the
graphs the reference builds with ``erdos_renyi_graph`` that order is ascending (edges are added in
lexicographic order) and the masks alone describe it. Graphs whose adjacency lists are not
ascending (e.g. the connectivity patch of gnn_dlasso_progressive.py:184-191 appends edges) carry
``order`` (P <= 8) / their visit lists (any P), so the kernels accumulate in exactly the
reference's order.

Quirks of the reference kept on purpose (it never checks ``len(graph_list) == len(b)``):
  * ``compute_sum_neighbors`` sizes its output by ``len(graph_list)`` and the result broadcasts
    against the state, so one graph for a batch of B gives every sample that graph's degrees;
  * ``compute_delta`` only walks ``range(len(graph_list))``: samples past it get delta = 0.
"""
from __future__ import annotations

import gc
import itertools
import operator

import numpy as np
import torch

_SHARED_CACHE: dict = {}
_INFO_CACHE: dict = {}
MASK_P = 64    # agents the uint64 neighbour masks describe (the fused kernels' layout)
MAX_P = 255    # agents the uint8 visit-list ids describe (every other kernel)


def _info(g, P: int) -> "_GraphInfo":
    """_GraphInfo of graph ``g``, memoised on its current adjacency (graphs are mutable: the key
    is the adjacency itself, never the object's identity)."""
    adj = tuple(tuple(g.neighbors(p)) for p in range(P))
    key = (P, adj)
    hit = _INFO_CACHE.get(key)
    if hit is None:
        hit = _GraphInfo(adj, P)
        if len(_INFO_CACHE) > 65536:
            _INFO_CACHE.clear()
        _INFO_CACHE[key] = hit
    return hit


class _GraphInfo:
    """Host arrays of one graph on agents 0..P-1."""

    __slots__ = ("mask", "deg", "order", "ascending", "vcnt", "vq", "adj")

    def __init__(self, adj, P: int):
        wide = P > MASK_P
        self.adj = adj
        self.mask = np.zeros(P, np.uint64)     # (all zero for P > MASK_P: no mask layout)
        self.deg = np.zeros(P, np.float32)
        self.order = np.zeros(P, np.uint32)
        self.ascending = True
        for p, nb in enumerate(adj):
            self.deg[p] = len(nb)
            for t, q in enumerate(nb):
                if not (0 <= q < P):
                    raise ValueError(f"neighbour id {q} of agent {p}: must be an agent 0..{P - 1}")
                if not wide:
                    self.mask[p] |= np.uint64(1) << np.uint64(q)
                if t < 8:
                    self.order[p] |= np.uint32(q & 15) << np.uint32(4 * t)
            self.ascending &= all(nb[i] < nb[i + 1] for i in range(len(nb) - 1))
        self.vcnt, self.vq = _visit_lists(adj, P)


def _visit_lists(adj, P: int):
    """Per agent p, the ids q whose term (y_p - y_q) compute_delta (unfolded_DLASSO.py:127-140)
    adds to delta[p], in order: the outer loop over p' visits p' < p (p in neighbors(p'): -=),
    then p itself (its neighbours in adjacency order: +=), then p' > p. A -= of fl(y_p' - y_p)
    equals a += of fl(y_p - y_p') exactly, so every entry is one ``acc + (y_p - y_q)``; a
    self-loop contributes its += and -= as two entries q = p."""
    into = [[] for _ in range(P)]          # into[p] = [p' ...] with p in neighbors(p'), by p'
    for pp, nb in enumerate(adj):
        for q in nb:
            if q != pp:
                into[q].append(pp)
    cnt = np.zeros(P, np.int32)
    flat = []
    for p in range(P):
        lst = [pp for pp in into[p] if pp < p]
        for q in adj[p]:
            lst.extend((q, q) if q == p else (q,))
        lst.extend(pp for pp in into[p] if pp > p)
        cnt[p] = len(lst)
        flat.extend(lst)
    return cnt, np.asarray(flat, np.uint8)


class GraphBatch:
    """Device-resident graph layouts for one forward call."""

    __slots__ = ("nbr", "deg", "shared", "order", "vptr", "vq", "fused_ok", "symmetric", "adj")

    def __init__(self, nbr, deg, shared, order, vptr, vq, fused_ok=True, symmetric=True, adj=None):
        self.nbr = nbr      # int64 (uint64 bit patterns) [P] if shared else [B, P]
        self.deg = deg      # float32 [P] if shared else [B, P]
        self.shared = shared
        self.order = order  # int32 [B, P] packed adjacency order, or None (ascending / shared)
        self.vptr = vptr    # int32 [P+1] if shared else [B*P+1]
        self.vq = vq        # uint8 visit lists
        # False when the fused kernel cannot follow the adjacency order (non-ascending lists with
        # P > 8): such batches take the stepwise path, which follows any order
        self.fused_ok = fused_ok
        # every graph undirected (p in N(q) <=> q in N(p)), as the reference's Erdos-Renyi graphs
        # are. compute_delta is symmetric for any adjacency, but the fused kernels' shared-graph
        # consensus (consensus_fma) reads one multiplier per unordered pair: a directed shared
        # graph takes the exact recomputation (forward) and the general adjoint (backward)
        self.symmetric = symmetric
        # P > MASK_P: dense 0/1 adjacency uint8 [1 if shared else B, P, P] (nbr is all zero)
        self.adj = adj

    @property
    def wide(self) -> bool:
        """More agents than the neighbour masks describe (no fused kernels)."""
        return self.adj is not None


def _symmetric(masks) -> bool:
    """Whether the uint64 neighbour masks [..., P] describe undirected graphs."""
    m = np.asarray(masks, np.uint64)
    P = m.shape[-1]
    bits = (m[..., :, None] >> np.arange(P, dtype=np.uint64)) & np.uint64(1)   # [..., p, q]
    return bool(np.array_equal(bits, np.swapaxes(bits, -1, -2)))


def _to_device(arrays, device):
    ts = [torch.from_numpy(np.ascontiguousarray(a)) for a in arrays]
    if torch.device(device).type == "cuda":
        ts = [t.pin_memory() for t in ts]
    return [t.to(device, non_blocking=True) for t in ts]


VQ_TAIL = 4   # zero bytes after the visit lists: kernels that read them as 32-bit words stay in bounds


def _vq_nonempty(vq):
    """The visit lists plus VQ_TAIL zero bytes (never empty: the ABI wants a valid pointer)."""
    return np.concatenate([vq, np.zeros(VQ_TAIL, np.uint8)])


def _batch(infos, P: int, device) -> GraphBatch:
    """Per-sample layouts from one _GraphInfo (or None: no edges) per sample."""
    B = len(infos)
    nbr = np.zeros((B, P), np.uint64)
    deg = np.zeros((B, P), np.float32)
    ordered = any(i is not None and not i.ascending for i in infos)
    fused_ok = not (ordered and P > 8)
    ordered &= fused_ok
    order = np.zeros((B, P), np.uint32) if ordered else None
    vcnt = np.zeros((B, P), np.int32)
    vqs = []
    for s, i in enumerate(infos):
        if i is None:
            continue
        nbr[s], deg[s] = i.mask, i.deg
        if ordered:
            order[s] = i.order
        vcnt[s] = i.vcnt
        vqs.append(i.vq)
    vptr = np.zeros(B * P + 1, np.int32)
    np.cumsum(vcnt.reshape(-1), out=vptr[1:])
    vq = _vq_nonempty(np.concatenate(vqs) if vqs else np.zeros(0, np.uint8))
    arrays = [nbr.view(np.int64), deg, vptr, vq] + ([order.view(np.int32)] if ordered else [])
    t = _to_device(arrays, device)
    return GraphBatch(t[0], t[1], False, t[4] if ordered else None, t[2], t[3], fused_ok, _symmetric(nbr))


def _adjacency(g, P: int):
    """graph.neighbors(p) for p = 0..P-1, as lists (networkx's adjacency dict when present)."""
    adj = getattr(g, "_adj", None)
    if adj is not None:
        return [list(adj[p]) for p in range(P)]
    return [list(g.neighbors(p)) for p in range(P)]


def _batch_vectorized(graph_list, P: int, device) -> GraphBatch:
    """Per-sample layouts for many distinct graphs: one Python pass collects the adjacency lists,
    everything else (masks, degrees, order nibbles, the reference-order visit lists) is numpy over
    the flattened (sample, agent, position) entries — the replacement for the per-sample,
    per-agent loops of compute_sum_neighbors / compute_delta at B in the thousands."""
    B = len(graph_list)
    gc_on = gc.isenabled()
    gc.disable()          # B*P short-lived lists would trigger full cyclic-GC passes
    try:
        lists = [nb for g in graph_list for nb in _adjacency(g, P)]      # B*P lists
    finally:
        if gc_on:
            gc.enable()
    cnt = np.fromiter((len(nb) for nb in lists), np.int64, count=B * P)
    q = np.fromiter(itertools.chain.from_iterable(lists), np.int64, count=int(cnt.sum()))
    if q.size and (q.min() < 0 or q.max() >= P):
        bad = q[(q < 0) | (q >= P)][0]
        raise ValueError(f"neighbour id {bad}: must be an agent 0..{P - 1}")
    row = np.repeat(np.arange(B * P), cnt)                 # (s, a) flattened
    start = np.zeros(B * P + 1, np.int64)
    np.cumsum(cnt, out=start[1:])
    t = np.arange(q.size) - start[row]                     # position in the adjacency list
    s_, a_ = row // P, row % P
    nbr = np.zeros(B * P, np.uint64)
    np.add.at(nbr, row, np.left_shift(np.uint64(1), q.astype(np.uint64)))   # unique per (s,a)
    deg = cnt.reshape(B, P).astype(np.float32)
    # ascending adjacency? (erdos_renyi_graph lists are; appended edges break it)
    desc = (t[1:] > 0) & (q[1:] < q[:-1]) if q.size > 1 else np.zeros(0, bool)
    ordered = bool(desc.any())
    fused_ok = not (ordered and P > 8)
    ordered &= fused_ok
    order = None
    if ordered:
        order = np.zeros(B * P, np.uint32)
        keep = t < 8
        np.add.at(order, row[keep], (q[keep] & 15).astype(np.uint32) << (4 * t[keep]).astype(np.uint32))
    # visit lists (see _visit_lists): for agent p of sample s, entries in the order compute_delta
    # accumulates them. For an undirected graph "p in N(p')" <=> "p' in N(p)", so they are
    #   N(p) n [0, p) ascending | N(p) in adjacency order (a self-loop twice) | N(p) n (p, P) ascending
    # and are placed without sorting: nonzero() of the dense neighbour matrix is row-major.
    dense = np.zeros((B * P, P), bool)
    dense[row, q] = True
    if not np.array_equal(dense.reshape(B, P, P), dense.reshape(B, P, P).transpose(0, 2, 1)):
        return None                                  # not symmetric: caller takes the exact path
    col = np.arange(P)
    below = dense & (col[None, :] < (np.arange(B * P) % P)[:, None])
    above = dense & (col[None, :] > (np.arange(B * P) % P)[:, None])
    loop = q == a_
    c0, c2 = below.sum(1), above.sum(1)
    c1 = cnt + np.bincount(row[loop], minlength=B * P)
    vptr = np.zeros(B * P + 1, np.int64)
    np.cumsum(c0 + c1 + c2, out=vptr[1:])
    vq = np.empty(int(vptr[-1]), np.uint8)
    r0, q0 = np.nonzero(below)
    vq[vptr[r0] + (np.arange(r0.size) - np.repeat(np.cumsum(c0) - c0, c0))] = q0
    # own lists: position t, shifted by the self-loop duplicates earlier in the same list
    before = np.cumsum(loop) - loop                 # self-loops strictly before each entry
    pos1 = vptr[row] + c0[row] + t + (before - before[start[row]]) if q.size else row
    vq[pos1] = q
    vq[pos1[loop] + 1] = q[loop]
    r2, q2 = np.nonzero(above)
    vq[vptr[r2] + c0[r2] + c1[r2] + (np.arange(r2.size) - np.repeat(np.cumsum(c2) - c2, c2))] = q2
    vptr = vptr.astype(np.int32)
    arrays = [nbr.view(np.int64).reshape(B, P), deg, vptr, _vq_nonempty(vq)]
    if ordered:
        arrays.append(order.view(np.int32).reshape(B, P))
    t_ = _to_device(arrays, device)
    return GraphBatch(t_[0], t_[1], False, t_[4] if ordered else None, t_[2], t_[3], fused_ok)


def _native():
    """dadmm_hip._ingest (csrc/dadmm_ingest.c), or None when the extension is not built."""
    global _NATIVE
    if _NATIVE is False:
        try:
            from . import _ingest
            _NATIVE = _ingest
        except ImportError:
            _NATIVE = None
    return _NATIVE


_NATIVE = False


def _batch_native(graph_list, P: int, device):
    """Per-sample layouts for a list of networkx graphs in one C pass over their adjacency dicts
    (dadmm_hip._ingest.batch: masks, degrees, order nibbles, reference-order visit lists; any
    adjacency, directed included). None when the extension is missing or a graph is not a
    dict-of-dicts networkx graph (the caller takes the Python path)."""
    mod = _native()
    if mod is None:
        return None
    try:
        nbr, deg, order, vptr, vq, ascending, symmetric = mod.batch(graph_list, P)
    except TypeError:
        return None
    B = len(graph_list)
    ordered = not ascending
    fused_ok = not (ordered and P > 8)
    ordered &= fused_ok
    arrays = [np.frombuffer(nbr, np.int64).reshape(B, P), np.frombuffer(deg, np.float32).reshape(B, P),
              np.frombuffer(vptr, np.int32), _vq_nonempty(np.frombuffer(vq, np.uint8))]
    if ordered:
        arrays.append(np.frombuffer(order, np.int32).reshape(B, P))
    t_ = _to_device(arrays, device)
    return GraphBatch(t_[0], t_[1], False, t_[4] if ordered else None, t_[2], t_[3], fused_ok,
                      bool(symmetric))


def _batch_wide(graph_list, P: int, batch_size: int, device) -> GraphBatch:
    """P > MASK_P agents: degrees, reference-order visit lists and the dense adjacency, no masks
    (fused_ok False). One graph object repeated over the batch gives the shared layout; a single
    graph for a larger batch keeps the reference's broadcast quirks (module docstring)."""
    G = len(graph_list)
    if G != batch_size and G != 1:
        raise RuntimeError(
            f"The size of tensor a ({batch_size}) must match the size of tensor b ({G}) at "
            "non-singleton dimension 0")
    g0 = graph_list[0]
    shared = G == batch_size and sum(1 for g in graph_list if g is g0) == G
    infos = [_info(g0, P)] if shared else [_info(g, P) for g in graph_list]
    Gn = len(infos)
    dense = np.zeros((Gn, P, P), np.uint8)
    for s, i in enumerate(infos):
        for p, nb in enumerate(i.adj):
            dense[s, p, list(nb)] = 1
    symmetric = bool(np.array_equal(dense, dense.transpose(0, 2, 1)))
    vcnt = np.stack([i.vcnt for i in infos])
    deg = np.stack([i.deg for i in infos])
    if G == 1 and batch_size > 1:        # degrees broadcast, delta only for sample 0
        vcnt = np.concatenate([vcnt, np.zeros((batch_size - 1, P), np.int32)])
        deg = np.broadcast_to(deg, (batch_size, P)).copy()
    vptr = np.zeros(vcnt.size + 1, np.int32)
    np.cumsum(vcnt.reshape(-1), out=vptr[1:])
    vq = _vq_nonempty(np.concatenate([i.vq for i in infos]))
    rows = 1 if shared else deg.shape[0]
    nbr = np.zeros((P,) if shared else (rows, P), np.int64)
    t = _to_device([nbr, deg[0] if shared else deg, vptr, vq, dense], device)
    return GraphBatch(t[0], t[1], shared, None, t[2], t[3], False, symmetric, t[4])


def n_graphs(graph_list, batch_size: int) -> int:
    """len(graph_list) as the reference's forward sees it; an already ingested GraphBatch counts
    as one graph per sample."""
    return batch_size if isinstance(graph_list, GraphBatch) else len(graph_list)


def ingest(graph_list, P: int, batch_size: int, device) -> GraphBatch:
    """The device layouts of ``graph_list`` (B networkx graphs, or one object repeated). A
    ``GraphBatch`` from an earlier ingest() is passed through: callers that reuse the same graphs
    across forwards (validation loops, benchmarks) ingest once — the tensor fast path."""
    if isinstance(graph_list, GraphBatch):
        gb = graph_list
        if gb.deg.shape[-1] != P or (not gb.shared and gb.deg.shape[0] != batch_size):
            raise ValueError(f"GraphBatch is for P={gb.deg.shape[-1]}"
                             f"{'' if gb.shared else f', B={gb.deg.shape[0]}'}; "
                             f"the forward needs P={P}, B={batch_size}")
        if gb.deg.device != torch.device(device):
            raise ValueError(f"GraphBatch lives on {gb.deg.device}, the forward runs on {device}")
        return gb
    if P > MAX_P:
        raise ValueError(f"P={P} > {MAX_P} agents does not fit the uint8 visit-list ids")
    G = len(graph_list)
    if G == 0:
        raise ValueError("graph_list is empty")
    if P > MASK_P:
        return _batch_wide(graph_list, P, batch_size, device)
    if G != batch_size and G != 1:
        # the reference's sum_neighbors [G,P,1,1] cannot broadcast against [B,P,n,1]
        raise RuntimeError(
            f"The size of tensor a ({batch_size}) must match the size of tensor b ({G}) at "
            "non-singleton dimension 0")
    g0 = graph_list[0]
    # one object repeated (the common case: [G] * B), by identity only (a graph type with a
    # value __eq__ must not collapse distinct graphs onto g0's layout); map(operator.is_) stays
    # in C (~10 ns per entry; a Python generator took ~150 us per forward at B = 4096 on the host,
    # against a 0.55 ms GPU forward)
    same = sum(map(operator.is_, graph_list, itertools.repeat(g0)))
    if same == G:                   # one object repeated
        per = {id(g0): _info(g0, P)}
    else:
        ids = {id(g) for g in graph_list}
        if len(ids) > 64 and G == batch_size:
            # many distinct graphs: one native pass (csrc/dadmm_ingest.c), else numpy
            gb = _batch_native(graph_list, P, device)
            if gb is None:
                gb = _batch_vectorized(graph_list, P, device)
            if gb is not None:
                return gb
        per = {}
        for g in graph_list:
            if id(g) not in per:
                per[id(g)] = _info(g, P)
    if len(per) == 1 and G == batch_size:
        i = next(iter(per.values()))
        if i.ascending:
            key = (str(device), P, i.mask.tobytes(), i.deg.tobytes(), i.vq.tobytes())
            hit = _SHARED_CACHE.get(key)
            if hit is None:
                vptr = np.zeros(P + 1, np.int32)
                np.cumsum(i.vcnt, out=vptr[1:])
                t = _to_device([i.mask.view(np.int64), i.deg, vptr, _vq_nonempty(i.vq)], device)
                hit = GraphBatch(t[0], t[1], True, None, t[2], t[3], symmetric=_symmetric(i.mask))
                if len(_SHARED_CACHE) > 256:
                    _SHARED_CACHE.clear()
                _SHARED_CACHE[key] = hit
            return hit
    if G == 1:   # broadcast degrees, delta only for sample 0 (see module docstring)
        i = per[id(graph_list[0])]
        gb = _batch([i] + [None] * (batch_size - 1), P, device)
        gb.deg = gb.deg.new_tensor(np.broadcast_to(i.deg, (batch_size, P)).copy())
        return gb
    return _batch([per[id(g)] for g in graph_list], P, device)


def generate_er(B: int, P: int, prob: float, seed: int, device, connect: bool = True) -> GraphBatch:
    """B per-sample Erdos-Renyi graphs on agents 0..P-1 generated ON THE DEVICE, already in the
    kernels' layouts (dadmm_graph_generate, csrc/dadmm_graphgen.hip): the progressive driver's
    ``nx.erdos_renyi_graph(P, prob)`` + connectivity patch (gnn_dlasso_progressive.py:181-191)
    and its ingestion, without networkx. Reproducible from ``seed`` (not networkx's RNG)."""
    import ctypes
    from . import _lib
    if P > 64:
        raise ValueError(f"P={P} > 64 agents does not fit the uint64 neighbour mask")
    device = torch.device(device)
    if device.type != "cuda":
        raise RuntimeError("generate_er runs on a ROCm GPU (device must be cuda/hip)")
    L = _lib.load()
    nbr = torch.empty((B, P), dtype=torch.int64, device=device)
    deg = torch.empty((B, P), dtype=torch.float32, device=device)
    with_order = connect and P <= 8
    order = torch.empty((B, P), dtype=torch.int32, device=device) if with_order else None
    vptr = torch.empty(B * P + 1, dtype=torch.int32, device=device)
    scratch = torch.empty(max(B, 1), dtype=torch.int32, device=device)
    vp = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None   # noqa: E731
    with torch.cuda.device(device):
        stream = ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
        args = (B, P, float(prob), int(seed) & (2 ** 64 - 1), int(connect))
        _lib.check("dadmm_graph_generate", L.dadmm_graph_generate(
            *args, vp(nbr), vp(deg), vp(order), vp(vptr), None, vp(scratch), stream))
        total = int(vptr[-1].item()) if B > 0 else 0      # sizes the visit lists (one sync)
        vq = torch.zeros(total + VQ_TAIL, dtype=torch.uint8, device=device)
        if B > 0:
            _lib.check("dadmm_graph_generate", L.dadmm_graph_generate(
                *args, vp(nbr), vp(deg), vp(order), vp(vptr), vp(vq), vp(scratch), stream))
        else:
            vptr.zero_()
    # non-ascending adjacency (connectivity edges) is followed through order (P <= 8) or the
    # visit lists; the fused kernel needs the former
    return GraphBatch(nbr, deg, False, order, vptr, vq, fused_ok=not (connect and P > 8))


def to_networkx(gb: GraphBatch, P: int, samples=None):
    """networkx graphs with the adjacency order a GraphBatch encodes (the own-list segment of each
    agent's visit list): the inverse of ingest(), for checking a GraphBatch against the host path
    and the oracle. Per-sample batches only. ``samples``: the sample indices to convert (default
    all of them; a slice of a large device-generated batch converts only what it needs)."""
    import networkx as nx
    if gb.shared:
        raise ValueError("to_networkx needs a per-sample GraphBatch")
    nbr = gb.nbr.cpu().numpy().view(np.uint64)
    vptr = gb.vptr.cpu().numpy()
    vq = gb.vq.cpu().numpy()
    out = []
    for s in (range(nbr.shape[0]) if samples is None else [int(i) for i in samples]):
        adj = {}
        for p in range(P):
            m = int(nbr[s, p])
            below = bin(m & ((1 << p) - 1)).count("1")
            d = bin(m).count("1")
            o = int(vptr[s * P + p]) + below
            adj[p] = [int(q) for q in vq[o:o + d]]
        # each agent's adjacency dict filled in the recorded order (graph.neighbors(p) follows
        # it); one shared attribute dict per undirected edge, as add_edge would make
        G = nx.Graph()
        G.add_nodes_from(range(P))
        data = {}
        for p in range(P):
            for q in adj[p]:
                G._adj[p][q] = data.setdefault((min(p, q), max(p, q)), {})
        out.append(G)
    return out


def from_csr(nbr_ptr, nbr_idx, deg, P: int, device) -> GraphBatch:
    """GraphBatch from neighbour lists already in CSR form (no networkx): ``nbr_ptr`` [B*P+1],
    ``nbr_idx`` (adjacency order), ``deg`` [B, P]. The tensor fast path for callers that keep
    graphs as arrays; per-sample layout."""
    nbr_ptr = np.asarray(nbr_ptr, np.int64)
    nbr_idx = np.asarray(nbr_idx, np.int64)
    deg = np.asarray(deg, np.float32)
    B = deg.shape[0]
    if nbr_ptr.shape[0] != B * P + 1:
        raise ValueError("nbr_ptr must have B*P+1 entries")
    infos = []
    for s in range(B):
        adj = [nbr_idx[nbr_ptr[s * P + p]:nbr_ptr[s * P + p + 1]].tolist() for p in range(P)]
        if any(q < 0 or q >= P for nb in adj for q in nb):
            raise ValueError(f"neighbour ids must be agents 0..{P - 1}")
        infos.append(_GraphInfo(adj, P))
    if P > MASK_P:
        class _Adj:   # the adjacency lists as a graph_list entry (neighbors(p))
            def __init__(self, adj):
                self._a = adj

            def neighbors(self, p):
                return iter(self._a[p])
        gb = _batch_wide([_Adj(i.adj) for i in infos], P, B, device)
    else:
        gb = _batch(infos, P, device)
    gb.deg = torch.from_numpy(deg.copy()).to(device)
    return gb
