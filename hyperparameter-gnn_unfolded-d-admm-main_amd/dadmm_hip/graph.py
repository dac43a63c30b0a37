"""Graph ingestion: ``graph_list`` (networkx graphs) -> neighbour bitmasks + degrees.

Replaces the Python loops of ``compute_sum_neighbors`` (unfolded_DLASSO.py:111-118) and the graph
walk of ``compute_delta`` (:127-140) with the device layout the kernel reads (include/dadmm.h):
``nbr[s][p]`` bit q set <=> q in graph_list[s].neighbors(p), ``deg[s][p] = len(neighbors(p))``.

compute_delta sums each agent's own neighbour terms in ``graph.neighbors(p)`` order. For the
graphs the reference builds with ``erdos_renyi_graph`` that order is ascending (edges are added in
lexicographic order) and the masks alone describe it. Graphs whose adjacency lists are not
ascending (e.g. the connectivity patch of gnn_dlasso_progressive.py:184-191 appends edges) also
get ``order``: the adjacency order packed 4 bits per neighbour, so the kernel accumulates in
exactly the reference's order (P <= 8).

Quirks of the reference kept on purpose (it never checks ``len(graph_list) == len(b)``):
  * ``compute_sum_neighbors`` sizes its output by ``len(graph_list)`` and the result broadcasts
    against the state, so one graph for a batch of B gives every sample that graph's degrees;
  * ``compute_delta`` only walks ``range(len(graph_list))``: samples past it get delta = 0.
"""
from __future__ import annotations

import numpy as np
import torch

_MASK_CACHE: dict = {}


def _graph_masks(G, P: int):
    """(mask uint64 [P], deg float32 [P], order uint32 [P] or None) for one graph."""
    masks = np.zeros(P, np.uint64)
    deg = np.zeros(P, np.float32)
    order = np.zeros(P, np.uint32)
    ascending = True
    for p in range(P):
        nb = list(G.neighbors(p))
        deg[p] = len(nb)
        for t, q in enumerate(nb):
            if not (0 <= q < P):
                raise ValueError(f"neighbour id {q} of agent {p}: must be an agent 0..{P - 1}")
            masks[p] |= np.uint64(1) << np.uint64(q)
            if t < 8:
                order[p] |= np.uint32(q & 15) << np.uint32(4 * t)
        ascending &= all(nb[i] < nb[i + 1] for i in range(len(nb) - 1))
    return masks, deg, (None if ascending else order)


class GraphBatch:
    """Device-resident neighbour masks and degrees for one forward call."""

    __slots__ = ("nbr", "deg", "shared", "order")

    def __init__(self, nbr: torch.Tensor, deg: torch.Tensor, shared: bool, order=None):
        self.nbr = nbr      # int64 (uint64 bit patterns) [P] if shared else [B, P]
        self.deg = deg      # float32 [P] if shared else [B, P]
        self.shared = shared
        self.order = order  # int32 [B, P] packed adjacency order, or None (ascending)


def ingest(graph_list, P: int, batch_size: int, device) -> GraphBatch:
    if P > 64:
        raise ValueError(f"P={P} > 64 agents does not fit the uint64 neighbour mask")
    G = len(graph_list)
    if G == 0:
        raise ValueError("graph_list is empty")
    if G != batch_size and G != 1:
        # the reference's sum_neighbors [G,P,1,1] cannot broadcast against [B,P,n,1]
        raise RuntimeError(
            f"The size of tensor a ({batch_size}) must match the size of tensor b ({G}) at "
            "non-singleton dimension 0")
    per = {}
    for g in graph_list:
        if id(g) not in per:
            per[id(g)] = _graph_masks(g, P)
    ordered = any(v[2] is not None for v in per.values())
    if ordered and P > 8:
        raise ValueError("graphs with non-ascending adjacency lists need P <= 8 agents")
    if len(per) == 1 and G == batch_size and not ordered:
        masks, deg, _ = next(iter(per.values()))
        key = (str(device), masks.tobytes(), deg.tobytes())
        hit = _MASK_CACHE.get(key)
        if hit is None:
            hit = GraphBatch(torch.from_numpy(masks.view(np.int64).copy()).to(device),
                             torch.from_numpy(deg.copy()).to(device), True)
            if len(_MASK_CACHE) > 256:
                _MASK_CACHE.clear()
            _MASK_CACHE[key] = hit
        return hit
    nbr = np.zeros((batch_size, P), np.uint64)
    degs = np.zeros((batch_size, P), np.float32)
    order = np.zeros((batch_size, P), np.uint32) if ordered else None

    def _fill(s, v):
        nbr[s], degs[s] = v[0], v[1]
        if ordered:
            order[s] = v[2] if v[2] is not None else _ascending_order(v[0], P)

    if G == 1:   # broadcast degrees, delta only for sample 0 (see module docstring)
        v = per[id(graph_list[0])]
        _fill(0, v)
        degs[:] = v[1]
    else:
        for s, g in enumerate(graph_list):
            _fill(s, per[id(g)])
    tensors = [torch.from_numpy(nbr.view(np.int64)), torch.from_numpy(degs)]
    if ordered:
        tensors.append(torch.from_numpy(order.view(np.int32)))
    if torch.device(device).type == "cuda":
        tensors = [t.pin_memory() for t in tensors]
    tensors = [t.to(device, non_blocking=True) for t in tensors]
    return GraphBatch(tensors[0], tensors[1], False, tensors[2] if ordered else None)


def _ascending_order(masks, P):
    """Packed ascending adjacency order for every agent of one graph -> uint32 [P]."""
    out = np.zeros(P, np.uint32)
    for p in range(P):
        o, t = 0, 0
        for q in range(P):
            if (int(masks[p]) >> q) & 1:
                o |= q << (4 * t)
                t += 1
        out[p] = o
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
    nbr = np.zeros((B, P), np.uint64)
    order = np.zeros((B, P), np.uint32)
    ordered = False
    for s in range(B):
        for p in range(P):
            nb = nbr_idx[nbr_ptr[s * P + p]:nbr_ptr[s * P + p + 1]]
            if ((nb < 0) | (nb >= P)).any():
                raise ValueError(f"neighbour ids must be agents 0..{P - 1}")
            for t, q in enumerate(nb):
                nbr[s, p] |= np.uint64(1) << np.uint64(q)
                if t < 8:
                    order[s, p] |= np.uint32(q) << np.uint32(4 * t)
            ordered |= bool((np.diff(nb) <= 0).any())
    if ordered and P > 8:
        raise ValueError("graphs with non-ascending adjacency lists need P <= 8 agents")
    out = [torch.from_numpy(nbr.view(np.int64)), torch.from_numpy(deg.copy())]
    if ordered:
        out.append(torch.from_numpy(order.view(np.int32)))
    out = [t.to(device) for t in out]
    return GraphBatch(out[0], out[1], False, out[2] if ordered else None)
