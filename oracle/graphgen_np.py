"""numpy restatement of the device ER graph generator (csrc/dadmm_graphgen.hip) — TEST
INFRASTRUCTURE ONLY (see oracle/__init__.py).

The generator stands in for the progressive driver's per-sample graphs
(gnn_dlasso_progressive.py:181-191: nx.erdos_renyi_graph(P, prob), then one edge between the
first nodes of consecutive connected components). Restated here from the kernel's definition:
pair u < v of sample s is an edge iff splitmix64(seed ^ splitmix64(s << 12 | u << 6 | v)) >> 40,
as a 24-bit fraction, is below prob (the float32 compare of the kernel); components in order of
their smallest node, each represented by it; adjacency lists ER-ascending then the connectivity
edges in insertion order. Returns networkx graphs (adjacency order preserved)."""
from __future__ import annotations

import numpy as np

M64 = (1 << 64) - 1


def _splitmix64(x):
    x = (x + 0x9E3779B97F4A7C15) & M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & M64
    return x ^ (x >> 31)


def graphs(B, P, prob, seed, connect=True):
    import networkx as nx
    thr = np.float32(prob)
    out = []
    for s in range(B):
        er = [[] for _ in range(P)]
        for u in range(P):
            for v in range(u + 1, P):
                h = _splitmix64((seed & M64) ^ _splitmix64((s << 12) | (u << 6) | v))
                if np.float32(h >> 40) * np.float32(1.0 / 16777216.0) < thr:
                    er[u].append(v)
                    er[v].append(u)
        adj = [sorted(x) for x in er]
        if connect:
            seen, reps = set(), []
            for p0 in range(P):
                if p0 in seen:
                    continue
                comp, stack = {p0}, [p0]
                while stack:
                    a = stack.pop()
                    for b in er[a]:
                        if b not in comp:
                            comp.add(b)
                            stack.append(b)
                seen |= comp
                reps.append(p0)
            for a, b in zip(reps[:-1], reps[1:]):
                adj[a].append(b)
                adj[b].append(a)
        G = nx.Graph()
        G.add_nodes_from(range(P))
        data = {}
        for p in range(P):
            for q in adj[p]:
                G._adj[p][q] = data.setdefault((min(p, q), max(p, q)), {})
        out.append(G)
    return out
