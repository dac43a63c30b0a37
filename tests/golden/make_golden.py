"""Generate the committed golden vectors (run from the repo root: python tests/golden/make_golden.py).

Each .npz holds every input of one forward (A, b, neighbour lists, degrees, hyper-parameter
table, y0/U0/d0) and the outputs of the CPU oracle: Y32 (order-matched fp32 restatement, all
iterates; the bit-exact target of the HIP kernel) and Y64 (the reference's Gram-form algorithm in
fp64, iterates k64). They pin the oracle across rounds (tests/test_oracle.py) and the kernel
against committed vectors (tests/test_gpu_parity.py). The reference itself could not be run here
(SURVEY.md §8c), so these are restatement outputs, not reference outputs.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import oracle as O  # noqa: E402

TRAINED = np.load(os.path.join(HERE, "fixture_25_iter_general_learning_seq_hyp_param.npy"))
MAXP = [0.1, 0.99, 0.99, 0.99]

CASES = {
    # name: (P, m, n, B, K, graph kind, hyp kind, variant)
    "small_trained_shared": (5, 16, 64, 8, 25, "shared", "trained", 0),
    "headline_shape_b2": (5, 64, 256, 2, 25, "shared", "trained", 0),
    "c1_shape_b4": (5, 50, 200, 4, 15, "shared", "zero", 0),
    "per_sample_graphs_gnn_variant": (4, 24, 96, 6, 10, "per_sample", "random", 1),
}


def build(name):
    P, m, n, B, K, gk, hk, variant = CASES[name]
    A, b, x = O.make_problem(P, m, n, B, seed=17 + P * n)
    if gk == "shared":
        graphs = [O.er_graph(P, 0.5, seed=7)] * B
    else:
        graphs = [O.connected_er_graph(P, 0.5, seed=50 + s) for s in range(B)]
    if hk == "trained":
        param = TRAINED[:K, :P]
    elif hk == "zero":
        param = np.zeros((K, P, 4), np.float32)
    else:
        param = (0.7 * np.random.default_rng(K).standard_normal((K, P, 4))).astype(np.float32)
    hyp = O.hyp_table(param, MAXP)
    rng = np.random.default_rng(2024)
    y0, U0, d0 = (1e-2 * rng.standard_normal((3, B, P, n))).astype(np.float32)
    nbr_ptr, nbr_idx, deg = O.graph_arrays(graphs, P)
    Y32, U32, _ = O.forward_f32(A, b, graphs, hyp, y0, U0, d0, variant=variant)
    Y64, U64, _ = O.forward_f64(A, b, graphs, hyp, y0, U0, d0, variant=variant)
    k64 = np.array([0, K // 2, K - 1], np.int32)      # fp64 iterates kept (size)
    return dict(A=A, b=b, x=x, nbr_ptr=nbr_ptr, nbr_idx=nbr_idx, deg=deg, hyp=hyp, y0=y0, U0=U0,
                d0=d0, variant=np.int32(variant), Y32=Y32, U32=U32, k64=k64, Y64=Y64[k64],
                U64=U64)


def graphs_from(g):
    """Rebuild networkx graphs (adjacency order preserved) from a golden's CSR lists."""
    import networkx as nx
    P = g["deg"].shape[1]
    out = []
    ptr, idx = g["nbr_ptr"], g["nbr_idx"]
    for s in range(g["deg"].shape[0]):
        G = nx.Graph()
        G.add_nodes_from(range(P))
        for p in range(P):
            for t in range(ptr[s * P + p], ptr[s * P + p + 1]):
                G.add_edge(p, int(idx[t]))
        out.append(G)
    return out


if __name__ == "__main__":
    for name in CASES:
        np.savez_compressed(os.path.join(HERE, f"golden_{name}.npz"), **build(name))
        print("wrote", name)
