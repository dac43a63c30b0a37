"""Device-side ER graph generation (dadmm_graph_generate, csrc/dadmm_graphgen.hip): the
progressive driver's per-sample graphs (gnn_dlasso_progressive.py:181-191) made on the GPU
directly in the kernels' layouts.

CPU: the numpy restatement (oracle/graphgen_np.py) has the reference's properties — connected
after the patch, edge rate ~ prob, adjacency ER-ascending then the patch edges.
GPU: the device batch equals host ingestion (dadmm_hip.graph.ingest) of the restatement's graphs
array for array (masks, degrees, order nibbles, visit lists), and a forward on it is bit-exact
against the oracle on the same graphs."""
import networkx as nx
import numpy as np
import pytest
import torch

import oracle as O
from oracle import graphgen_np


@pytest.mark.parametrize("P,prob", [(5, 0.3), (16, 0.3), (50, 0.5), (64, 0.05)])
def test_restatement_graphs_are_connected(P, prob):
    gs = graphgen_np.graphs(40, P, prob, seed=11)
    assert all(nx.is_connected(G) for G in gs)
    er = graphgen_np.graphs(40, P, prob, seed=11, connect=False)
    rate = np.mean([G.number_of_edges() / (P * (P - 1) / 2) for G in er])
    assert abs(rate - prob) < 0.05 + 3 * np.sqrt(prob * (1 - prob) / (40 * P * (P - 1) / 2))
    for G, H in zip(gs, er):    # the patch only adds edges, appended after the ER ones
        for p in range(P):
            nb, base = list(G.neighbors(p)), list(H.neighbors(p))
            assert nb[:len(base)] == base == sorted(base)


def test_restatement_depends_on_seed_and_sample():
    a = graphgen_np.graphs(4, 9, 0.4, seed=1)
    b = graphgen_np.graphs(4, 9, 0.4, seed=2)
    edges = lambda gs: [sorted(G.edges()) for G in gs]   # noqa: E731
    assert edges(a) != edges(b)
    assert len({tuple(e) for e in edges(a)}) > 1


@pytest.mark.gpu
@pytest.mark.parametrize("B,P,prob,connect", [(37, 5, 0.3, True), (200, 16, 0.3, True),
                                              (9, 50, 0.5, True), (64, 8, 0.2, True),
                                              (33, 12, 0.4, False), (5, 64, 0.05, True)])
def test_device_batch_equals_host_ingestion(cuda, B, P, prob, connect):
    from dadmm_hip import generate_er, ingest, to_networkx
    seed = 1234 + P
    gb = generate_er(B, P, prob, seed, cuda, connect=connect)
    torch.cuda.synchronize()
    host = graphgen_np.graphs(B, P, prob, seed, connect=connect)
    ref = ingest(host, P, B, cuda)
    assert torch.equal(gb.nbr, ref.nbr) and torch.equal(gb.deg, ref.deg)
    assert torch.equal(gb.vptr, ref.vptr)
    assert torch.equal(gb.vq[: int(gb.vptr[-1])], ref.vq[: int(ref.vptr[-1])])
    if gb.order is not None and ref.order is not None:
        assert torch.equal(gb.order, ref.order)
    back = to_networkx(gb, P)
    for G, H in zip(back, host):
        assert [list(G.neighbors(p)) for p in range(P)] == [list(H.neighbors(p)) for p in range(P)]
        if connect:
            assert nx.is_connected(G)


@pytest.mark.gpu
@pytest.mark.parametrize("P,n,m,B,K,path", [(5, 256, 64, 48, 10, "auto"), (16, 512, 64, 20, 6, "auto"),
                                           (5, 128, 32, 30, 8, "stepwise")])
def test_forward_on_device_graphs_bit_exact(cuda, P, n, m, B, K, path):
    from dadmm_hip import PreparedOperator, forward_raw, generate_er, to_networkx
    gb = generate_er(B, P, 0.3, 77, cuda)
    graphs = to_networkx(gb, P)
    A, b, _ = O.make_problem(P, m, n, B, seed=5)
    rng = np.random.default_rng(3)
    y0, U0, d0 = (1e-2 * rng.standard_normal((3, B, P, n))).astype(np.float32)
    hyp = O.hyp_table((0.4 * rng.standard_normal((K, P, 4))).astype(np.float32), [0.1, 0.99, 0.99, 0.99])
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(cuda)   # noqa: E731
    op = PreparedOperator(t(A))
    Y, U, st = forward_raw(op, t(b), gb, t(hyp), t(y0), t(U0), t(d0), want_U=True, path=path)
    from dadmm_hip.ops import split_cols
    sc = split_cols(op, B, K, gb, hyp_rows=P) if path == "auto" else 0   # dadmm_split.hip order
    Yo, Uo, sto = O.forward_f32(A, b, graphs, hyp, y0, U0, d0, split_cols=sc)
    assert int(st.item()) == sto == 0
    assert np.array_equal(Y.cpu().numpy(), Yo)
    assert np.array_equal(U.cpu().numpy(), Uo)
