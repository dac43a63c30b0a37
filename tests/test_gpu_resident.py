"""GPU parity of the agent-resident fused forward (csrc/dadmm_resident.hip) against the oracle
and against the row-divided fused kernel (csrc/dadmm_fused.hip).

Both kernels serve ``dadmm_forward`` for n_pad = 256, P in {4, 5}; the environment variable
DADMM_FUSED_DIVISION selects one ("rows", the default, or "agents"). Bar: bit-exact
(np.array_equal) on every iterate and on U_K against oracle.forward_f32 and against each other,
and the same guard status words (path "fused": the kernels only flag; path "auto": the gated
stepwise recomputation makes the result exact).
"""
import numpy as np
import pytest
import torch

import oracle as O

pytestmark = pytest.mark.gpu

MAXP = [0.1, 0.99, 0.99, 0.99]
DIVISIONS = ["agents", "rows"]


def _inits(B, P, n, seed=99):
    rng = np.random.default_rng(seed)
    return (1e-2 * rng.standard_normal((3, B, P, n))).astype(np.float32)


def _run(dev, division, A, b, graphs, hyp, y0, U0, d0, variant=0, path="fused", monkeypatch=None):
    from dadmm_hip import PreparedOperator, forward_raw, ingest
    monkeypatch.setenv("DADMM_FUSED_DIVISION", division)
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)   # noqa: E731
    B = y0.shape[0]
    op = PreparedOperator(t(A))
    g = ingest(graphs, A.shape[0], B, dev)
    Y, U, st = forward_raw(op, t(b), g, t(hyp), t(y0), t(U0), t(d0), variant=variant,
                           want_U=True, path=path)
    torch.cuda.synchronize()
    return Y.cpu().numpy(), U.cpu().numpy(), int(st.item())


CASES = [
    # P, m, n, B, K, prob, per_sample, variant, hyp_rows
    (5, 64, 256, 40, 25, 0.5, False, 0, 5),    # the headline shape, ragged B
    (5, 64, 256, 17, 25, 0.5, True, 0, 5),     # per-sample connected graphs
    (5, 50, 200, 32, 15, 0.5, False, 0, 5),    # BASELINE configs[0]'s shape (n padded to 256)
    (4, 64, 192, 16, 12, 0.3, False, 0, 4),
    (4, 33, 256, 21, 9, 0.8, True, 1, 4),      # GNN variant clamps, odd m
    (5, 64, 256, 48, 10, 1.0, False, 1, 1),    # complete graph, 'same' hyper-parameters
    (5, 64, 244, 16, 6, 0.0, False, 0, 5),     # no edges at all
]


@pytest.mark.parametrize("P,m,n,B,K,prob,per_sample,variant,H", CASES)
def test_resident_bit_exact(cuda, monkeypatch, P, m, n, B, K, prob, per_sample, variant, H):
    A, b, _ = O.make_problem(P, m, n, B, seed=31 * P + n)
    graphs = ([O.connected_er_graph(P, prob, seed=500 + s) for s in range(B)] if per_sample
              else [O.er_graph(P, prob, seed=11)] * B)
    y0, U0, d0 = _inits(B, P, n, seed=B + K)
    rng = np.random.default_rng(K)
    hyp = O.hyp_table((0.5 * rng.standard_normal((K, H, 4))).astype(np.float32), MAXP)
    Yo, Uo, sto = O.forward_f32(A, b, graphs, hyp, y0, U0, d0, variant=variant)
    assert sto == 0
    out = {}
    for div in DIVISIONS:
        Y, U, st = _run(cuda, div, A, b, graphs, hyp, y0, U0, d0, variant=variant,
                        monkeypatch=monkeypatch)
        assert st == 0, (div, st)
        assert np.array_equal(Y, Yo), (div, np.abs(Y - Yo).max(), np.argwhere(Y != Yo)[:4])
        assert np.array_equal(U, Uo), div
        out[div] = Y
    assert np.array_equal(out["agents"], out["rows"])


def test_resident_trained_headline(cuda, monkeypatch):
    """The trained seq_hyp fixture at the headline shape (the bench's hyper-parameters)."""
    import os
    P, m, n, B, K = 5, 64, 256, 64, 25
    param = np.load(os.path.join(os.path.dirname(__file__), "golden",
                                 "fixture_25_iter_general_learning_seq_hyp_param.npy"))
    A, b, _ = O.make_problem(P, m, n, B, seed=1234)
    G = O.er_graph(P, 0.5, seed=7)
    y0, U0, d0 = _inits(B, P, n, seed=3)
    hyp = O.hyp_table(param, MAXP)
    Y, U, st = _run(cuda, "agents", A, b, [G] * B, hyp, y0, U0, d0, monkeypatch=monkeypatch)
    Yo, Uo, sto = O.forward_f32(A, b, [G] * B, hyp, y0, U0, d0)
    assert st == sto == 0
    assert np.array_equal(Y, Yo) and np.array_equal(U, Uo)


def test_resident_flags_nonfinite_inputs(cuda, monkeypatch):
    """Path 'fused' (no gate): the agent-resident kernel raises the same status bits as the
    row-divided one for NaN / Inf in b, y0, U0 and the hyper-parameter table."""
    P, m, n, B, K = 5, 64, 256, 20, 4
    A, b, _ = O.make_problem(P, m, n, B, seed=1)
    G = O.er_graph(P, 0.5, seed=1)
    y0, U0, d0 = _inits(B, P, n)
    hyp = O.hyp_table(np.zeros((K, P, 4), np.float32), MAXP)
    b2 = b.copy(); b2[3, 1, 2] = np.nan
    y2 = y0.copy(); y2[0, 4, 255] = np.inf
    U2 = U0.copy(); U2[19, 2, 63] = -np.inf
    h2 = hyp.copy(); h2[1, 0, 0] = np.nan
    cases = [(b2, y0, U0, hyp, 4), (b, y2, U0, hyp, 1), (b, y0, U2, hyp, 2), (b, y0, U0, h2, 8),
             (b, y0, U0, hyp, 0)]
    for bb, yy, uu, hh, bit in cases:
        sts = [_run(cuda, div, A, bb, [G] * B, hh, yy, uu, d0, monkeypatch=monkeypatch)[2]
               for div in DIVISIONS]
        assert (sts[0] & bit) == bit and (bit != 0 or sts[0] == 0), (bit, sts)
        assert (sts[0] & 15) == (sts[1] & 15), sts


def test_resident_guards_exact_through_the_gate(cuda, monkeypatch):
    """Path 'auto': a guard event in the agent-resident kernel's batch sends it through the
    gated exact recomputation; the result equals the oracle's guarded forward."""
    P, m, n, B, K = 5, 64, 256, 24, 6
    A, b, _ = O.make_problem(P, m, n, B, seed=2)
    G = O.er_graph(P, 0.5, seed=2)
    y0, U0, d0 = _inits(B, P, n, seed=5)
    hyp = O.hyp_table(np.zeros((K, P, 4), np.float32), MAXP)
    y2 = y0.copy(); y2[7, 3, 100] = np.nan
    Y, U, st = _run(cuda, "agents", A, b, [G] * B, hyp, y2, U0, d0, path="auto",
                    monkeypatch=monkeypatch)
    Yo, Uo, sto = O.forward_f32(A, b, [G] * B, hyp, y2, U0, d0)
    assert st == sto and st & 1
    assert np.array_equal(Y, Yo) and np.array_equal(U, Uo)


def test_resident_directed_shared_graph_exact(cuda, monkeypatch):
    """A directed shared adjacency (successor lists): the per-agent consensus chains follow the
    visits of compute_delta for any adjacency, so the fused launch alone is already exact."""
    import networkx as nx
    P, m, n, B, K = 5, 64, 256, 16, 5
    A, b, _ = O.make_problem(P, m, n, B, seed=4)
    G = nx.DiGraph()
    G.add_nodes_from(range(P))
    G.add_edges_from([(0, 1), (0, 3), (2, 1), (3, 4), (4, 0), (1, 4)])
    y0, U0, d0 = _inits(B, P, n, seed=8)
    rng = np.random.default_rng(1)
    hyp = O.hyp_table((0.3 * rng.standard_normal((K, P, 4))).astype(np.float32), MAXP)
    Y, U, st = _run(cuda, "agents", A, b, [G] * B, hyp, y0, U0, d0, monkeypatch=monkeypatch)
    Yo, Uo, sto = O.forward_f32(A, b, [G] * B, hyp, y0, U0, d0)
    assert st == 0 and sto == 0
    assert np.array_equal(Y, Yo) and np.array_equal(U, Uo)
