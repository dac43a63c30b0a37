"""GPU parity of the column-split forward for small batches (csrc/dadmm_split.hip,
dadmm_forward_split) against the oracle's split-order restatement.

The split forward cuts each 16-sample tile's n_pad columns into slices of 64 (one workgroup each)
and sums the GEMM1 partials R = ((c_0 + c_1) + c_2) + ... (slice 0's chain from -b):
oracle.forward_f32(..., split_cols=64) restates that order, and the kernel must match it
bit-for-bit (np.array_equal on every iterate and on U_K) for every graph kind, both variants,
ragged batches (B not a multiple of 16), padded n and m, several tiles per workgroup group, and
BASELINE configs[1] itself (P=5, n=256, m_p=64, B=1024, K=25). The guards go through the gated
stepwise recomputation exactly as after the fused kernel.
"""
import os

import numpy as np
import pytest
import torch

import oracle as O

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")
TRAINED = np.load(os.path.join(GOLD, "fixture_25_iter_general_learning_seq_hyp_param.npy"))
MAXP = [0.1, 0.99, 0.99, 0.99]


def _t(x, dev):
    return torch.from_numpy(np.ascontiguousarray(x)).to(dev)


def _inits(B, P, n, seed=99):
    rng = np.random.default_rng(seed)
    return (1e-2 * rng.standard_normal((3, B, P, n))).astype(np.float32)


def _hyp(K, P, seed=3, same=False):
    rng = np.random.default_rng(seed)
    param = (0.3 * rng.standard_normal((K, 1 if same else P, 4))).astype(np.float32)
    return O.hyp_table(param, MAXP)


def _run(dev, A, b, graphs, hyp, y0, U0, d0, variant=0, path="split"):
    from dadmm_hip import PreparedOperator, forward_raw, ingest
    from dadmm_hip.ops import split_cols
    B = y0.shape[0]
    op = PreparedOperator(_t(A, dev))
    g = ingest(graphs, A.shape[0], B, dev)
    Y, U, st = forward_raw(op, _t(b, dev), g, _t(hyp, dev), _t(y0, dev), _t(U0, dev), _t(d0, dev),
                           variant=variant, want_U=True, path=path)
    torch.cuda.synchronize()
    sc = split_cols(op, B, hyp.shape[0], g, hyp_rows=hyp.shape[1])
    return Y.cpu().numpy(), U.cpu().numpy(), int(st.item()), sc


def _check(Y, U, Yo, Uo):
    assert np.array_equal(Y, Yo), (f"{np.sum(Y != Yo)} of {Y.size} differ, max |diff| "
                                   f"{np.abs(Y - Yo).max()} first at {np.argwhere(Y != Yo)[:3].tolist()}")
    assert np.array_equal(U, Uo), f"U_K: {np.sum(U != Uo)} differ"


CASES = [
    # P, m,  n,  B,  K, graph,      variant, same
    (5, 64, 256, 40, 25, "shared", 0, False),    # the headline shape, ragged batch
    (5, 64, 256, 64, 10, "lane", 0, False),      # per-sample connected ER graphs
    (5, 64, 256, 48, 8, "ordered", 1, False),    # non-ascending adjacency order, GNN clamps
    (6, 64, 256, 33, 6, "shared", 0, True),      # P = 6, DADMM_mode 'same'
    (3, 50, 200, 20, 7, "lane", 0, False),       # padded m and n (n_pad 256)
    (4, 64, 128, 70, 9, "shared", 1, False),     # n_pad 128: two slices
    (2, 64, 100, 16, 5, "lane", 0, False),       # n_pad 128, padded columns
    (1, 32, 256, 24, 4, "shared", 0, False),     # one agent (no consensus)
]


@pytest.mark.parametrize("P,m,n,B,K,graph,variant,same", CASES)
def test_split_forward_bit_exact(cuda, P, m, n, B, K, graph, variant, same):
    A, b, _ = O.make_problem(P, m, n, B, seed=11 + P + n)
    if graph == "shared":
        graphs = [O.er_graph(P, 0.5, seed=7)] * B
    else:
        graphs = [O.connected_er_graph(P, 0.5, seed=200 + s) for s in range(B)]
        if graph == "ordered":
            import networkx as nx
            rng = np.random.default_rng(5)
            out = []
            for g0 in graphs:       # same edges, adjacency lists inserted in a shuffled order
                g1 = nx.Graph()
                g1.add_nodes_from(range(P))
                edges = list(g0.edges())
                rng.shuffle(edges)
                g1.add_edges_from((v, u) if rng.random() < 0.5 else (u, v) for u, v in edges)
                out.append(g1)
            graphs = out
    y0, U0, d0 = _inits(B, P, n)
    hyp = _hyp(K, P, same=same)
    Y, U, st, sc = _run(cuda, A, b, graphs, hyp, y0, U0, d0, variant)
    assert sc == 64 and st == 0
    Yo, Uo, sto = O.forward_f32(A, b, graphs, hyp, y0, U0, d0, variant=variant, split_cols=64)
    assert sto == 0
    _check(Y, U, Yo, Uo)


def test_split_order_differs_from_unsplit_but_within_fp32_noise(cuda):
    """The split order is a different fp32 evaluation: it must NOT equal the fused order
    bit-for-bit at the headline shape (the test would otherwise not discriminate), and the two
    stay within the fp32 noise band of each other (final-iterate MSE vs fp64 alike)."""
    P, m, n, B, K = 5, 64, 256, 32, 25
    A, b, _ = O.make_problem(P, m, n, B, seed=1234)
    G = O.er_graph(P, 0.5, seed=7)
    y0, U0, d0 = _inits(B, P, n)
    hyp = O.hyp_table(TRAINED, MAXP)
    Y, _, st, _ = _run(cuda, A, b, [G] * B, hyp, y0, U0, d0)
    Yf, _, _ = O.forward_f32(A, b, [G] * B, hyp, y0, U0, d0)
    Y64, _, _ = O.forward_f64(A, b, [G] * B, hyp, y0, U0, d0)
    assert st == 0 and not np.array_equal(Y, Yf)
    mse_split = float(((Y[-1] - Y64[-1]) ** 2).mean())
    mse_fused = float(((Yf[-1] - Y64[-1]) ** 2).mean())
    assert mse_split <= 1e-5 and mse_fused <= 1e-5, (mse_split, mse_fused)


def test_configs1_full_batch_bit_exact(cuda):
    """BASELINE configs[1] as the module runs it: DLASSO_unfolded at P=5, n=256, m_p=64, B=1024,
    K=25 with the trained table; the auto path takes the split forward (64 tiles x 4 slices =
    256 workgroups) and every iterate equals the split-order oracle."""
    import argparse

    import unfolded_DLASSO
    from dadmm_hip.ops import split_cols
    P, m, n, B, K = 5, 64, 256, 1024, 25
    A, b, _ = O.make_problem(P, m, n, B, seed=4321)
    G = O.er_graph(P, 0.5, seed=7)
    args = argparse.Namespace(GHN_iter_num=K, DADMM_mode="diff", alpha_max=0.1, tau_max=0.99,
                              rho_max=0.99, eta_max=0.99, max_penalty_threshold=0.8,
                              penalty_reduction_factor=0.95)
    model = unfolded_DLASSO.DLASSO_unfolded(_t(A, cuda)[None], args).to(cuda).eval()
    with torch.no_grad():
        model.seq_hyp.param.copy_(torch.from_numpy(TRAINED))
    y0, U0, d0 = _inits(B, P, n, seed=5)
    with torch.no_grad():
        Y, _ = model(_t(b, cuda)[..., None], [G] * B,
                     inits=tuple(_t(x, cuda)[..., None] for x in (y0, U0, d0)))
    torch.cuda.synchronize()
    assert int(model.last_status.item()) == 0
    assert split_cols(model.operator(), B, K) == 64
    table = model.hyp_table(K).detach().cpu().numpy()
    Yo, _, sto = O.forward_f32(A, b, [G] * B, table, y0, U0, d0, split_cols=64)
    assert sto == 0
    Yh = Y[..., 0].cpu().numpy()
    assert np.array_equal(Yh, Yo), f"{np.sum(Yh != Yo)} of {Yh.size} differ"


def test_split_several_tiles_per_group(cuda):
    """B = 2048 at n_pad 256: 128 tiles over 64 workgroup groups (each walks two tiles, the
    epoch words and partial slots carried across them); bit-exact on every sample."""
    from dadmm_hip.ops import split_cols
    P, m, n, B, K = 5, 64, 256, 2048, 6
    A, b, _ = O.make_problem(P, m, n, B, seed=77)
    graphs = [O.connected_er_graph(P, 0.5, seed=900 + s % 97) for s in range(B)]
    y0, U0, d0 = _inits(B, P, n, seed=8)
    hyp = _hyp(K, P)
    Y, U, st, sc = _run(cuda, A, b, graphs, hyp, y0, U0, d0, path="auto")
    assert sc == 64 and st == 0
    Yo, Uo, _ = O.forward_f32(A, b, graphs, hyp, y0, U0, d0, split_cols=64)
    _check(Y, U, Yo, Uo)


def test_split_guards_recompute_exactly(cuda):
    """A non-finite y0 entry (reference guard :55-57) and a NaN gradient (:84-86): the split
    launch flags the batch and the gated stepwise launch recomputes it with the guards applied,
    exactly as the oracle's guarded restatement (its order: the stepwise path's)."""
    P, m, n, B, K = 5, 64, 256, 40, 6
    A, b, _ = O.make_problem(P, m, n, B, seed=3)
    G = O.er_graph(P, 0.5, seed=7)
    y0, U0, d0 = _inits(B, P, n)
    y0[3, 2, 17] = np.nan
    hyp = _hyp(K, P)
    Y, U, st, _ = _run(cuda, A, b, [G] * B, hyp, y0, U0, d0, path="auto")
    Yo, Uo, sto = O.forward_f32(A, b, [G] * B, hyp, y0, U0, d0)
    assert st == sto and sto & 1
    _check(Y, U, Yo, Uo)
    b2 = b.copy()
    b2[5, 1, 3] = np.nan
    Y, U, st, _ = _run(cuda, A, b2, [G] * B, hyp, *_inits(B, P, n), path="auto")
    Yo, Uo, sto = O.forward_f32(A, b2, [G] * B, hyp, *_inits(B, P, n))
    assert st == sto and sto != 0
    _check(Y, U, Yo, Uo)


def test_split_under_concurrent_load(cuda):
    """Uneven load (MI355X_MICROARCH.md: test hand-offs under load, consumers L1-warm): the split
    forward runs while a second stream keeps GEMMs in flight, four times back to back on the
    same scratch sizes. Each result is either the split order (the slices were co-resident) or,
    after a timed-out wait, the exact stepwise recomputation (the unsplit order) — never
    anything else."""
    P, m, n, B, K = 5, 64, 256, 512, 12
    A, b, _ = O.make_problem(P, m, n, B, seed=21)
    G = O.er_graph(P, 0.5, seed=7)
    y0, U0, d0 = _inits(B, P, n, seed=4)
    hyp = _hyp(K, P)
    Ys = O.forward_f32(A, b, [G] * B, hyp, y0, U0, d0, split_cols=64)[0]
    Yf = O.forward_f32(A, b, [G] * B, hyp, y0, U0, d0)[0]
    side = torch.cuda.Stream(cuda)
    x = torch.randn(4096, 4096, device=cuda)
    for _ in range(4):
        with torch.cuda.stream(side):
            for _ in range(8):
                x = torch.tanh(x @ x * 1e-3)
        Y, _, st, _ = _run(cuda, A, b, [G] * B, hyp, y0, U0, d0, path="auto")
        assert np.array_equal(Y, Ys) or np.array_equal(Y, Yf)
    torch.cuda.synchronize()
