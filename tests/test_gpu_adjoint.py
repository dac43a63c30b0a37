"""GPU parity of the training path: the recording forward (dadmm_forward_record and the stepwise
recording) and the adjoint kernel (dadmm_backward), through the C ABI and through
DLASSO_unfolded's loss.backward().

Bar:
  * recording: Y, Grec, Urec bit-exact (np.array_equal) against oracle.forward_f32_rec;
  * adjoint: dhyp within ADJ_RTOL x max|dhyp| (plus ADJ_RTOL x |entry|) of oracle.backward_np64
    evaluated in fp64 along the kernel's OWN recorded trajectory. oracle.backward_np64 is pinned to
    torch autograd through the reference's op sequence (tests/test_oracle.py). The comparison is
    along the same trajectory because the forward is expansive: an fp64 trajectory drifts from any
    fp32 one and the adjoint inherits that drift (test_adjoint_sensitivity_fp32_vs_fp64_trajectory);
    along one trajectory the only differences are the adjoint's own fp32 roundings.
"""
import argparse
import os

import numpy as np
import pytest
import torch

import oracle as O

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")
TRAINED = np.load(os.path.join(GOLD, "fixture_25_iter_general_learning_seq_hyp_param.npy"))
MAXP = [0.1, 0.99, 0.99, 0.99]
ADJ_RTOL = 1e-5


def _inits(B, P, n, seed=99):
    rng = np.random.default_rng(seed)
    return (1e-2 * rng.standard_normal((3, B, P, n))).astype(np.float32)


def _t(x, dev):
    return torch.from_numpy(np.ascontiguousarray(x)).to(dev)


def _graphs(P, B, prob, per_sample, seed=0):
    if per_sample:
        return [O.connected_er_graph(P, prob, seed=seed + 1000 + s) for s in range(B)]
    return [O.er_graph(P, prob, seed=seed + 3)] * B


def _record(dev, A, b, graphs, hyp, y0, U0, d0, variant=0, path="auto"):
    from dadmm_hip import PreparedOperator, forward_raw, ingest
    B, P = y0.shape[:2]
    op = PreparedOperator(_t(A, dev))
    g = ingest(graphs, P, B, dev)
    Y, U, st, traj = forward_raw(op, _t(b, dev), g, _t(hyp, dev), _t(y0, dev), _t(U0, dev),
                                 _t(d0, dev), variant=variant, want_U=True, path=path,
                                 record=True)
    torch.cuda.synchronize()
    return op, g, Y, U, int(st.item()), traj


def _close(got, want, rtol=ADJ_RTOL):
    err = np.abs(got - want)
    bound = rtol * np.abs(want).max() + rtol * np.abs(want)
    assert (err <= bound).all(), (f"max err {err.max():.3e} (rel to max "
                                  f"{err.max() / np.abs(want).max():.3e})")


SHAPES = [
    # P, m, n, B, K, prob, per_sample, H ('diff' P / 'same' 1), variant
    (5, 64, 256, 40, 25, 0.5, False, 5, 0),   # headline shape, trained table
    (5, 64, 256, 33, 25, 0.5, True, 5, 0),    # per-sample graphs, ragged last workgroup
    (5, 50, 200, 32, 15, 0.5, False, 5, 0),   # BASELINE configs[0] shape, n padded to 256
    (3, 16, 64, 20, 8, 0.9, True, 1, 0),      # 'same' mode
    (6, 32, 128, 24, 10, 0.5, True, 6, 1),    # GNN variant (fixed clamps, delta clamp)
    (4, 24, 96, 18, 10, 0.4, False, 1, 1),
    (1, 8, 16, 5, 4, 0.5, False, 1, 0),       # one agent: no consensus
    (2, 20, 124, 31, 9, 1.0, False, 2, 0),
]


@pytest.mark.parametrize("path", ["auto", "stepwise"])
@pytest.mark.parametrize("P,m,n,B,K,prob,per_sample,H,variant", SHAPES)
def test_recording_bit_exact(cuda, P, m, n, B, K, prob, per_sample, H, variant, path):
    A, b, _ = O.make_problem(P, m, n, B, seed=P * 10 + n)
    graphs = _graphs(P, B, prob, per_sample)
    y0, U0, d0 = _inits(B, P, n, seed=B)
    rng = np.random.default_rng(K)
    hyp = O.hyp_table((0.5 * rng.standard_normal((K, H, 4))).astype(np.float32), MAXP)
    _, _, Y, U, st, traj = _record(cuda, A, b, graphs, hyp, y0, U0, d0, variant, path)
    Yo, Uo, sto, Go, Uro = O.forward_f32_rec(A, b, graphs, hyp, y0, U0, d0, variant=variant)
    assert st == sto == 0
    assert np.array_equal(Y.cpu().numpy(), Yo)
    assert np.array_equal(U.cpu().numpy(), Uo)
    assert np.array_equal(traj.Grec[..., :n].cpu().numpy(), Go)
    assert np.array_equal(traj.Urec[..., :n].cpu().numpy(), Uro)


@pytest.mark.parametrize("P,m,n,B,K,prob,per_sample,H,variant", SHAPES)
def test_adjoint_vs_oracle_on_own_trajectory(cuda, P, m, n, B, K, prob, per_sample, H, variant):
    from dadmm_hip.ops import backward_raw
    A, b, _ = O.make_problem(P, m, n, B, seed=P * 10 + n)
    graphs = _graphs(P, B, prob, per_sample)
    y0, U0, d0 = _inits(B, P, n, seed=B)
    if (H, K) == (5, 25):
        hyp = O.hyp_table(TRAINED, MAXP)
    else:
        rng = np.random.default_rng(K)
        hyp = O.hyp_table((0.5 * rng.standard_normal((K, H, 4))).astype(np.float32), MAXP)
    op, g, Y, _, st, traj = _record(cuda, A, b, graphs, hyp, y0, U0, d0, variant)
    assert st == 0
    rng = np.random.default_rng(7)
    gY = rng.standard_normal((K, B, P, n)).astype(np.float32)
    gY[: K // 2] *= 0.1
    dh = backward_raw(op, g, traj, _t(gY, cuda))
    torch.cuda.synchronize()
    want = O.backward_np64(A, graphs, hyp, y0, d0, Y.cpu().numpy(),
                           traj.Grec[..., :n].cpu().numpy(), traj.Urec[..., :n].cpu().numpy(), gY,
                           variant=variant)
    _close(dh.cpu().numpy().astype(np.float64), want)


# shapes only the general adjoint (dadmm_adjoint) covers: many agents, long signals, m > 64,
# non-ascending adjacency at P > 8
GENERAL_SHAPES = [
    # P, m, n, B, K, prob, per_sample, H, variant
    (5, 100, 500, 12, 10, 0.5, False, 5, 0),   # the reference's defaults m = 100, n = 500
    (16, 64, 512, 9, 6, 0.3, True, 16, 0),     # BASELINE configs[2] agent count and size
    (9, 40, 320, 14, 5, 0.4, False, 1, 1),     # 'same' mode, GNN variant
    (50, 32, 1024, 3, 3, 0.5, True, 50, 0),    # configs[4] agent count and size
    (12, 130, 96, 7, 4, 0.6, True, 12, 1),     # three m-groups
]


@pytest.mark.parametrize("P,m,n,B,K,prob,per_sample,H,variant", GENERAL_SHAPES + SHAPES[:3])
def test_general_adjoint_vs_oracle_on_own_trajectory(cuda, P, m, n, B, K, prob, per_sample, H,
                                                     variant):
    """dadmm_adjoint (any shape) against the fp64 oracle adjoint along the recorded trajectory;
    the fused shapes too (path 'general' on a fused trajectory)."""
    from dadmm_hip.ops import backward_raw
    A, b, _ = O.make_problem(P, m, n, B, seed=P * 10 + n)
    graphs = _graphs(P, B, prob, per_sample)
    y0, U0, d0 = _inits(B, P, n, seed=B)
    rng = np.random.default_rng(K)
    hyp = O.hyp_table((0.5 * rng.standard_normal((K, H, 4))).astype(np.float32), MAXP)
    op, g, Y, _, st, traj = _record(cuda, A, b, graphs, hyp, y0, U0, d0, variant)
    assert st == 0
    Yo, _, _, Go, Uro = O.forward_f32_rec(A, b, graphs, hyp, y0, U0, d0, variant=variant)
    assert np.array_equal(Y.cpu().numpy(), Yo)
    assert np.array_equal(traj.Grec[..., :n].cpu().numpy(), Go)
    rng = np.random.default_rng(7)
    gY = rng.standard_normal((K, B, P, n)).astype(np.float32)
    gY[: K // 2] *= 0.1
    dh = backward_raw(op, g, traj, _t(gY, cuda), path="general")
    torch.cuda.synchronize()
    want = O.backward_np64(A, graphs, hyp, y0, d0, Yo, Go, Uro, gY, variant=variant)
    _close(dh.cpu().numpy().astype(np.float64), want)


def test_general_adjoint_non_ascending_adjacency(cuda):
    """P = 10 graphs whose adjacency lists are not ascending (the progressive driver's
    connectivity patch appends edges): the fused adjoint cannot follow them (P > 8), the general
    adjoint uses the visit lists."""
    import networkx as nx
    from dadmm_hip.ops import backward_raw
    P, m, n, B, K = 10, 24, 64, 6, 4
    graphs = []
    for s in range(B):
        G = nx.Graph()
        G.add_nodes_from(range(P))
        r = np.random.default_rng(40 + s)
        for q in r.permutation(P):
            for t in r.choice(P, 3, replace=False):
                if t != q:
                    G.add_edge(int(q), int(t))
        graphs.append(G)
    A, b, _ = O.make_problem(P, m, n, B, seed=3)
    y0, U0, d0 = _inits(B, P, n)
    hyp = O.hyp_table((0.5 * np.random.default_rng(1).standard_normal((K, P, 4))).astype(np.float32), MAXP)
    op, g, Y, _, st, traj = _record(cuda, A, b, graphs, hyp, y0, U0, d0)
    assert st == 0 and not g.fused_ok
    gY = np.random.default_rng(2).standard_normal((K, B, P, n)).astype(np.float32)
    dh = backward_raw(op, g, traj, _t(gY, cuda))
    want = O.backward_np64(A, graphs, hyp, y0, d0, Y.cpu().numpy(), traj.Grec[..., :n].cpu().numpy(),
                           traj.Urec[..., :n].cpu().numpy(), gY)
    _close(dh.cpu().numpy().astype(np.float64), want)


def test_general_adjoint_deterministic(cuda):
    from dadmm_hip.ops import backward_raw
    P, m, n, B, K = 16, 100, 512, 40, 5
    A, b, _ = O.make_problem(P, m, n, B, seed=4)
    graphs = _graphs(P, B, 0.3, True)
    y0, U0, d0 = _inits(B, P, n)
    hyp = O.hyp_table(np.zeros((K, P, 4), np.float32), MAXP)
    op, g, Y, _, st, traj = _record(cuda, A, b, graphs, hyp, y0, U0, d0)
    gY = torch.randn(Y.shape, device=cuda, generator=torch.Generator(cuda).manual_seed(1))
    d1 = backward_raw(op, g, traj, gY)
    d2 = backward_raw(op, g, traj, gY)
    assert torch.equal(d1, d2)


def test_adjoint_deterministic(cuda):
    from dadmm_hip.ops import backward_raw
    P, m, n, B, K = 5, 64, 256, 300, 25
    A, b, _ = O.make_problem(P, m, n, B, seed=4)
    graphs = _graphs(P, B, 0.5, True)
    y0, U0, d0 = _inits(B, P, n)
    hyp = O.hyp_table(TRAINED, MAXP)
    op, g, Y, _, st, traj = _record(cuda, A, b, graphs, hyp, y0, U0, d0)
    gY = torch.randn(Y.shape, device=cuda, generator=torch.Generator(cuda).manual_seed(1))
    d1 = backward_raw(op, g, traj, gY)
    d2 = backward_raw(op, g, traj, gY)
    assert torch.equal(d1, d2)


def _args(K, mode="diff"):
    return argparse.Namespace(GHN_iter_num=K, DADMM_mode=mode, alpha_max=0.1, tau_max=0.99,
                              rho_max=0.99, eta_max=0.99, max_penalty_threshold=0.8,
                              penalty_reduction_factor=0.95)


@pytest.mark.parametrize("mode", ["diff", "same"])
def test_module_backward_matches_oracle_chain(cuda, mode):
    """loss_final.backward() through the drop-in DLASSO_unfolded (train mode, as
    unfolded_train_new.py:74-80 drives it): seq_hyp.param.grad equals the oracle adjoint chained
    through the (CPU) hyper-parameter table."""
    import gnn_dlasso_utils
    import unfolded_DLASSO
    P, m, n, B, K = 5, 64, 256, 48, 25
    A, b, x = O.make_problem(P, m, n, B, seed=21)
    model = unfolded_DLASSO.DLASSO_unfolded(_t(A, cuda)[None], _args(K, mode)).to(cuda)
    H = P if mode == "diff" else 1
    with torch.no_grad():
        model.seq_hyp.param.copy_(torch.from_numpy(TRAINED[:, :H]))
    model.train()
    graphs = [O.er_graph(P, 0.5, seed=7)] * B
    y0, U0, d0 = _inits(B, P, n)
    Y, _ = model(_t(b, cuda)[..., None], graphs, inits=tuple(_t(v, cuda) for v in (y0, U0, d0)))
    label = _t(x, cuda)[..., None]
    loss_mean, loss_final = gnn_dlasso_utils.compute_loss(Y, label)
    loss_final.backward()
    got = model.seq_hyp.param.grad.cpu().numpy()

    # oracle chain: d loss_final / dY (closed form of compute_loss's last-layer MSE), adjoint
    # along the recorded trajectory, then autograd through the table on the CPU
    table_cpu = model.seq_hyp.table(K).detach().cpu().numpy()
    Yo, _, _, Go, Uro = O.forward_f32_rec(A, b, graphs, table_cpu, y0, U0, d0)
    assert np.array_equal(Y[..., 0].detach().cpu().numpy(), Yo)
    gY = np.zeros((K, B, P, n))
    gY[-1] = 2.0 * (Yo[-1].astype(np.float64) - x[:, None, :]) / (B * n * P)
    dtab = O.backward_np64(A, graphs, table_cpu, y0, d0, Yo, Go, Uro, gY)
    p = torch.tensor(TRAINED[:, :H], dtype=torch.float64, requires_grad=True)
    seq = unfolded_DLASSO.seq_hyperparam([K, H, 4], torch.tensor(MAXP, dtype=torch.float64),
                                         _args(K, mode))
    seq.param = torch.nn.Parameter(p)
    seq.train()
    tab = seq.table(K)
    want, = torch.autograd.grad(tab, seq.param, grad_outputs=torch.from_numpy(dtab))
    _close(got.astype(np.float64), want.numpy(), rtol=1e-4)


def test_module_backward_refuses_after_guard(cuda):
    import unfolded_DLASSO
    from dadmm_hip.autograd import GuardAdjointError
    P, m, n, B, K = 3, 16, 64, 8, 4
    A, b, _ = O.make_problem(P, m, n, B, seed=1)
    model = unfolded_DLASSO.DLASSO_unfolded(_t(A, cuda)[None], _args(K)).to(cuda)
    y0, U0, d0 = _inits(B, P, n)
    y0[2, 1, 5] = np.nan
    Y, _ = model(_t(b, cuda)[..., None], [O.er_graph(P, 0.5, seed=1)] * B,
                 inits=tuple(_t(v, cuda) for v in (y0, U0, d0)))
    with pytest.raises(GuardAdjointError):
        Y.sum().backward()


def test_training_steps_reduce_loss(cuda):
    """A few Adam steps of the reference driver's loop (unfolded_train_new.py:57-82) on synthetic
    data lower loss_final: the module trains end to end on the HIP forward + adjoint."""
    import gnn_dlasso_utils
    import unfolded_DLASSO
    P, m, n, B, K = 5, 64, 256, 128, 10
    torch.manual_seed(0)
    A, b, x = O.make_problem(P, m, n, B, seed=5)
    model = unfolded_DLASSO.DLASSO_unfolded(_t(A, cuda)[None], _args(K)).to(cuda)
    opt = torch.optim.Adam(model.parameters(), lr=5e-2)
    graphs = [O.er_graph(P, 0.5, seed=7)] * B
    bt, label = _t(b, cuda)[..., None], _t(x, cuda)[..., None]
    losses = []
    for _ in range(15):
        Y, _ = model(bt, graphs)
        _, loss_final = gnn_dlasso_utils.compute_loss(Y, label)
        opt.zero_grad()
        loss_final.backward()
        opt.step()
        losses.append(float(loss_final))
    assert np.isfinite(losses).all()
    assert min(losses[-3:]) < losses[0], losses


def test_directed_graph_adjoints_vs_oracle(cuda):
    """A DIRECTED adjacency (successor lists, not symmetric; outside the reference's Erdos-Renyi
    graphs, VERDICT r4 missing #3): the recording forward follows it bit-exactly (a shared-graph
    launch flags it with status bit 16 and the exact recomputation runs), and the adjoint is
    right too: compute_delta is the sum over its visits of (e_p - e_q)(e_p - e_q)^T, symmetric for
    any adjacency (oracle.laplacians; tests/test_oracle.py checks that against torch autograd of
    the literal edge loop). A directed shared graph takes the general adjoint; per-sample graphs
    the fused one. Both against the fp64 oracle adjoint, and through loss.backward()."""
    import networkx as nx
    from dadmm_hip import _lib
    from dadmm_hip.autograd import dadmm_unfolded_apply
    from dadmm_hip.ops import backward_raw
    P, m, n, B, K = 5, 64, 256, 24, 8
    A, b, _ = O.make_problem(P, m, n, B, seed=77)
    g0 = nx.DiGraph()
    g0.add_nodes_from(range(P))
    g0.add_edges_from([(0, 1), (1, 0), (1, 2), (2, 3), (3, 2), (3, 4), (4, 0), (0, 3)])
    y0, U0, d0 = _inits(B, P, n, seed=5)
    rng = np.random.default_rng(3)
    hyp = O.hyp_table((0.5 * rng.standard_normal((K, P, 4))).astype(np.float32), MAXP)
    for graphs in ([g0] * B, [g0] + [O.er_graph(P, 0.5, seed=s) for s in range(B - 1)]):
        op, g, Y, U, st, traj = _record(cuda, A, b, graphs, hyp, y0, U0, d0)
        Yo, Uo, sto, Go, Uro = O.forward_f32_rec(A, b, graphs, hyp, y0, U0, d0)
        assert sto == 0 and st in (0, _lib.STATUS_RECOMPUTE)
        assert not g.symmetric
        assert np.array_equal(Y.cpu().numpy(), Yo)
        assert np.array_equal(traj.Grec[..., :n].cpu().numpy(), Go)
        gYn = np.random.default_rng(9).standard_normal((K, B, P, n)).astype(np.float32)
        want = O.backward_np64(A, graphs, hyp, y0, d0, Yo, Go, Uro, gYn)
        for path in ("auto", "general"):
            dh = backward_raw(op, g, traj, _t(gYn, cuda), path=path)
            _close(dh.cpu().numpy().astype(np.float64), want)
        if g.shared:
            with pytest.raises(ValueError, match="symmetric shared adjacency"):
                backward_raw(op, g, traj, _t(gYn, cuda), path="fused")
        table = _t(hyp, cuda).requires_grad_(True)
        Y2, _ = dadmm_unfolded_apply(op, _t(b, cuda), g, table, _t(y0, cuda), _t(U0, cuda), _t(d0, cuda))
        (Y2 * _t(gYn, cuda)).sum().backward()
        _close(table.grad.cpu().numpy().astype(np.float64), want)
