"""GPU: more than 64 agents (VERDICT r3 missing #1 / next #7). The reference walks any graph
(unfolded_DLASSO.py:111-140, gnn_dlasso_models_progressive.py:245-276); beyond the 64 agents a
uint64 neighbour mask describes, a batch is ingested as degrees + reference-order visit lists (a
CSR form of the adjacency) + a dense adjacency for the GCN normalisation (dadmm_hip/graph.py
_batch_wide), and runs on the non-fused kernels: the tiled per-iteration launches with the gated
stepwise recomputation, the stepwise path, the general adjoint, and the GNN model's per-iteration
kernels with the fused inference hypernetwork.

Bar: bit-exact (np.array_equal) against oracle.forward_f32 / forward_f32_rec /
forward_f32_gram (the CSR-driven C restatement) on every iterate, U_K and the recorded
trajectory; the adjoint within 1e-5 of oracle.backward_np64 along its own trajectory; the
hypernetwork within 1e-4 of oracle/gnn_np.py (parity vs torch_geometric unpinned)."""
import argparse

import numpy as np
import pytest
import torch

import oracle as O

pytestmark = pytest.mark.gpu

MAXP = [0.1, 0.99, 0.99, 0.99]


def _t(x, dev):
    return torch.from_numpy(np.ascontiguousarray(x)).to(dev)


def _inits(B, P, n, seed):
    rng = np.random.default_rng(seed)
    return (1e-2 * rng.standard_normal((3, B, P, n))).astype(np.float32)


def _graphs(P, B, prob, per_sample, seed):
    if per_sample:
        return [O.connected_er_graph(P, prob, seed=seed + s) for s in range(B)]
    return [O.er_graph(P, prob, seed=seed)] * B


@pytest.mark.parametrize("path", ["auto", "stepwise", "tiled"])
@pytest.mark.parametrize("P,m,n,B,K,prob,per_sample,variant,H", [
    (80, 16, 64, 6, 5, 0.1, True, 0, 80),     # per-sample connected ER graphs on 80 agents
    (80, 24, 128, 5, 4, 0.3, False, 1, 1),    # one shared graph, GNN clamps, 'same' mode
    (100, 8, 32, 3, 3, 0.05, True, 0, 100),
])
def test_wide_forward_bit_exact(cuda, path, P, m, n, B, K, prob, per_sample, variant, H):
    from dadmm_hip import PreparedOperator, forward_raw, ingest
    A, b, _ = O.make_problem(P, m, n, B, seed=P + n)
    graphs = _graphs(P, B, prob, per_sample, seed=3000)
    y0, U0, d0 = _inits(B, P, n, seed=K)
    rng = np.random.default_rng(P * K)
    hyp = O.hyp_table((0.5 * rng.standard_normal((K, H, 4))).astype(np.float32), MAXP)
    g = ingest(graphs, P, B, cuda)
    assert g.wide and not g.fused_ok and g.symmetric
    op = PreparedOperator(_t(A, cuda))
    Y, U, st = forward_raw(op, _t(b, cuda), g, _t(hyp, cuda), _t(y0, cuda), _t(U0, cuda),
                           _t(d0, cuda), variant=variant, want_U=True, path=path)
    torch.cuda.synchronize()
    Yo, Uo, sto = O.forward_f32(A, b, graphs, hyp, y0, U0, d0, variant=variant)
    assert int(st.item()) == sto == 0
    assert np.array_equal(Y.cpu().numpy(), Yo), f"max |diff| {np.abs(Y.cpu().numpy() - Yo).max()}"
    assert np.array_equal(U.cpu().numpy(), Uo)


def test_wide_guard_fired_exact(cuda):
    """A NaN in b at P = 80: the batch-global gradient guard (unfolded_DLASSO.py:84-86) fires and
    the gated stepwise recomputation reproduces the reference's reset exactly."""
    from dadmm_hip import PreparedOperator, forward_raw, ingest
    P, m, n, B, K = 80, 16, 64, 4, 3
    A, b, _ = O.make_problem(P, m, n, B, seed=8)
    b[2, 70, 3] = np.nan
    graphs = _graphs(P, B, 0.1, True, seed=3100)
    y0, U0, d0 = _inits(B, P, n, seed=9)
    hyp = O.hyp_table(np.zeros((K, P, 4), np.float32), MAXP)
    op = PreparedOperator(_t(A, cuda))
    Y, U, st = forward_raw(op, _t(b, cuda), ingest(graphs, P, B, cuda), _t(hyp, cuda), _t(y0, cuda),
                           _t(U0, cuda), _t(d0, cuda), want_U=True)
    torch.cuda.synchronize()
    Yo, Uo, sto = O.forward_f32(A, b, graphs, hyp, y0, U0, d0)
    assert sto != 0 and int(st.item()) == sto
    assert np.array_equal(Y.cpu().numpy(), Yo, equal_nan=True)
    assert np.array_equal(U.cpu().numpy(), Uo, equal_nan=True)


def test_wide_module_forward_and_backward(cuda):
    """DLASSO_unfolded at P = 80 through the module API (networkx graph_list, one shared graph):
    the forward bit-exact, and loss_final.backward() reaches seq_hyp.param through the general
    adjoint (two waves per workgroup at this agent count), matching oracle.backward_np64 chained
    through the hyper-parameter table."""
    import unfolded_DLASSO
    from dadmm_hip import PreparedOperator, forward_raw, ingest
    from dadmm_hip.ops import backward_raw
    P, m, n, B, K = 80, 16, 64, 5, 4
    A, b, x = O.make_problem(P, m, n, B, seed=12)
    graphs = _graphs(P, B, 0.1, True, seed=3200)
    y0, U0, d0 = _inits(B, P, n, seed=13)
    rng = np.random.default_rng(14)
    hyp = O.hyp_table((0.5 * rng.standard_normal((K, P, 4))).astype(np.float32), MAXP)
    op = PreparedOperator(_t(A, cuda))
    g = ingest(graphs, P, B, cuda)
    Y, U, st, traj = forward_raw(op, _t(b, cuda), g, _t(hyp, cuda), _t(y0, cuda), _t(U0, cuda),
                                 _t(d0, cuda), want_U=True, record=True)
    torch.cuda.synchronize()
    Yo, Uo, sto, Go, Uro = O.forward_f32_rec(A, b, graphs, hyp, y0, U0, d0)
    assert int(st.item()) == sto == 0
    assert np.array_equal(Y.cpu().numpy(), Yo)
    assert np.array_equal(traj.Grec[..., :n].cpu().numpy(), Go)
    assert np.array_equal(traj.Urec[..., :n].cpu().numpy(), Uro)
    gY = np.random.default_rng(15).standard_normal((K, B, P, n)).astype(np.float32)
    dh = backward_raw(op, g, traj, _t(gY, cuda)).cpu().numpy().astype(np.float64)
    want = O.backward_np64(A, graphs, hyp, y0, d0, Yo, Go, Uro, gY)
    err = np.abs(dh - want)
    assert (err <= 1e-5 * np.abs(want).max() + 1e-5 * np.abs(want)).all(), err.max()

    args = argparse.Namespace(GHN_iter_num=K, DADMM_mode="diff", alpha_max=0.1, tau_max=0.99,
                              rho_max=0.99, eta_max=0.99, max_penalty_threshold=0.8,
                              penalty_reduction_factor=0.95)
    model = unfolded_DLASSO.DLASSO_unfolded(_t(A, cuda)[None], args).to(cuda)
    G = O.er_graph(P, 0.1, seed=3300)
    Ym, _ = model(_t(b, cuda)[..., None], [G] * B, inits=tuple(_t(v, cuda) for v in (y0, U0, d0)))
    table = model.hyp_table(K).detach().cpu().numpy()
    Ymo, _, _ = O.forward_f32(A, b, [G] * B, table, y0, U0, d0)
    assert np.array_equal(Ym[..., 0].detach().cpu().numpy(), Ymo)
    import gnn_dlasso_utils
    _, lf = gnn_dlasso_utils.compute_loss(Ym, _t(x, cuda)[..., None])
    lf.backward()
    gp = model.seq_hyp.param.grad
    assert gp is not None and torch.isfinite(gp).all() and gp.abs().max() > 0


def test_wide_gnn_model_eval(cuda):
    """DLASSO_GNNHyp3_Progressive at P = 80 (per-sample connected graphs, eval, fused inference
    hypernetwork on the per-iteration path and the graphed replay): every iteration's
    hyper-parameters vs oracle/gnn_np.py and the recurrence bit-exact vs forward_f32_gram."""
    import gnn_dlasso_models_progressive as GM
    from oracle import gnn_np
    P, m, n, B, K = 80, 16, 64, 3, 3
    A, b, _ = O.make_problem(P, m, n, B, seed=21)
    torch.manual_seed(22)
    args = argparse.Namespace(GHN_iter_num=K, GHyp_hidden=16, DADMM_mode="diff", alpha_max=0.1,
                              tau_max=0.99, rho_max=0.99, eta_max=0.99)
    model = GM.DLASSO_GNNHyp3_Progressive(_t(A, cuda)[None], args).to(cuda).eval()
    graphs = _graphs(P, B, 0.1, True, seed=3400)
    inits = _inits(B, P, n, seed=23)
    rec = []
    model.on_hyp = lambda AtAy, Atb, out: rec.append(
        (torch.cat([AtAy, Atb], dim=2).cpu(), torch.stack([o[:, :, 0, 0] for o in out], dim=1).cpu()))
    with torch.no_grad():
        Y, _ = model(_t(b, cuda)[..., None], graphs, inits=tuple(_t(v, cuda) for v in inits))
    assert model.last_backend == "hip-eval"
    assert int(model.last_status.item()) == 0 and len(rec) == K
    sd = {k: v.detach().cpu().numpy().astype(np.float64) for k, v in model.state_dict().items()}
    maxima = tuple(float(np.float32(v)) for v in MAXP)
    for k in range(K):
        feats, got = rec[k]
        want = gnn_np.hypernetwork(sd, feats.numpy().astype(np.float64), graphs, maxima, False)
        for c in range(4):
            w = want[c][..., 0, 0] if want[c].ndim == 4 else want[c]
            np.testing.assert_allclose(got[:, c].numpy(), w.reshape(got[:, c].shape), rtol=1e-4,
                                       atol=1e-4 * np.abs(w).max(), err_msg=f"iteration {k}, c {c}")
    table = np.stack([r[1].numpy() for r in rec]).astype(np.float32)
    Yo, _, st = O.forward_f32_gram(A, b, graphs, table, *inits, variant=1, hyp_mode=1)
    assert st == 0
    Yg = Y[..., 0].cpu().numpy()
    assert np.array_equal(Yg, Yo), f"max |diff| {np.abs(Yg - Yo).max():.3e}"
    model.on_hyp = None
    with torch.no_grad():
        Y2, _ = model(_t(b, cuda)[..., None], graphs, inits=tuple(_t(v, cuda) for v in inits))
    assert model.last_backend == "hip-eval-graph"
    assert np.array_equal(Y2[..., 0].cpu().numpy(), Yg)
