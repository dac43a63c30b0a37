"""The drop-in modules on CPU tensors (the reference's default device, configurations.py:108):
``dadmm_cpu`` runs the reference's op sequence in torch eager ops. Checked against the oracle's
literal fp32 replay of unfolded_DLASSO.py:34-110 (oracle/ref_torch.forward: per-agent Gram
matmuls, Python compute_delta, the guards), its fp64 restatement, and fp64 torch autograd of the
reference ops for the gradients. Tolerances: fp32 rounding (delta is a matrix product here, a
sequential add chain in the reference)."""
import argparse
import copy

import numpy as np
import pytest
import torch

import oracle as O
from oracle import ref_torch as RT


def _args(K, mode="diff", hidden=8):
    return argparse.Namespace(GHN_iter_num=K, DADMM_mode=mode, alpha_max=0.1, tau_max=0.99, rho_max=0.99,
                              eta_max=0.99, max_penalty_threshold=0.8, penalty_reduction_factor=0.95,
                              GHyp_hidden=hidden)


def _inits(B, P, n, seed):
    g = torch.Generator().manual_seed(seed)
    return tuple(1e-2 * torch.randn(B, P, n, 1, generator=g) for _ in range(3))


def _close(got, want, rel=2e-5):
    got, want = np.asarray(got, np.float64), np.asarray(want, np.float64)
    scale = max(1.0, float(np.abs(want).max()))
    err = float(np.abs(got - want).max())
    assert err <= rel * scale, f"max |got - want| {err:.3e} > {rel:.0e} x {scale:.3e}"


@pytest.mark.parametrize("P,m,n,B,K,mode,per_sample", [(5, 20, 32, 6, 8, "diff", True),
                                                       (4, 10, 16, 3, 6, "same", False),
                                                       (7, 12, 24, 2, 25, "diff", True)])
def test_unfolded_cpu_matches_reference_ops(P, m, n, B, K, mode, per_sample):
    import unfolded_DLASSO as U
    A, b, _ = O.make_problem(P, m, n, B, seed=P + K)
    graphs = ([O.connected_er_graph(P, 0.5, seed=10 + s) for s in range(B)] if per_sample
              else [O.er_graph(P, 0.5, seed=3)] * B)
    mod = U.DLASSO_unfolded(torch.from_numpy(A)[None], _args(K, mode)).eval()
    with torch.no_grad():
        mod.seq_hyp.param.copy_(0.3 * torch.randn(mod.seq_hyp.param.shape, generator=torch.Generator().manual_seed(1)))
    inits = _inits(B, P, n, seed=K)
    with torch.no_grad():
        Y, hyp = mod(torch.from_numpy(b)[..., None], graphs, inits=inits)
    assert Y.shape == (K, B, P, n, 1) and Y.device.type == "cpu"
    tab = mod.seq_hyp.table(K).detach().numpy()
    assert torch.equal(hyp, torch.from_numpy(tab[K - 1])[..., None])
    y0, U0, d0 = (t[..., 0].numpy() for t in inits)
    ref = RT.forward(A, b, graphs, tab, y0, U0, d0)
    if K <= 8:   # (over more iterations sign(y) near 0 amplifies fp32 rounding: the MSE bound below)
        _close(Y[..., 0].numpy(), ref)
    Y64, _ = O.forward_np64(A, b, graphs, tab, y0, U0, d0)
    for want in (ref[-1], Y64[-1]):   # north_star's final-iterate tolerance
        assert float(np.mean((Y[-1, ..., 0].numpy() - want) ** 2)) <= 1e-5
    assert int(mod.last_status[0]) == 0


def test_unfolded_cpu_guards_follow_the_reference():
    """A NaN in y0 resets y at k = 0 (unfolded_DLASSO.py:55-58), as the literal replay does."""
    import unfolded_DLASSO as U
    P, m, n, B, K = 4, 10, 16, 3, 5
    A, b, _ = O.make_problem(P, m, n, B, seed=2)
    graphs = [O.connected_er_graph(P, 0.5, seed=s) for s in range(B)]
    mod = U.DLASSO_unfolded(torch.from_numpy(A)[None], _args(K)).eval()
    y0, U0, d0 = _inits(B, P, n, seed=3)
    y0[1, 2, 5] = float("nan")
    with torch.no_grad():
        Y, _ = mod(torch.from_numpy(b)[..., None], graphs, inits=(y0, U0, d0))
    assert int(mod.last_status[0]) & 1
    tab = mod.seq_hyp.table(K).detach().numpy()
    _close(Y[..., 0].numpy(), RT.forward(A, b, graphs, tab, *(t[..., 0].numpy() for t in (y0, U0, d0))))


def test_unfolded_cpu_default_inits_are_the_reference_draws():
    """Without inits the forward draws randn((B,P,n,1)) * 1e-2 three times, in the reference's
    order (:49-51), from torch's CPU generator."""
    import unfolded_DLASSO as U
    P, m, n, B, K = 3, 8, 12, 4, 4
    A, b, _ = O.make_problem(P, m, n, B, seed=4)
    graphs = [O.er_graph(P, 0.6, seed=1)] * B
    mod = U.DLASSO_unfolded(torch.from_numpy(A)[None], _args(K)).eval()
    torch.manual_seed(123)
    with torch.no_grad():
        Y, _ = mod(torch.from_numpy(b)[..., None], graphs)
    torch.manual_seed(123)
    draws = [torch.randn((B, P, n, 1)) * 1e-2 for _ in range(3)]
    tab = mod.seq_hyp.table(K).detach().numpy()
    _close(Y[..., 0].numpy(), RT.forward(A, b, graphs, tab, *(t[..., 0].numpy() for t in draws)))


def test_unfolded_cpu_gradient_matches_reference_autograd():
    """d<R, Y>/d table through the CPU path (fp32) vs fp64 torch autograd of the reference ops
    (oracle/ref_torch.forward_autograd); and loss.backward() reaches seq_hyp.param."""
    import dadmm_cpu
    import unfolded_DLASSO as U
    from dadmm_hip.graph import ingest
    P, m, n, B, K = 5, 16, 24, 4, 6
    A, b, _ = O.make_problem(P, m, n, B, seed=8)
    graphs = [O.connected_er_graph(P, 0.5, seed=30 + s) for s in range(B)]
    mod = U.DLASSO_unfolded(torch.from_numpy(A)[None], _args(K)).train()
    tab = mod.seq_hyp.table(K).detach()
    inits = _inits(B, P, n, seed=5)
    R = torch.randn(K, B, P, n, generator=torch.Generator().manual_seed(6))
    t32 = tab.clone().requires_grad_(True)
    gb = ingest(graphs, P, B, torch.device("cpu"))
    Y, _ = dadmm_cpu.unfolded_forward(torch.from_numpy(A)[None], torch.from_numpy(b), gb, t32, K, inits)
    (Y * R).sum().backward()
    t64 = tab.double().requires_grad_(True)
    Y64 = RT.forward_autograd(A, b, graphs, t64, *(t[..., 0].numpy() for t in inits))[0]
    (Y64 * R.double()).sum().backward()
    _close(t32.grad.numpy(), t64.grad.numpy(), rel=1e-3)
    Ym, _ = mod(torch.from_numpy(b)[..., None], graphs, inits=inits)
    (Ym[..., 0] * R).sum().backward()
    assert mod.seq_hyp.param.grad is not None and torch.isfinite(mod.seq_hyp.param.grad).all()


@pytest.mark.parametrize("mode", ["diff", "same"])
def test_gnn_cpu_matches_reference_autograd_ops(mode):
    """DLASSO_GNNHyp3_Progressive on CPU tensors (eval) vs the reference's GNN loop in fp64 torch
    ops (oracle/ref_torch.gnn_forward_autograd with the same hypernetwork modules in fp64);
    train mode runs forward + compute_loss + backward."""
    import gnn_dlasso_models_progressive as GM
    import gnn_dlasso_utils
    from dadmm_hip.graph import ingest
    P, m, n, B, K = 5, 12, 16, 4, 3
    A, b, x = O.make_problem(P, m, n, B, seed=9)
    graphs = [O.connected_er_graph(P, 0.5, seed=40 + s) for s in range(B)]
    model = GM.DLASSO_GNNHyp3_Progressive(torch.from_numpy(A)[None], _args(K, mode)).eval()
    inits = _inits(B, P, n, seed=7)
    bt = torch.from_numpy(b)[..., None]
    with torch.no_grad():
        Y, hyp = model(bt, graphs, inits=inits)
    assert model.last_backend == "cpu" and Y.shape == (K, B, P, n, 1)
    gb = ingest(graphs, P, B, torch.device("cpu"))
    a_hat = GM.normalized_adjacency(gb.nbr, P, dtype=torch.float64)
    m64 = copy.deepcopy(model).double()
    with torch.no_grad():
        Y64, h64 = RT.gnn_forward_autograd(m64, A, b, graphs, *(t[..., 0].numpy() for t in inits), K, a_hat)
    _close(Y[..., 0].numpy(), Y64.numpy(), rel=1e-4)
    for got, want in zip(hyp, h64):
        _close(got.numpy(), want.numpy(), rel=1e-4)
    model.train()
    Y, _ = model(bt, graphs, inits=inits)
    _, loss = gnn_dlasso_utils.compute_loss(Y, torch.from_numpy(x)[..., None])
    loss.backward()
    grads = [p.grad for p in model.parameters() if p.requires_grad]
    assert all(g is not None and torch.isfinite(g).all() for g in grads)


@pytest.mark.parametrize("driver", ["train_unfolded", "train_gnn"])
def test_drivers_train_on_the_cpu(driver, tmp_path, monkeypatch):
    """--device cpu (the reference's default, configurations.py:108): both drivers run an epoch
    on the CPU path (the GNN driver draws its graphs with networkx there, as the reference does)."""
    import importlib
    monkeypatch.chdir(tmp_path)
    mod = importlib.import_module(driver)
    args = ["--device", "cpu", "--P", "4", "--m", "8", "--n", "16", "--GHN_iter_num", "3",
            "--batch_size", "8", "--train_size", "16", "--test_size", "8", "--num_epochs", "1", "--seed", "2"]
    if driver == "train_gnn":
        args += ["--GHyp_hidden", "8"]
    mod.main(args)
