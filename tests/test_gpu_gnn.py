"""GPU: the GNN-hypernetwork model (DLASSO_GNNHyp3_Progressive) on the per-iteration HIP path.

Bar:
  * the D-ADMM recurrence, given the hyper-parameters the hypernetwork produced in every
    iteration, is BIT-EXACT against oracle.forward_f32_gram (the reference's GNN-model loop,
    gnn_dlasso_models_progressive.py:148-240, in the kernels' operation order), guards included;
  * the hypernetwork (torch on the GPU, fp32) matches the numpy fp64 edge-list restatement of
    GCNConv & co. (oracle/gnn_np.py) within 1e-4 relative — parity unpinned against
    torch_geometric itself (absent);
  * gradients of every parameter through loss.backward() (HIP adjoint of each iteration + gram
    adjoint + torch autograd of the hypernetwork) match torch autograd of a CPU fp64 replay of the
    reference's loop (oracle/ref_torch.gnn_forward_autograd) within 2e-3 of each parameter's
    largest gradient, at a depth (K = 3) where fp32 and fp64 trajectories have not drifted apart.
"""
import argparse

import numpy as np
import pytest
import torch

import oracle as O
from oracle import gnn_np, ref_torch

pytestmark = pytest.mark.gpu


def _args(K, mode="diff", hidden=16, alpha_max=0.1):
    return argparse.Namespace(GHN_iter_num=K, GHyp_hidden=hidden, DADMM_mode=mode,
                              alpha_max=alpha_max, tau_max=0.99, rho_max=0.99, eta_max=0.99)


def _t(x, dev):
    return torch.from_numpy(np.ascontiguousarray(x)).to(dev)


def _setup(dev, P, m, n, B, K, mode, per_sample, seed=0, hidden=16):
    import gnn_dlasso_models_progressive as G
    A, b, x = O.make_problem(P, m, n, B, seed=seed + 5)
    torch.manual_seed(seed)
    model = G.DLASSO_GNNHyp3_Progressive(_t(A, dev)[None], _args(K, mode, hidden)).to(dev)
    if per_sample:
        graphs = [O.connected_er_graph(P, 0.5, seed=seed * 100 + s) for s in range(B)]
    else:
        graphs = [O.er_graph(P, 0.5, seed=seed + 7)] * B
    rng = np.random.default_rng(seed)
    y0, U0, d0 = (1e-2 * rng.standard_normal((3, B, P, n))).astype(np.float32)
    return model, A, b, x, graphs, (y0, U0, d0)


def _recording(model):
    """Record (features, hyp) of every iteration through the model's on_hyp observer (either
    hypernetwork backend)."""
    rec = []

    def hook(AtAy, Atb, out):
        rec.append((AtAy.detach().clone(), Atb.detach().clone(), [o.detach().clone() for o in out]))

    model.on_hyp = hook
    return rec


def _hyp_table(rec, B, H):
    # [K][B][4][H] from each iteration's (alpha, tau, rho, eta) [B, H, 1, 1]
    return np.stack([torch.stack([o[..., 0, 0] for o in r[2]], dim=1).cpu().numpy()
                     for r in rec]).reshape(len(rec), B, 4, H).astype(np.float32)


@pytest.mark.parametrize("mode,per_sample", [("diff", True), ("same", False), ("diff", False)])
def test_recurrence_bit_exact_given_hypernetwork_outputs(cuda, mode, per_sample):
    P, m, n, B, K = 5, 32, 64, 24, 6
    model, A, b, x, graphs, inits = _setup(cuda, P, m, n, B, K, mode, per_sample)
    model.eval()
    rec = _recording(model)
    with torch.no_grad():
        Y, hyp = model(_t(b, cuda)[..., None], graphs, inits=tuple(_t(v, cuda) for v in inits))
    H = 1 if mode == "same" else P
    assert Y.shape == (K, B, P, n, 1) and hyp[0].shape == (B, H, 1, 1)
    assert int(model.last_status.item()) == 0
    table = _hyp_table(rec, B, H)
    Yo, _, st = O.forward_f32_gram(A, b, graphs, table, *inits, variant=1, hyp_mode=1)
    assert st == 0
    assert np.array_equal(Y[..., 0].cpu().numpy(), Yo), np.abs(Y[..., 0].cpu().numpy() - Yo).max()


@pytest.mark.parametrize("P,m,n,B,K", [
    (13, 40, 200, 9, 3),    # n past one 128-column update block, m = 40: a partial gram m-block
    (50, 32, 1024, 2, 2),   # BASELINE configs[4]'s agent count and signal length
    # enough (agent, tile) work for the LDS-resident gram (gram_lds_kernel): three m-blocks (m = 40),
    # n_pad > n, a partial last 16-sample tile and several tiles per workgroup
    (16, 40, 200, 1990, 2),
    # the small-grid gram (gram_kernel<true>: m = 64, n_pad = 256, <= 512 items), partial last tile
    (5, 64, 256, 40, 3),
])
def test_recurrence_bit_exact_larger_shapes(cuda, P, m, n, B, K):
    """The update kernel's column blocks / agent-row pairs and the gram kernel's operand ring and
    m-block skip at shapes beyond the small cases above."""
    model, A, b, x, graphs, inits = _setup(cuda, P, m, n, B, K, "diff", True, seed=3)
    model.eval()
    rec = _recording(model)
    with torch.no_grad():
        Y, _ = model(_t(b, cuda)[..., None], graphs, inits=tuple(_t(v, cuda) for v in inits))
    assert int(model.last_status.item()) == 0
    table = _hyp_table(rec, B, P)
    Yo, _, st = O.forward_f32_gram(A, b, graphs, table, *inits, variant=1, hyp_mode=1)
    assert st == 0
    assert np.array_equal(Y[..., 0].cpu().numpy(), Yo), np.abs(Y[..., 0].cpu().numpy() - Yo).max()


def test_hypernetwork_matches_numpy_restatement(cuda):
    P, m, n, B, K = 5, 32, 64, 12, 2
    model, A, b, x, graphs, inits = _setup(cuda, P, m, n, B, K, "diff", True)
    model.eval()
    rec = _recording(model)
    with torch.no_grad():
        model(_t(b, cuda)[..., None], graphs, inits=tuple(_t(v, cuda) for v in inits))
    sd = {k: v.detach().cpu().numpy().astype(np.float64) for k, v in model.state_dict().items()}
    maxima = tuple(float(np.float32(v)) for v in (0.1, 0.99, 0.99, 0.99))
    for AtAy, Atb, out in rec:
        feats = torch.cat([AtAy, Atb], dim=2).cpu().numpy().astype(np.float64)
        want = gnn_np.hypernetwork(sd, feats, graphs, maxima, False)
        for g, w in zip(out, want):
            g = g[..., 0, 0].cpu().numpy()
            np.testing.assert_allclose(g, w, rtol=1e-4, atol=1e-4 * np.abs(w).max())


def test_configs4_model_vs_numpy_restatement(cuda):
    """BASELINE configs[4]'s model: P = 50 agents, n = 1024, m = 32, GHyp_hidden = 100, per-sample
    connected ER(0.5) graphs, K = 10 iterations, eval mode (fused HIP hypernetwork), with
    non-trivial BatchNorm running statistics. Every iteration's (alpha, tau, rho, eta) against the
    numpy fp64 restatement of GNNHypernetwork3 + decoder + fc (oracle/gnn_np.py) on the features
    the kernels produced, and the whole recurrence bit-exact against oracle.forward_f32_gram
    given those hyper-parameters."""
    P, m, n, B, K = 50, 32, 1024, 3, 10
    model, A, b, x, graphs, inits = _setup(cuda, P, m, n, B, K, "diff", True, seed=4, hidden=100)
    g = torch.Generator().manual_seed(9)
    with torch.no_grad():
        for name, buf in model.named_buffers():
            if name.endswith("running_mean"):
                buf.copy_(0.1 * torch.randn(buf.shape, generator=g))
            elif name.endswith("running_var"):
                buf.copy_(0.5 + torch.rand(buf.shape, generator=g))
        for name, prm in model.named_parameters():
            if ".bn" in name:
                prm.add_(0.05 * torch.randn(prm.shape, generator=g).to(prm.device))
    model.eval()
    rec = _recording(model)
    with torch.no_grad():
        Y, _ = model(_t(b, cuda)[..., None], graphs, inits=tuple(_t(v, cuda) for v in inits))
    assert int(model.last_status.item()) == 0
    assert len(rec) == K
    sd = {k: v.detach().cpu().numpy().astype(np.float64) for k, v in model.state_dict().items()}
    maxima = tuple(float(np.float32(v)) for v in (0.1, 0.99, 0.99, 0.99))
    for AtAy, Atb, out in rec:
        feats = torch.cat([AtAy, Atb], dim=2).cpu().numpy().astype(np.float64)
        want = gnn_np.hypernetwork(sd, feats, graphs, maxima, False)
        for got, w in zip(out, want):
            got = got[..., 0, 0].cpu().numpy()
            np.testing.assert_allclose(got, w, rtol=1e-4, atol=1e-4 * np.abs(w).max())
    table = _hyp_table(rec, B, P)
    Yo, _, st = O.forward_f32_gram(A, b, graphs, table, *inits, variant=1, hyp_mode=1)
    assert st == 0
    assert np.array_equal(Y[..., 0].cpu().numpy(), Yo), np.abs(Y[..., 0].cpu().numpy() - Yo).max()


@pytest.mark.parametrize("P,m,n,B,K,mode,per_sample", [(5, 32, 64, 24, 6, "diff", True),
                                                        (5, 16, 64, 10, 4, "same", False),
                                                        (13, 40, 200, 9, 3, "diff", True)])
def test_hip_graph_replay_matches_eager(cuda, P, m, n, B, K, mode, per_sample):
    """The inference forward replayed from a captured HIP graph (_EvalGraphPlan) equals the
    launch-by-launch forward bit for bit, call after call with new inputs (b, inits, graphs):
    the plan copies them in and writes a fresh Y each time."""
    model, A, b, x, graphs, inits = _setup(cuda, P, m, n, B, K, mode, per_sample, seed=2)
    model.eval()
    outs = {}
    for use in (False, True):
        model.use_hip_graph = use
        res = []
        for call in range(3):
            rng = np.random.default_rng(100 + call)
            y0, U0, d0 = (1e-2 * rng.standard_normal((3, B, P, n))).astype(np.float32)
            bb = b * (1.0 + 0.1 * call)
            gs = graphs if call != 1 else [O.connected_er_graph(P, 0.6, seed=900 + s) for s in range(B)]
            if not per_sample:
                gs = [gs[0]] * B
            with torch.no_grad():
                Y, hyp = model(_t(bb, cuda)[..., None], gs,
                               inits=tuple(_t(v, cuda) for v in (y0, U0, d0)))
            res.append((Y.clone(), [h.clone() for h in hyp], int(model.last_status.item())))
        outs[use] = res
    assert len(model._graph_plans) >= 1
    for (Ye, he, se), (Yg, hg, sg) in zip(outs[False], outs[True]):
        assert se == sg == 0
        assert torch.equal(Ye, Yg)
        assert all(torch.equal(a, c) for a, c in zip(he, hg))
    # fresh outputs: the first call's Y is not overwritten by the later replays
    assert not torch.equal(outs[True][0][0], outs[True][2][0])


def test_hip_graph_back_to_back_replays(cuda):
    """Replays enqueued back to back (no host sync between them), with allocations in between
    (the forward's own RNG draws): every replay starts from zeroed guard flags (status 0) and
    equals the launch-by-launch forward. Regression: a hipMemsetAsync captured into the graph
    replayed with a corrupted fill pattern from the second launch on (all guards set)."""
    from dadmm_hip.ops import draw_inits
    P, m, n, B, K = 5, 32, 64, 24, 5
    model, A, b, x, graphs, _ = _setup(cuda, P, m, n, B, K, "diff", True, seed=3)
    model.eval()
    sets = [tuple(torch.randn(B, P, n, device=cuda) * 1e-2 for _ in range(3)) for _ in range(6)]
    bt = _t(b, cuda)[..., None]
    with torch.no_grad():
        model.use_hip_graph = False
        want = [model(bt, graphs, inits=s)[0].clone() for s in sets]
        model.use_hip_graph = True
        got = []
        for s in sets:
            draw_inits((B, P, n), torch.device(cuda))     # allocation churn between replays
            Y, _ = model(bt, graphs, inits=s)
            got.append((Y, model.last_status))
        model(bt, graphs)                                  # drawn inits
        got_drawn = model.last_status
    torch.cuda.synchronize()
    assert [int(st.item()) for _, st in got] == [0] * len(sets)
    assert int(got_drawn.item()) == 0
    for (Y, _), Ye in zip(got, want):
        assert torch.equal(Y, Ye)


def test_features_are_the_reference_gram_and_atb(cuda):
    """AtAy_0 = AtA @ y0 and Atb = compute_Atx(b) (fp64 check, fp32 tolerance)."""
    P, m, n, B, K = 4, 24, 48, 10, 1
    model, A, b, x, graphs, inits = _setup(cuda, P, m, n, B, K, "diff", False)
    model.eval()
    rec = _recording(model)
    with torch.no_grad():
        model(_t(b, cuda)[..., None], graphs, inits=tuple(_t(v, cuda) for v in inits))
    AtAy, Atb, _ = rec[0]
    A64 = A.astype(np.float64)
    want_g = np.einsum("pri,prj,bpj->bpi", A64, A64, inits[0].astype(np.float64))
    want_b = np.einsum("pri,bpr->bpi", A64, b.astype(np.float64))
    np.testing.assert_allclose(AtAy.cpu().numpy(), want_g, rtol=1e-4, atol=1e-4 * np.abs(want_g).max())
    np.testing.assert_allclose(Atb.cpu().numpy(), want_b, rtol=1e-4, atol=1e-4 * np.abs(want_b).max())


@pytest.mark.parametrize("P,m,n,B", [(4, 24, 48, 10), (16, 32, 256, 96), (50, 32, 1024, 40), (5, 64, 256, 40)])
def test_gram_acc_equals_gram_plus_add(cuda, P, m, n, B):
    """dadmm_gnn_gram_acc (out += A^T A x, the adjoint's one-launch accumulation) == out + the
    gram of x, bit for bit, on the item kernel and the LDS-resident gram; with an addend, the bits
    of a separate add after."""
    from dadmm_hip import _lib
    from dadmm_hip.gnn_ops import GnnRun
    from dadmm_hip.graph import ingest
    model, A, b, x, graphs, inits = _setup(cuda, P, m, n, B, 1, "diff", False)
    bb = _t(b, cuda)
    run = GnnRun(model.operator(), bb, ingest(graphs, P, B, cuda), 1, P, _lib.VARIANT_GNN,
                 *(_t(v, cuda) for v in inits), False)
    ns = run.op.n_store
    g = torch.Generator(device=cuda).manual_seed(P + n)
    xin = torch.zeros(B, P, ns, device=cuda)
    xin[..., :n] = torch.randn(B, P, n, device=cuda, generator=g)
    out0 = torch.zeros(B, P, ns, device=cuda)
    out0[..., :n] = torch.randn(B, P, n, device=cuda, generator=g)
    want = out0 + run.gram(0, x=xin)
    got = run.gram_acc(xin, out0.clone())
    assert torch.equal(got[..., :n], want[..., :n])
    # with the addend (ABI 17: the training backward's loss gradient on y_k): (out + gram) + addend
    add = torch.zeros(B, P, ns, device=cuda)
    add[..., :n] = torch.randn(B, P, n, device=cuda, generator=g)
    got = run.gram_acc(xin, out0.clone(), addend=add)
    assert torch.equal(got[..., :n], (want + add)[..., :n])


@pytest.mark.parametrize("mode,n,directed", [("diff", 32, False), ("same", 32, False),
                                             ("diff", 36, False), ("diff", 32, True)])
def test_backward_matches_cpu_autograd(cuda, mode, n, directed):
    """model.eval() under autograd: gradients of every parameter vs torch autograd of the CPU fp64
    replay. n = 32: the whole forward as one GnnTrainFn node (one library call per iteration);
    n = 36 (n % 16 != 0): HyperTrainFn's launch-by-launch path. The BatchNorm running statistics
    are randomised first (eval mode normalises with them), and must come out unchanged."""
    import gnn_dlasso_models_progressive as G
    from dadmm_hip.graph import ingest
    P, m, B, K = 4, 16, 8, 3
    model, A, b, x, graphs, inits = _setup(cuda, P, m, n, B, K, mode, True, hidden=8)
    if directed:   # successor lists (VERDICT r4 missing #3: the step adjoint refused them)
        import networkx as nx
        rng = np.random.default_rng(4)
        graphs = []
        for _ in range(B):
            dg = nx.DiGraph()
            dg.add_nodes_from(range(P))
            dg.add_edges_from((p, q) for p in range(P) for q in range(P) if p != q and rng.random() < 0.5)
            graphs.append(dg)
    gen = torch.Generator().manual_seed(11)
    enc = model.encoder
    with torch.no_grad():
        for bn in (enc.bn1, enc.bn2, enc.bn3, enc.bn4, enc.bn5):
            bn.running_mean.copy_(0.3 * torch.randn(bn.num_features, generator=gen))
            bn.running_var.copy_(0.5 + torch.rand(bn.num_features, generator=gen))
    before = {k: v.clone() for k, v in model.state_dict().items() if "running" in k}
    model.eval()
    gY = torch.randn(K, B, P, n, 1, generator=torch.Generator().manual_seed(2))
    Y, _ = model(_t(b, cuda)[..., None], graphs, inits=tuple(_t(v, cuda) for v in inits))
    # eval mode with autograd (VERDICT r3 missing #4, r4 missing #2): the HIP training kernels
    # with BatchNorm on the running statistics and no dropout, forward and backward
    assert model.last_backend == "hip-eval-grad"
    (Y * gY.to(cuda)).sum().backward()
    got = {k: p.grad.detach().cpu().numpy() for k, p in model.named_parameters()}
    after = model.state_dict()
    assert all(torch.equal(before[k], after[k]) for k in before)

    cpu = G.DLASSO_GNNHyp3_Progressive(torch.from_numpy(A)[None], _args(K, mode, 8)).double()
    cpu.load_state_dict({k: v.cpu() for k, v in model.state_dict().items()})
    cpu.eval()
    a_hat = G.normalized_adjacency(ingest(graphs, P, B, "cpu").nbr, P, torch.float64)
    Yc, _ = ref_torch.gnn_forward_autograd(cpu, A, b, graphs, *inits, K=K, a_hat=a_hat)
    np.testing.assert_allclose(Y[..., 0].detach().cpu().numpy(), Yc.detach().numpy(), rtol=1e-4,
                               atol=1e-4)
    (Yc * gY[..., 0].double()).sum().backward()
    for k, p in cpu.named_parameters():
        w = p.grad.numpy()
        scale = np.abs(w).max()
        assert scale > 0, k
        err = np.abs(got[k] - w).max() / scale
        assert err <= 2e-3, (k, err)


def test_guard_on_nonfinite_y0_bit_exact(cuda):
    P, m, n, B, K = 4, 16, 32, 8, 4
    model, A, b, x, graphs, inits = _setup(cuda, P, m, n, B, K, "diff", True)
    model.eval()
    y0, U0, d0 = inits
    y0 = y0.copy()
    y0[3, 2, 7] = np.inf
    rec = _recording(model)
    with torch.no_grad():
        Y, _ = model(_t(b, cuda)[..., None], graphs, inits=tuple(_t(v, cuda) for v in (y0, U0, d0)))
    st = int(model.last_status.item())
    table = _hyp_table(rec, B, P)
    Yo, _, sto = O.forward_f32_gram(A, b, graphs, table, y0, U0, d0, variant=1, hyp_mode=1)
    assert st == sto and st & 1
    assert np.array_equal(Y[..., 0].cpu().numpy(), Yo)


@pytest.mark.parametrize("k_bad,shape", [(1, (4, 16, 32, 8, 5)), (3, (4, 16, 32, 8, 5)),
                                         (1, (5, 64, 256, 24, 4))])
def test_guard_on_nonfinite_ynext_bit_exact(cuda, k_bad, shape):
    """A NaN alpha from the hypernetwork at iteration k_bad makes y_next non-finite: the
    reference keeps y_k and appends it (gnn_dlasso_models_progressive.py:235-237), so Y[k_bad]
    must hold y_k, also when k_bad < K - 1 (the slot is rewritten by the next iteration). The
    m = 64, n = 256 shape runs the small-grid gram, whose x source then takes the flag walk."""
    P, m, n, B, K = shape
    model, A, b, x, graphs, inits = _setup(cuda, P, m, n, B, K, "diff", True)
    model.eval()
    model.hyper_backend = "torch"
    orig = model.hypernetwork
    calls = []

    def patched(*args):
        out = orig(*args)
        if len(calls) == k_bad:
            out[0][2, 1] = float("nan")   # alpha of sample 2, agent 1
        calls.append(1)
        return out

    model.hypernetwork = patched
    rec = _recording(model)
    with torch.no_grad():
        Y, _ = model(_t(b, cuda)[..., None], graphs, inits=tuple(_t(v, cuda) for v in inits))
    st = int(model.last_status.item())
    table = _hyp_table(rec, B, P)
    assert np.isnan(table[k_bad]).any()
    y0, U0, d0 = inits
    Yo, _, sto = O.forward_f32_gram(A, b, graphs, table, y0, U0, d0, variant=1, hyp_mode=1)
    assert st == sto and st & 8
    Yg = Y[..., 0].cpu().numpy()
    assert np.isfinite(Yg).all()
    assert np.array_equal(Yg, Yo)


@pytest.mark.parametrize("k_bad", [0, 2])
def test_guard_on_nan_gradient_bit_exact(cuda, k_bad):
    """A NaN tau at iteration k_bad makes the gradient NaN: the reference zeroes the whole batch's
    gradient (gnn_dlasso_models_progressive.py:216-218). The fused step forms the gradient
    optimistically and its resolve launch redoes the update with G = 0; Y must match the oracle."""
    P, m, n, B, K = 4, 16, 32, 8, 4
    model, A, b, x, graphs, inits = _setup(cuda, P, m, n, B, K, "diff", True)
    model.eval()
    model.hyper_backend = "torch"
    orig = model.hypernetwork
    calls = []

    def patched(*args):
        out = orig(*args)
        if len(calls) == k_bad:
            out[1][5, 2] = float("nan")   # tau of sample 5, agent 2
        calls.append(1)
        return out

    model.hypernetwork = patched
    rec = _recording(model)
    with torch.no_grad():
        Y, _ = model(_t(b, cuda)[..., None], graphs, inits=tuple(_t(v, cuda) for v in inits))
    st = int(model.last_status.item())
    table = _hyp_table(rec, B, P)
    assert np.isnan(table[k_bad]).any()
    y0, U0, d0 = inits
    Yo, _, sto = O.forward_f32_gram(A, b, graphs, table, y0, U0, d0, variant=1, hyp_mode=1)
    assert st == sto and st & 4
    assert np.array_equal(Y[..., 0].cpu().numpy(), Yo)


def test_train_mode_step_updates_bn_and_trains(cuda):
    """train(): dropout on, per-sample BatchNorm statistics, running stats updated B*K times per
    forward; loss.backward() + AdamW step run (progressive driver's loop, :196-214)."""
    import gnn_dlasso_utils
    P, m, n, B, K = 5, 32, 64, 16, 4
    model, A, b, x, graphs, inits = _setup(cuda, P, m, n, B, K, "diff", True)
    model.train()
    opt = torch.optim.AdamW(model.parameters(), lr=1e-3)
    nbt0 = int(model.encoder.bn1.num_batches_tracked)
    Y, hyp = model(_t(b, cuda)[..., None], graphs, training_iterations=K + 2)
    assert Y.shape[0] == K + 2                  # training_iterations is not capped by self.K
    assert int(model.encoder.bn1.num_batches_tracked) == nbt0 + B * (K + 2)
    _, loss_final = gnn_dlasso_utils.compute_loss(Y, _t(x, cuda)[..., None])
    opt.zero_grad()
    loss_final.backward()
    torch.nn.utils.clip_grad_norm_(model.parameters(), 100.0)
    grads = [p.grad for p in model.parameters() if p.grad is not None]
    assert grads and all(torch.isfinite(g).all() for g in grads)
    opt.step()
