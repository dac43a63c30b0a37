"""GPU: the fused inference-mode hypernetwork kernels (dadmm_hyper_*, csrc/dadmm_hyper.hip).

Bar: each launch against a plain torch fp32 reference of the same op on the same device (the
reference's own eager ops: nn.Linear, GCNConv restated densely, F.leaky_relu, BatchNorm1d in eval,
LayerNorm, sigmoid + clamps), within fp32 GEMM rounding: |got - want| <= 1e-5 * (1 + |want|) +
2e-6 * sqrt(K) * max|want| — the kernels sum in a fixed MFMA order, torch's hipBLASLt in another.
Shapes cover rows / columns that are not multiples of the 32-row / 64-column tiles, K tails, the
split cat(AtAy, Atb) input (n % 16 == 0) and the concatenated one (n = 100), split-K decoder
linears up to configs[4]'s K = P * 4h = 20000, per-sample and shared graphs, P = 1..50 and both
head modes. Model
level: DLASSO_GNNHyp3_Progressive in eval + no_grad (fused backend) against the same model on the
torch backend, iteration by iteration on identical features, and against the numpy fp64
edge-list restatement of GCNConv (test_gpu_gnn.py::test_hypernetwork_matches_numpy_restatement).
"""
import argparse
import ctypes

import numpy as np
import pytest
import torch
import torch.nn.functional as F

import oracle as O

pytestmark = pytest.mark.gpu


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _s():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _close(got, want, K):
    got, want = got.double(), want.double()
    tol = 1e-5 * (1 + want.abs()) + 2e-6 * np.sqrt(K) * want.abs().max()
    err = (got - want).abs() - tol
    assert torch.isfinite(got).all()
    assert err.max() <= 0, float(((got - want).abs()).max())


@pytest.fixture(scope="module")
def L():
    from dadmm_hip import _lib
    return _lib.load()


# the last three shapes take the LDS-DMA operand ring (>= 32 k-steps per workgroup) with 128-row
# (9000 rows) and 64-row (6000 rows) tiles, a K tail (K % 16 = 8) and a split input
@pytest.mark.parametrize("rows,K,N,K1", [(1, 4, 4, 4), (17, 20, 20, 20), (300, 100, 200, 100),
                                         (1024, 2000, 400, 2000), (1000, 512, 100, 256),
                                         (129, 36, 65, 16), (9000, 1000, 400, 1000),
                                         (9000, 1032, 400, 512), (6000, 600, 400, 600)])
def test_linear_matches_torch(cuda, L, rows, K, N, K1):
    g = torch.Generator(device=cuda).manual_seed(rows + K)
    x = torch.randn(rows, K, device=cuda, generator=g)
    W = torch.randn(N, K, device=cuda, generator=g) / np.sqrt(K)
    bias = torch.randn(N, device=cuda, generator=g)
    y = torch.full((rows, N + 3), 7.0, device=cuda)          # ldy > N: the pad column survives
    if K1 < K:   # split input: columns [0, K1) and [K1, K) from separate, padded buffers
        x1 = torch.zeros(rows, K1 + 4, device=cuda)
        x2 = torch.zeros(rows, K - K1 + 8, device=cuda)
        x1[:, :K1], x2[:, :K - K1] = x[:, :K1], x[:, K1:]
        rc = L.dadmm_hyper_linear(rows, K, N, _p(x1), K1 + 4, K1, _p(x2), K - K1 + 8, _p(W),
                                  _p(bias), _p(y), N + 3, _s())
    else:
        rc = L.dadmm_hyper_linear(rows, K, N, _p(x), K, K, None, 0, _p(W), _p(bias), _p(y), N + 3,
                                  _s())
    assert rc == 0, L.dadmm_last_error()
    _close(y[:, :N], F.linear(x, W, bias), K)
    assert (y[:, N:] == 7.0).all()


def _ahat(nbr, P, dev):
    import gnn_dlasso_models_progressive as G
    return G.normalized_adjacency(nbr, P).to(dev).contiguous()


@pytest.mark.parametrize("B,P,K,N,per_sample", [(7, 5, 512, 100, True), (33, 5, 100, 200, False),
                                                (9, 16, 200, 400, True), (3, 50, 400, 400, True),
                                                (1, 1, 8, 4, False), (40, 2, 64, 36, True),
                                                (512, 50, 1024, 100, True),    # DMA ring, 128 rows
                                                # gcn32_kernel (32x32x2 MFMA, 256-row tiles): 400-wide
                                                # layers of configs[4], a K tail (100 % 16), shared graph
                                                (1024, 50, 400, 400, True), (1024, 50, 100, 200, True),
                                                (2000, 16, 200, 200, False),
                                                # small grids (the inference layer never splits K)
                                                (60, 5, 400, 400, True), (9, 16, 200, 400, False)])
def test_gcn_layer_matches_torch(cuda, L, B, P, K, N, per_sample):
    from dadmm_hip.graph import ingest
    G = B if per_sample else 1
    graphs = [O.connected_er_graph(P, 0.4, seed=31 * i + P) for i in range(G)] if P > 1 else \
        [O.er_graph(1, 0.5, seed=0)]
    gb = ingest(graphs, P, G, cuda)
    ahat = _ahat(gb.nbr.reshape(G, P), P, cuda)
    gen = torch.Generator(device=cuda).manual_seed(B * P + N)
    x = torch.randn(B * P, K, device=cuda, generator=gen)
    W = torch.randn(N, K, device=cuda, generator=gen) / np.sqrt(K)
    bias, rm, bw, bb = (torch.randn(N, device=cuda, generator=gen) for _ in range(4))
    rv = torch.rand(N, device=cuda, generator=gen) + 0.5
    y = torch.empty(B * P, N, device=cuda)
    rc = L.dadmm_hyper_gcn(B, P, K, N, _p(x), K, K, None, 0, _p(W), _p(bias), _p(ahat),
                           int(per_sample), _p(rm), _p(rv), _p(bw), _p(bb), 1e-5, 0.01, _p(y), N,
                           _s())
    assert rc == 0, L.dadmm_last_error()
    z = torch.matmul(ahat, F.linear(x, W).view(B, P, N)) + bias          # GCNConv (dense)
    z = F.leaky_relu(z).reshape(B * P, N)
    want = F.batch_norm(z, rm, rv, bw, bb, False, 0.0, 1e-5)
    _close(y, want, K)


@pytest.mark.parametrize("rows,K,N,ldy", [(1280, 400, 256, 256), (37, 100, 48, 52), (20480, 400, 256, 256)])
def test_linear_ex_addend_in_place_is_linear_plus_add(cuda, L, rows, K, N, ldy):
    """dadmm_hyper_linear_ex with addend == y (the GNN adjoint's dAtAy accumulation) equals
    dadmm_hyper_linear followed by an add, bit for bit; columns past N are left alone."""
    gen = torch.Generator(device=cuda).manual_seed(rows + K)
    x = torch.randn(rows, K, device=cuda, generator=gen)
    W = torch.randn(N, K, device=cuda, generator=gen) / K ** 0.5
    y0 = torch.randn(rows, ldy, device=cuda, generator=gen)
    lin = torch.zeros(rows, ldy, device=cuda)
    assert L.dadmm_hyper_linear(rows, K, N, _p(x), K, K, None, 0, _p(W), None, _p(lin), ldy, _s()) == 0
    want = y0.clone()
    want[:, :N] += lin[:, :N]
    got = y0.clone()
    rc = L.dadmm_hyper_linear_ex(rows, K, N, _p(x), K, K, None, 0, _p(W), None, _p(got), ldy, _p(got), ldy,
                                 _s())
    assert rc == 0, L.dadmm_last_error()
    assert torch.equal(got, want)


@pytest.mark.parametrize("B,P,n,N,per_sample", [(7, 5, 256, 100, True), (40, 50, 512, 100, True),
                                                (9, 16, 64, 20, False), (3, 2, 16, 8, True),
                                                (1024, 50, 1024, 100, True)])   # gcn32_kernel
def test_gcn_ex_split_layer_matches_torch(cuda, L, B, P, n, N, per_sample):
    """Layer 1 as the model's eval path runs it (hypernetwork_eval_prepare): the raw Atb half
    A_hat (xb W[:, n:]^T) once, then the AtAy half's GEMM with that term added before the bias,
    against torch's GCNConv on cat(xa, xb)."""
    from dadmm_hip.graph import ingest
    G = B if per_sample else 1
    graphs = [O.connected_er_graph(P, 0.4, seed=7 * i + P) for i in range(G)]
    gb = ingest(graphs, P, G, cuda)
    ahat = _ahat(gb.nbr.reshape(G, P), P, cuda)
    gen = torch.Generator(device=cuda).manual_seed(B * P + N + n)
    xa = torch.randn(B * P, n + 4, device=cuda, generator=gen)     # padded rows (ld = n + 4)
    xb = torch.randn(B * P, n + 4, device=cuda, generator=gen)
    W = torch.randn(N, 2 * n, device=cuda, generator=gen) / np.sqrt(2 * n)
    bias, rm, bw, bb = (torch.randn(N, device=cuda, generator=gen) for _ in range(4))
    rv = torch.rand(N, device=cuda, generator=gen) + 0.5
    c1 = torch.empty(B * P, N, device=cuda)
    rc = L.dadmm_hyper_gcn_ex(B, P, n, N, _p(xb), n + 4, W.data_ptr() + 4 * n, 2 * n, None, 0, None, _p(ahat),
                              int(per_sample), None, None, None, None, 0.0, 0.0, 1, _p(c1), N, _s())
    assert rc == 0, L.dadmm_last_error()
    zb = torch.matmul(ahat, F.linear(xb[:, :n], W[:, n:]).view(B, P, N)).reshape(B * P, N)
    _close(c1, zb, n)
    y = torch.empty(B * P, N, device=cuda)
    rc = L.dadmm_hyper_gcn_ex(B, P, n, N, _p(xa), n + 4, _p(W), 2 * n, _p(c1), N, _p(bias), _p(ahat),
                              int(per_sample), _p(rm), _p(rv), _p(bw), _p(bb), 1e-5, 0.01, 0, _p(y), N, _s())
    assert rc == 0, L.dadmm_last_error()
    x = torch.cat([xa[:, :n], xb[:, :n]], dim=1)
    z = torch.matmul(ahat, F.linear(x, W).view(B, P, N)) + bias
    want = F.batch_norm(F.leaky_relu(z).reshape(B * P, N), rm, rv, bw, bb, False, 0.0, 1e-5)
    _close(y, want, 2 * n)


@pytest.mark.parametrize("rows,C,act", [(5, 400, False), (1024, 400, True), (3, 2048, True),
                                        (70, 36, False)])
def test_rownorm_matches_torch(cuda, L, rows, C, act):
    gen = torch.Generator(device=cuda).manual_seed(rows + C)
    x = 3 * torch.randn(rows, C, device=cuda, generator=gen) + 1
    w, b = torch.randn(C, device=cuda, generator=gen), torch.randn(C, device=cuda, generator=gen)
    y = torch.empty_like(x)
    assert L.dadmm_hyper_rownorm(rows, C, _p(x), _p(w), _p(b), 1e-5, int(act), 0.01, _p(y), _s()) == 0
    want = F.layer_norm(x, (C,), w, b, 1e-5)
    if act:
        want = F.leaky_relu(want, 0.01)
    _close(y, want, C)
    # in place (how the model uses it)
    assert L.dadmm_hyper_rownorm(rows, C, _p(x), _p(w), _p(b), 1e-5, int(act), 0.01, _p(x), _s()) == 0
    torch.testing.assert_close(x, y, rtol=0, atol=0)


@pytest.mark.parametrize("rows,K,N", [(1024, 2000, 400), (1024, 400, 200), (1024, 20000, 400),
                                      (37, 36, 100), (5, 200, 8)])
def test_linear_ln_matches_torch(cuda, L, rows, K, N):
    """One decoder block (Linear -> LayerNorm -> LeakyReLU) through the split-K GEMM whose
    partials the LayerNorm launch sums (deterministic: two launches agree bit for bit)."""
    gen = torch.Generator(device=cuda).manual_seed(rows + K + N)
    x = torch.randn(rows, K, device=cuda, generator=gen)
    W = torch.randn(N, K, device=cuda, generator=gen) / np.sqrt(K)
    bias, lw, lb = (torch.randn(N, device=cuda, generator=gen) for _ in range(3))
    scratch = torch.empty(max(L.dadmm_hyper_linear_ln_scratch_bytes(rows, K, N), 16) // 4, device=cuda)
    y, y2 = torch.empty(rows, N, device=cuda), torch.empty(rows, N, device=cuda)
    for out in (y, y2):
        rc = L.dadmm_hyper_linear_ln(rows, K, N, _p(x), K, _p(W), _p(bias), _p(lw), _p(lb), 1e-5, 1,
                                     0.01, _p(out), _p(scratch), _s())
        assert rc == 0, L.dadmm_last_error()
    want = F.leaky_relu(F.layer_norm(F.linear(x, W, bias), (N,), lw, lb, 1e-5), 0.01)
    _close(y, want, K)
    assert torch.equal(y, y2)


@pytest.mark.parametrize("B,Kh,H", [(64, 100, 5), (7, 16, 1), (300, 100, 16)])
def test_head_matches_torch(cuda, L, B, Kh, H):
    gen = torch.Generator(device=cuda).manual_seed(B + H)
    x = torch.randn(B, Kh, device=cuda, generator=gen)
    W = 3 * torch.randn(4 * H, Kh, device=cuda, generator=gen) / np.sqrt(Kh)
    bias = torch.randn(4 * H, device=cuda, generator=gen)
    hyp = torch.empty(B, 4, H, device=cuda)
    mx = (0.1, 0.99, 0.99, 0.99)
    assert L.dadmm_hyper_head(B, Kh, H, _p(x), Kh, _p(W), _p(bias), *mx, _p(hyp), _s()) == 0
    h = torch.clamp(torch.sigmoid(F.linear(x, W, bias)), min=1e-4, max=0.9999).view(B, 4, H)
    want = torch.stack([h[:, 0] * torch.tensor(mx[0]).to(cuda),
                        torch.clamp(h[:, 1] * torch.tensor(mx[1]).to(cuda), max=0.9999),
                        torch.clamp(h[:, 2] * torch.tensor(mx[2]).to(cuda), max=0.9999),
                        torch.clamp(h[:, 3] * torch.tensor(mx[3]).to(cuda), max=0.9999)], dim=1)
    _close(hyp, want, Kh)


def _model(dev, P, m, n, K, hidden, mode, seed=0):
    import gnn_dlasso_models_progressive as G
    A, b, x = O.make_problem(P, m, n, 64, seed=seed + 5)
    torch.manual_seed(seed)
    args = argparse.Namespace(GHN_iter_num=K, GHyp_hidden=hidden, DADMM_mode=mode, alpha_max=0.1,
                              tau_max=0.99, rho_max=0.99, eta_max=0.99)
    model = G.DLASSO_GNNHyp3_Progressive(torch.from_numpy(A)[None].to(dev), args).to(dev)
    with torch.no_grad():   # non-trivial BatchNorm running statistics
        for i in range(1, 6):
            bn = getattr(model.encoder, f"bn{i}")
            bn.running_mean.normal_(0, 0.3)
            bn.running_var.uniform_(0.5, 2.0)
            bn.weight.normal_(1, 0.1)
            bn.bias.normal_(0, 0.1)
    return model.eval(), A, b


@pytest.mark.parametrize("P,n,hidden,mode,per_sample", [(5, 64, 16, "diff", True),
                                                        (5, 256, 100, "diff", True),
                                                        (5, 128, 100, "same", False),
                                                        (16, 64, 20, "diff", True),
                                                        (6, 100, 12, "diff", True)])
def test_model_fused_matches_torch_backend(cuda, P, n, hidden, mode, per_sample):
    """Same features in, same hyper-parameters out: the torch backend's features of every
    iteration go through the fused kernels; and the whole forward on either backend."""
    from dadmm_hip import hyper_ops
    from dadmm_hip.graph import ingest
    import gnn_dlasso_models_progressive as G
    B, K = 48, 3
    model, A, b = _model(cuda, P, 32, n, K, hidden, mode)
    graphs = ([O.connected_er_graph(P, 0.5, seed=s) for s in range(B)] if per_sample
              else [O.er_graph(P, 0.5, seed=3)] * B)
    rng = np.random.default_rng(1)
    inits = tuple(torch.from_numpy((1e-2 * rng.standard_normal((B, P, n))).astype(np.float32)).to(cuda)
                  for _ in range(3))
    bt = torch.from_numpy(b[:B]).to(cuda)[..., None]
    rec_t, rec_f = [], []
    model.hyper_backend = "torch"
    model.on_hyp = lambda f, a, o: rec_t.append((f.clone(), a.clone(), [t.clone() for t in o]))
    with torch.no_grad():
        Yt, _ = model(bt, graphs, inits=inits)
    model.hyper_backend = "auto"
    model.on_hyp = lambda f, a, o: rec_f.append([t.clone() for t in o])
    with torch.no_grad():
        Yf, hf = model(bt, graphs, inits=inits)
    assert len(rec_f) == K and hf[0].shape == (B, 1 if mode == "same" else P, 1, 1)
    H = 1 if mode == "same" else P
    gb = ingest(graphs, P, B, cuda)
    ahat = G.normalized_adjacency(gb.nbr, P)
    ahat = (ahat[None] if gb.shared else ahat).contiguous()
    bufs = hyper_ops.HyperBuffers(B, P, 4 * hidden, [4 * hidden, 2 * hidden, hidden], H, cuda)
    for feats, atb, out in rec_t:
        ns = (n + 3) & ~3
        AtAy = torch.zeros(B, P, ns, device=cuda)
        Atb = torch.zeros(B, P, ns, device=cuda)
        AtAy[..., :n], Atb[..., :n] = feats, atb
        with torch.no_grad():
            got = hyper_ops.hypernetwork_eval(model, AtAy, Atb, n, ahat, not gb.shared, bufs)
        for g, w in zip(got, out):
            torch.testing.assert_close(g, w, rtol=2e-5, atol=2e-6)
    # whole forward: same hyper-parameters up to f32 rounding, so the iterates agree closely
    for a, c in zip(rec_f, [r[2] for r in rec_t]):
        for g, w in zip(a, c):
            torch.testing.assert_close(g, w, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(Yf, Yt, rtol=1e-3, atol=1e-4)
