"""GPU: oracle checks at the configurations the other files leave out.

* The GNN model (DLASSO_GNNHyp3_Progressive, gnn_dlasso_models_progressive.py:131-243) at the
  reference's own defaults, the configuration of its one published GNN result: P = 5, m = 100,
  n = 500, GHyp_hidden = 100 (configurations.py:6-9, :118), on the reference's shipped operator
  results/25_iter_general_learning/A.pt [1, 5, 100, 500] (tests/golden, read without unpickling),
  per-sample connected ER(0.5) graphs (gnn_dlasso_progressive.py:181-191). This exercises the m > 64
  gram path of dadmm_gnn.hip and the 2n = 1000-wide first GCN layer inside the model.
    - eval: every iteration's (alpha, tau, rho, eta) within 1e-4 of the numpy fp64 restatement of
      the hypernetwork (oracle/gnn_np.py) on the features the kernels produced, and the whole
      K = 25 recurrence BIT-EXACT against oracle.forward_f32_gram given those hyper-parameters;
    - train (model.train(), HIP training hypernetwork, Dropout p = 0 so both sides see the same
      network): every parameter gradient of loss_final.backward() against CPU fp64 autograd of the
      reference's loop (oracle/ref_torch.gnn_forward_autograd), within 8x the error torch fp32 on
      the GPU makes against the same fp64 reference (+1e-5 of the gradient's scale).
* configs[4]'s model (P = 50, n = 1024, m = 32, h = 100, per-sample ER(0.5)) at its own depth
  K = 50, B = 2: hyp per iteration vs gnn_np and the recurrence bit-exact.
* The headline batch itself (B = 4096, P = 5, n = 256, m = 64, K = 25, BASELINE configs[1] / H):
  one DLASSO_unfolded.forward with the trained seq_hyp fixture, a strided slice of 32 samples
  compared bit-for-bit with oracle.forward_f32 (samples are independent under the shared graph),
  and the final-iterate MSE of the slice vs oracle.forward_f64 <= 1e-5 (north_star).
Parity with torch_geometric itself and with the reference's own outputs stays unpinned (SURVEY
§8(c)): these compare against the repo's oracle restatements.
"""
import argparse
import copy
import os

import numpy as np
import pytest
import torch

import oracle as O
from oracle import gnn_np, ref_torch

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")
MAXP = [0.1, 0.99, 0.99, 0.99]


def _t(x, dev):
    return torch.from_numpy(np.ascontiguousarray(x)).to(dev)


def _gnn_args(K, hidden=100, mode="diff"):
    return argparse.Namespace(GHN_iter_num=K, GHyp_hidden=hidden, DADMM_mode=mode,
                              alpha_max=0.1, tau_max=0.99, rho_max=0.99, eta_max=0.99)


def _randomise_bn(model, seed):
    """Non-trivial BatchNorm running statistics and affine parameters (a trained model's)."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for name, buf in model.named_buffers():
            if name.endswith("running_mean"):
                buf.copy_(0.1 * torch.randn(buf.shape, generator=g))
            elif name.endswith("running_var"):
                buf.copy_(0.5 + torch.rand(buf.shape, generator=g))
        for name, prm in model.named_parameters():
            if ".bn" in name:
                prm.add_(0.05 * torch.randn(prm.shape, generator=g).to(prm.device))


def _record(model):
    rec = []
    model.on_hyp = lambda AtAy, Atb, out: rec.append(
        (AtAy.detach().clone(), Atb.detach().clone(), [o.detach().clone() for o in out]))
    return rec


def _check_eval(model, A, b, graphs, inits, K, dev):
    """hyp per iteration vs gnn_np, recurrence bit-exact vs forward_f32_gram."""
    B, P = b.shape[:2]
    model.eval()
    rec = _record(model)
    with torch.no_grad():
        Y, _ = model(_t(b, dev)[..., None], graphs, inits=tuple(_t(v, dev) for v in inits))
    assert int(model.last_status.item()) == 0
    assert len(rec) == K
    sd = {k: v.detach().cpu().numpy().astype(np.float64) for k, v in model.state_dict().items()}
    maxima = tuple(float(np.float32(v)) for v in MAXP)
    n = A.shape[-1]
    for k, (AtAy, Atb, out) in enumerate(rec):
        feats = torch.cat([AtAy[..., :n], Atb[..., :n]], dim=2).cpu().numpy().astype(np.float64)
        want = gnn_np.hypernetwork(sd, feats, graphs, maxima, False)
        for c, (got, w) in enumerate(zip(out, want)):
            got = got[..., 0, 0].cpu().numpy()
            np.testing.assert_allclose(got, w, rtol=1e-4, atol=1e-4 * np.abs(w).max(),
                                       err_msg=f"iteration {k}, hyper-parameter {c}")
    table = np.stack([torch.stack([o[..., 0, 0] for o in r[2]], dim=1).cpu().numpy()
                      for r in rec]).reshape(K, B, 4, P).astype(np.float32)
    Yo, _, st = O.forward_f32_gram(A, b, graphs, table, *inits, variant=1, hyp_mode=1)
    assert st == 0
    Yg = Y[..., 0].cpu().numpy()
    assert np.array_equal(Yg, Yo), f"max |diff| {np.abs(Yg - Yo).max():.3e}"
    return Yg


def _reference_defaults(dev, B, seed):
    import gnn_dlasso_models_progressive as G
    A = np.load(os.path.join(GOLD, "fixture_25_iter_general_learning_A.npy"))      # [1,5,100,500]
    _, P, m, n = A.shape
    rng = np.random.default_rng(seed)
    x = (2.0 * rng.standard_normal((B, n)) * (rng.random((B, n)) <= 0.25)).astype(np.float32)
    b = np.einsum("pmn,bn->bpm", A[0].astype(np.float64), x).astype(np.float32)
    inits = tuple((1e-2 * rng.standard_normal((3, B, P, n))).astype(np.float32))
    graphs = [O.connected_er_graph(P, 0.5, seed=seed * 100 + s) for s in range(B)]
    torch.manual_seed(seed)
    model = G.DLASSO_GNNHyp3_Progressive(_t(A, dev), _gnn_args(25)).to(dev)
    return model, A[0], b, x, graphs, inits


def test_gnn_reference_defaults_eval_k25(cuda):
    model, A, b, x, graphs, inits = _reference_defaults(cuda, B=4, seed=1)
    _randomise_bn(model, 11)
    Y = _check_eval(model, A, b, graphs, inits, 25, cuda)
    assert np.isfinite(Y).all()


def _train_grads(model, b, graphs, inits, label, K, dev):
    Y, _ = model(_t(b, dev)[..., None], graphs, K, inits=tuple(_t(v, dev) for v in inits))
    import gnn_dlasso_utils
    _, loss_final = gnn_dlasso_utils.compute_loss(Y, label)
    loss_final.backward()
    return {k: p.grad.detach().double().cpu() for k, p in model.named_parameters()}


def test_gnn_reference_defaults_train_gradients(cuda):
    """Training step at the reference defaults through the HIP training hypernetwork."""
    import gnn_dlasso_models_progressive as G
    from dadmm_hip.graph import ingest
    B, K = 4, 3
    model, A, b, x, graphs, inits = _reference_defaults(cuda, B=B, seed=2)
    _randomise_bn(model, 12)
    for mod in [model.encoder.dropout] + [model.decoder[i] for i in (1, 5, 9)]:
        mod.p = 0.0
    ref32 = copy.deepcopy(model)
    ref32.hyper_backend = "torch"
    cpu = copy.deepcopy(model).cpu().double()
    model.train(), ref32.train(), cpu.train()
    label = _t(x, cuda)[..., None]
    got = _train_grads(model, b, graphs, inits, label, K, cuda)
    assert model.last_backend == "hip-train"
    want32 = _train_grads(ref32, b, graphs, inits, label, K, cuda)

    a_hat = G.normalized_adjacency(ingest(graphs, 5, B, "cpu").nbr, 5, torch.float64)
    Yc, _ = ref_torch.gnn_forward_autograd(cpu, A, b, graphs, *inits, K=K, a_hat=a_hat)
    lab = torch.from_numpy(x).double()
    loss_final = ((Yc[-1] - lab[:, None, :]) ** 2).mean(dim=(0, 2)).sum() / 5 + 1e-8
    loss_final.backward()
    for name, p in cpu.named_parameters():
        w64 = p.grad.detach()
        scale = float(w64.abs().max())
        assert scale > 0, name
        e_hip = float((got[name] - w64).abs().max())
        e_t32 = float((want32[name] - w64).abs().max())
        assert np.isfinite(e_hip), name
        assert e_hip <= 8.0 * e_t32 + 1e-5 * scale, \
            f"{name}: |hip - fp64| {e_hip:.3e}, |torch32 - fp64| {e_t32:.3e}, scale {scale:.3e}"


def test_configs4_model_full_depth_k50(cuda):
    """BASELINE configs[4]'s model at its own depth, K = 50 (B = 2)."""
    import gnn_dlasso_models_progressive as G
    P, m, n, B, K = 50, 32, 1024, 2, 50
    A, b, x = O.make_problem(P, m, n, B, seed=9)
    torch.manual_seed(4)
    model = G.DLASSO_GNNHyp3_Progressive(_t(A, cuda)[None], _gnn_args(K)).to(cuda)
    _randomise_bn(model, 13)
    graphs = [O.connected_er_graph(P, 0.5, seed=400 + s) for s in range(B)]
    rng = np.random.default_rng(4)
    inits = tuple((1e-2 * rng.standard_normal((3, B, P, n))).astype(np.float32))
    Y = _check_eval(model, A, b, graphs, inits, K, cuda)
    assert np.isfinite(Y).all()


def test_headline_batch_4096_strided_slice_bit_exact(cuda):
    """One forward over the full headline batch; 32 samples (every 128th) vs the oracle."""
    import unfolded_DLASSO
    P, m, n, B, K = 5, 64, 256, 4096, 25
    param = np.load(os.path.join(GOLD, "fixture_25_iter_general_learning_seq_hyp_param.npy"))
    A, b, x = O.make_problem(P, m, n, B, seed=1234)
    graphs = [O.er_graph(P, 0.5, seed=7)] * B
    rng = np.random.default_rng(99)
    y0, U0, d0 = (1e-2 * rng.standard_normal((3, B, P, n))).astype(np.float32)
    args = argparse.Namespace(GHN_iter_num=K, DADMM_mode="diff", alpha_max=0.1, tau_max=0.99,
                              rho_max=0.99, eta_max=0.99, max_penalty_threshold=0.8,
                              penalty_reduction_factor=0.95)
    model = unfolded_DLASSO.DLASSO_unfolded(_t(A, cuda)[None], args).to(cuda).eval()
    with torch.no_grad():
        model.seq_hyp.param.copy_(torch.from_numpy(param))
        Y, _ = model(_t(b, cuda)[..., None], graphs, inits=tuple(_t(v, cuda) for v in (y0, U0, d0)))
    assert int(model.last_status.item()) == 0
    sl = np.arange(0, B, 128) + np.arange(32) % 7          # every 128th sample, jittered
    Ys = Y[:, torch.from_numpy(sl).to(cuda), :, :, 0].cpu().numpy()
    table = model.hyp_table(K).detach().cpu().numpy()
    Yo, _, st = O.forward_f32(A, b[sl], [graphs[0]] * len(sl), table, y0[sl], U0[sl], d0[sl])
    assert st == 0
    assert np.array_equal(Ys, Yo), f"max |diff| {np.abs(Ys - Yo).max():.3e}"
    Y64, _, _ = O.forward_f64(A, b[sl], [graphs[0]] * len(sl), table, y0[sl], U0[sl], d0[sl])
    mse = float(((Ys[-1].astype(np.float64) - Y64[-1]) ** 2).mean())
    assert mse <= 1e-5, mse


def test_configs2_full_batch_strided_slice_bit_exact(cuda):
    """BASELINE configs[2] at its own size: B = 4096, P = 16, n = 512, m = 64, K = 25, per-sample
    ER(0.3) graphs (the tiled path + the gated stepwise recomputation). One forward over the
    whole batch; a strided slice of 16 samples bit-for-bit against oracle.forward_f32 (samples
    are independent), status 0."""
    import unfolded_DLASSO
    P, m, n, B, K = 16, 64, 512, 4096, 25
    A, b, x = O.make_problem(P, m, n, B, seed=2024)
    graphs = [O.er_graph(P, 0.3, seed=50_000 + s) for s in range(B)]
    rng = np.random.default_rng(5)
    y0, U0, d0 = (1e-2 * rng.standard_normal((3, B, P, n))).astype(np.float32)
    args = argparse.Namespace(GHN_iter_num=K, DADMM_mode="diff", alpha_max=0.1, tau_max=0.99,
                              rho_max=0.99, eta_max=0.99, max_penalty_threshold=0.8,
                              penalty_reduction_factor=0.95)
    torch.manual_seed(6)
    model = unfolded_DLASSO.DLASSO_unfolded(_t(A, cuda)[None], args).to(cuda).eval()
    with torch.no_grad():
        Y, _ = model(_t(b, cuda)[..., None], graphs, inits=tuple(_t(v, cuda) for v in (y0, U0, d0)))
    assert int(model.last_status.item()) == 0
    sl = np.arange(0, B, 256) + np.arange(16) % 5
    Ys = Y[:, torch.from_numpy(sl).to(cuda), :, :, 0].cpu().numpy()
    table = model.hyp_table(K).detach().cpu().numpy()
    Yo, _, st = O.forward_f32(A, b[sl], [graphs[s] for s in sl], table, y0[sl], U0[sl], d0[sl])
    assert st == 0
    assert np.array_equal(Ys, Yo), f"max |diff| {np.abs(Ys - Yo).max():.3e}"


def test_configs4_shard_full_batch_strided_slice(cuda):
    """BASELINE configs[4]'s per-GPU shard at its own size: B = 1024, P = 50, n = 1024, m = 32,
    K = 50, h = 100, per-sample connected ER(0.5) graphs. One eval forward over the whole shard
    (every iteration's hyper-parameters recorded); for a strided slice of 4 samples the
    hypernetwork's outputs at iterations 0, 24 and 49 against oracle/gnn_np.py (1e-4) and the
    whole recurrence bit-for-bit against oracle.forward_f32_gram given the recorded table."""
    import gnn_dlasso_models_progressive as G
    P, m, n, B, K = 50, 32, 1024, 1024, 50
    A, b, x = O.make_problem(P, m, n, B, seed=31)
    torch.manual_seed(8)
    model = G.DLASSO_GNNHyp3_Progressive(_t(A, cuda)[None], _gnn_args(K)).to(cuda)
    _randomise_bn(model, 21)
    model.eval()
    graphs = [O.connected_er_graph(P, 0.5, seed=600 + s) for s in range(B)]
    rng = np.random.default_rng(12)
    inits = tuple((1e-2 * rng.standard_normal((3, B, P, n))).astype(np.float32))
    sl = np.arange(0, B, 256) + np.arange(4) % 3
    sl_t = torch.from_numpy(sl).to(cuda)
    rec = []
    model.on_hyp = lambda AtAy, Atb, out: rec.append(
        (torch.cat([AtAy[sl_t, :, :n], Atb[sl_t, :, :n]], dim=2).cpu(),
         torch.stack([o[sl_t, :, 0, 0] for o in out], dim=1).cpu()))
    with torch.no_grad():
        Y, _ = model(_t(b, cuda)[..., None], graphs, inits=tuple(_t(v, cuda) for v in inits))
    assert int(model.last_status.item()) == 0
    assert len(rec) == K
    sd = {k: v.detach().cpu().numpy().astype(np.float64) for k, v in model.state_dict().items()}
    maxima = tuple(float(np.float32(v)) for v in MAXP)
    gsl = [graphs[s] for s in sl]
    for k in (0, 24, 49):
        feats, got = rec[k]
        want = gnn_np.hypernetwork(sd, feats.numpy().astype(np.float64), gsl, maxima, False)
        for c in range(4):
            w = want[c][..., 0, 0] if want[c].ndim == 4 else want[c]
            np.testing.assert_allclose(got[:, c].numpy(), w.reshape(got[:, c].shape), rtol=1e-4,
                                       atol=1e-4 * np.abs(w).max(), err_msg=f"iteration {k}, c {c}")
    table = np.stack([r[1].numpy() for r in rec]).astype(np.float32)          # [K, 4 samples, 4, P]
    Ys = Y[:, sl_t, :, :, 0].cpu().numpy()
    Yo, _, st = O.forward_f32_gram(A, b[sl], gsl, table, *(v[sl] for v in inits), variant=1, hyp_mode=1)
    assert st == 0
    assert np.array_equal(Ys, Yo), f"max |diff| {np.abs(Ys - Yo).max():.3e}"


def _dev_inits(shape, seed, dev):
    """y0, U0, d0 = 1e-2 N(0, 1) drawn on the device (the full-batch tests' inits: several GB at
    configs[4], so not drawn on the host); the slices the oracle needs are copied back."""
    g = torch.Generator(device=dev).manual_seed(seed)
    return tuple(1e-2 * torch.randn(shape, generator=g, device=dev) for _ in range(3))


def test_configs3_global_batch_32768_strided_slice_bit_exact(cuda):
    """BASELINE configs[3] at its GLOBAL batch on one GPU: B = 32768, P = 5, n = 256, m = 64,
    K = 25 (the batch the 8-GPU run shards 8 ways; Y = 4.2 GB), shared ER(0.5) graph, the trained
    seq_hyp fixture. One DLASSO_unfolded.forward over the whole batch (unfolded_DLASSO.py:53-109),
    status 0, a strided slice of 32 samples bit-for-bit against oracle.forward_f32 and the slice's
    final-iterate MSE vs oracle.forward_f64 <= 1e-5 (north_star)."""
    import unfolded_DLASSO
    P, m, n, B, K = 5, 64, 256, 32768, 25
    param = np.load(os.path.join(GOLD, "fixture_25_iter_general_learning_seq_hyp_param.npy"))
    A, b, _ = O.make_problem(P, m, n, B, seed=3232)
    G = O.er_graph(P, 0.5, seed=7)
    inits = _dev_inits((B, P, n), 33, cuda)
    args = argparse.Namespace(GHN_iter_num=K, DADMM_mode="diff", alpha_max=0.1, tau_max=0.99,
                              rho_max=0.99, eta_max=0.99, max_penalty_threshold=0.8,
                              penalty_reduction_factor=0.95)
    model = unfolded_DLASSO.DLASSO_unfolded(_t(A, cuda)[None], args).to(cuda).eval()
    with torch.no_grad():
        model.seq_hyp.param.copy_(torch.from_numpy(param))
        Y, _ = model(_t(b, cuda)[..., None], [G] * B, inits=inits)
    assert int(model.last_status.item()) == 0
    assert tuple(Y.shape) == (K, B, P, n, 1)
    sl = np.arange(0, B, 1024) + np.arange(32) % 11       # every 1024th sample, jittered
    sl_t = torch.from_numpy(sl).to(cuda)
    Ys = Y[:, sl_t, :, :, 0].cpu().numpy()
    y0, U0, d0 = (v[sl_t].cpu().numpy() for v in inits)
    del Y
    table = model.hyp_table(K).detach().cpu().numpy()
    Yo, _, st = O.forward_f32(A, b[sl], [G] * len(sl), table, y0, U0, d0)
    assert st == 0
    assert np.array_equal(Ys, Yo), f"max |diff| {np.abs(Ys - Yo).max():.3e}"
    Y64, _, _ = O.forward_f64(A, b[sl], [G] * len(sl), table, y0, U0, d0)
    mse = float(((Ys[-1].astype(np.float64) - Y64[-1]) ** 2).mean())
    assert mse <= 1e-5, mse


def test_configs4_global_batch_8192_k50(cuda):
    """BASELINE configs[4] at its GLOBAL batch on one GPU: DLASSO_GNNHyp3_Progressive, B = 8192,
    P = 50, n = 1024, m = 32, K = 50, h = 100, per-sample connected ER(0.5) graphs generated on the
    device (dadmm_graph_generate: gnn_dlasso_progressive.py:181-191's graph model). Y is
    50 x 8192 x 50 x 1024 x 4 B = 84 GB and one iterate 1.68 GB, so every kernel's 64-bit
    addressing is exercised. Two eval forwards over the whole batch:
      * launch by launch with every iteration's hyper-parameters recorded (on_hyp): for a strided
        slice of 4 samples the hypernetwork outputs at iterations 0, 25 and 49 against
        oracle/gnn_np.py (1e-4) and the whole K = 50 recurrence bit-for-bit against
        oracle.forward_f32_gram given the recorded table (gnn_dlasso_models_progressive.py:131-243);
      * the production path (one replay of the captured HIP graph): the slice bit-identical to
        the first forward, status 0."""
    import gnn_dlasso_models_progressive as GM
    from dadmm_hip.graph import generate_er, to_networkx
    P, m, n, B, K = 50, 32, 1024, 8192, 50
    A, b, _ = O.make_problem(P, m, n, B, seed=88)
    torch.manual_seed(18)
    model = GM.DLASSO_GNNHyp3_Progressive(_t(A, cuda)[None], _gnn_args(K)).to(cuda)
    _randomise_bn(model, 28)
    model.eval()
    gb = generate_er(B, P, 0.5, 8192, cuda)
    inits = _dev_inits((B, P, n), 44, cuda)
    sl = np.arange(0, B, 2048) + np.arange(4) % 3 + 2047 * (np.arange(4) == 3)
    sl_t = torch.from_numpy(sl).to(cuda)
    rec = []
    model.on_hyp = lambda AtAy, Atb, out: rec.append(
        (torch.cat([AtAy[sl_t, :, :n], Atb[sl_t, :, :n]], dim=2).cpu(),
         torch.stack([o[sl_t, :, 0, 0] for o in out], dim=1).cpu()))
    bt = _t(b, cuda)[..., None]
    with torch.no_grad():
        Y, _ = model(bt, gb, inits=inits)
    assert model.last_backend == "hip-eval"
    assert int(model.last_status.item()) == 0
    assert len(rec) == K and tuple(Y.shape) == (K, B, P, n, 1)
    Ys = Y[:, sl_t, :, :, 0].cpu().numpy()
    del Y
    torch.cuda.empty_cache()

    sd = {k: v.detach().cpu().numpy().astype(np.float64) for k, v in model.state_dict().items()}
    maxima = tuple(float(np.float32(v)) for v in MAXP)
    gsl = to_networkx(gb, P, samples=sl)
    for k in (0, 25, 49):
        feats, got = rec[k]
        want = gnn_np.hypernetwork(sd, feats.numpy().astype(np.float64), gsl, maxima, False)
        for c in range(4):
            w = want[c][..., 0, 0] if want[c].ndim == 4 else want[c]
            np.testing.assert_allclose(got[:, c].numpy(), w.reshape(got[:, c].shape), rtol=1e-4,
                                       atol=1e-4 * np.abs(w).max(), err_msg=f"iteration {k}, c {c}")
    table = np.stack([r[1].numpy() for r in rec]).astype(np.float32)          # [K, 4, 4, P]
    y0, U0, d0 = (v[sl_t].cpu().numpy() for v in inits)
    Yo, _, st = O.forward_f32_gram(A, b[sl], gsl, table, y0, U0, d0, variant=1, hyp_mode=1)
    assert st == 0
    assert np.array_equal(Ys, Yo), f"max |diff| {np.abs(Ys - Yo).max():.3e}"

    model.on_hyp = None
    with torch.no_grad():
        Y2, _ = model(bt, gb, inits=inits)
    assert model.last_backend == "hip-eval-graph"
    assert int(model.last_status.item()) == 0
    Y2s = Y2[:, sl_t, :, :, 0].cpu().numpy()
    assert np.array_equal(Y2s, Ys), f"graphed vs launch-by-launch: max |diff| {np.abs(Y2s - Ys).max():.3e}"
