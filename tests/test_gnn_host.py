"""CPU: the GNN-hypernetwork model's host side — PyG-compatible parameter names, the per-sample
BatchNorm (train-mode statistics and sequential running-stat updates), the normalized adjacency,
and the batched torch hypernetwork against the numpy edge-list restatement of GCNConv
(oracle/gnn_np.py; parity unpinned against torch_geometric, which is absent)."""
import argparse

import numpy as np
import pytest
import torch

import oracle as O
from oracle import gnn_np


def _args(K=4, mode="diff", hidden=8):
    return argparse.Namespace(GHN_iter_num=K, GHyp_hidden=hidden, DADMM_mode=mode, alpha_max=0.1,
                              tau_max=0.99, rho_max=0.99, eta_max=0.99)


def _model(P=5, m=8, n=12, mode="diff", hidden=8):
    import gnn_dlasso_models_progressive as G
    torch.manual_seed(0)
    A = torch.randn(1, P, m, n)
    return G.DLASSO_GNNHyp3_Progressive(A, _args(mode=mode, hidden=hidden))


@pytest.mark.parametrize("mode,H", [("diff", 5), ("same", 1)])
def test_state_dict_uses_pyg_names(mode, H):
    sd = _model(mode=mode).state_dict()
    keys = set(sd)
    for i in range(1, 6):
        assert f"encoder.conv{i}.lin.weight" in keys and f"encoder.conv{i}.bias" in keys
        for suffix in ("weight", "bias", "running_mean", "running_var", "num_batches_tracked"):
            assert f"encoder.bn{i}.{suffix}" in keys
    assert {"encoder.norm.weight", "encoder.norm.bias"} <= keys
    for i in (0, 2, 4, 6, 8, 10):
        assert f"decoder.{i}.weight" in keys
    assert tuple(sd["fc.weight"].shape) == (4 * H, 8)
    np.testing.assert_array_equal(sd["fc.bias"][:4].numpy(), np.float32([-0.5, -1.0, -0.8, -1.2]))
    assert tuple(sd["encoder.conv1.lin.weight"].shape) == (8, 24)   # 2n -> h


def test_per_sample_batch_norm_equals_reference_loop():
    """The reference calls bn(x_i) for every sample i in turn (train mode): per-sample batch
    statistics over the P nodes and one running-stat update per sample, in sample order."""
    import gnn_dlasso_models_progressive as G
    torch.manual_seed(1)
    B, P, C = 6, 5, 7
    x = torch.randn(B, P, C, dtype=torch.float64)
    bn = torch.nn.BatchNorm1d(C).double()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.2, 0.2)
        bn.running_mean.uniform_(-1, 1)
        bn.running_var.uniform_(0.5, 2)
    ref = torch.nn.BatchNorm1d(C).double()
    ref.load_state_dict(bn.state_dict())
    bn.train()
    ref.train()
    got = G._per_sample_batch_norm(x, bn)
    want = torch.stack([ref(x[i]) for i in range(B)])
    torch.testing.assert_close(got, want, rtol=1e-12, atol=1e-12)
    torch.testing.assert_close(bn.running_mean, ref.running_mean, rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(bn.running_var, ref.running_var, rtol=1e-6, atol=1e-7)
    assert int(bn.num_batches_tracked) == int(ref.num_batches_tracked) == B
    bn.eval()
    ref.eval()
    torch.testing.assert_close(G._per_sample_batch_norm(x, bn),
                               torch.stack([ref(x[i]) for i in range(B)]), rtol=1e-6, atol=1e-7)


def test_per_sample_batch_norm_single_node_raises_like_torch():
    import gnn_dlasso_models_progressive as G
    bn = torch.nn.BatchNorm1d(3)
    with pytest.raises(ValueError):
        G._per_sample_batch_norm(torch.randn(2, 1, 3), bn)


def test_normalized_adjacency_matches_gcn_norm():
    import gnn_dlasso_models_progressive as G
    from dadmm_hip.graph import ingest
    P, B = 6, 4
    graphs = [O.connected_er_graph(P, 0.4, seed=s) for s in range(B)]
    gb = ingest(graphs, P, B, "cpu")
    a_hat = G.normalized_adjacency(gb.nbr, P).numpy()
    for s, g in enumerate(graphs):
        x = np.eye(P)
        want = gnn_np.gcn_conv(x, np.eye(P), np.zeros(P), g, P)   # aggregation of the identity
        np.testing.assert_allclose(a_hat[s], want.T, rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("mode", ["diff", "same"])
def test_hypernetwork_matches_edge_list_restatement(mode):
    """The batched dense GCN of the build == the per-sample edge-list GCNConv restatement (eval)."""
    import gnn_dlasso_models_progressive as G
    from dadmm_hip.graph import ingest
    P, m, n, B = 5, 8, 12, 7
    model = _model(P, m, n, mode).double().eval()
    with torch.no_grad():                      # non-trivial running statistics
        for i in range(1, 6):
            bn = getattr(model.encoder, f"bn{i}")
            bn.running_mean.uniform_(-0.5, 0.5)
            bn.running_var.uniform_(0.5, 2.0)
    graphs = [O.connected_er_graph(P, 0.5, seed=10 + s) for s in range(B)]
    a_hat = G.normalized_adjacency(ingest(graphs, P, B, "cpu").nbr, P, torch.float64)
    feats = torch.randn(B, P, 2 * n, dtype=torch.float64)
    with torch.no_grad():
        got = model.hypernetwork(feats[..., :n], feats[..., n:], a_hat)
    sd = {k: v.numpy().astype(np.float64) for k, v in model.state_dict().items()}
    maxima = tuple(float(np.float32(v)) for v in (0.1, 0.99, 0.99, 0.99))   # float32 attributes
    want = gnn_np.hypernetwork(sd, feats.numpy(), graphs, maxima, mode == "same")
    for g, w in zip(got, want):
        np.testing.assert_allclose(g[..., 0, 0].numpy(), w, rtol=1e-10, atol=1e-12)


def test_forward_runs_cpu_tensors_on_the_cpu_path():
    """CPU tensors (the reference's default device) run dadmm_cpu's torch ops; the HIP library
    serves CUDA tensors only (tests/test_cpu_path.py checks the values)."""
    model = _model()
    b = torch.randn(3, 5, 8, 1)
    Y, hyp = model(b, [O.er_graph(5, 0.5, seed=1)] * 3)
    assert Y.device.type == "cpu" and model.last_backend == "cpu" and len(hyp) == 4


def test_forward_needs_one_graph_per_sample():
    model = _model()
    with pytest.raises(IndexError):
        model(torch.randn(3, 5, 8, 1), [O.er_graph(5, 0.5, seed=1)])


def test_hyper_caches_follow_live_modules_and_survive_deepcopy():
    """the hypernetwork's cached module tuples / parameter list are validated against
    the live model on every use (a replaced fc is seen), and they live outside the module, so a
    deepcopy of a model that ran carries no host plan (CDLL / ctypes structs)."""
    import argparse
    import copy

    import torch.nn as nn

    import gnn_dlasso_models_progressive as GM
    from dadmm_hip import hyper_ops
    args = argparse.Namespace(GHN_iter_num=3, GHyp_hidden=8, DADMM_mode="diff", alpha_max=0.1,
                              tau_max=0.99, rho_max=0.99, eta_max=0.99)
    model = GM.DLASSO_GNNHyp3_Progressive(torch.zeros(1, 3, 4, 16), args)
    p0 = hyper_ops.param_list(model)
    assert p0[-2] is model.fc.weight
    assert hyper_ops.param_list(model) is p0                 # cached while nothing changes
    model.fc = nn.Linear(8, 12)
    p1 = hyper_ops.param_list(model)
    assert p1[-2] is model.fc.weight and p1 is not p0
    assert hyper_ops._modules(model)[2][0] is model.decoder[0]
    model.decoder[0].weight = nn.Parameter(torch.zeros_like(model.decoder[0].weight))
    assert hyper_ops.param_list(model)[22] is model.decoder[0].weight
    assert not any(k.startswith("_hyper") or k.startswith("_native") for k in model.__dict__)
    twin = copy.deepcopy(model)
    assert hyper_ops.param_list(twin)[-2] is twin.fc.weight
