"""numpy fp64 restatement of the GNN hypernetwork of DLASSO_GNNHyp3_Progressive (eval mode) —
TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Follows gnn_dlasso_models_progressive.py:9-72 (GNNHypernetwork3), :93-123 (decoder, fc) and
:167-196 (sigmoid, clamp, per-component scaling and clamps). torch_geometric is not installed and
its version is unpinned (requirements.txt:11), so GCNConv is restated from torch_geometric's
published algorithm in its own edge-list form (PARITY UNPINNED against torch_geometric):
  * from_networkx(G).edge_index: both directions of every undirected edge;
  * gcn_norm: add_remaining_self_loops (fill value 1), deg[i] = sum of weights of edges into i,
    norm(e: j -> i) = deg[j]^-1/2 * w * deg[i]^-1/2;
  * out[i] = sum over edges j -> i of norm * (x W^T)[j], then + bias.
Eval mode: BatchNorm1d uses its running statistics, Dropout is the identity.
"""
from __future__ import annotations

import numpy as np


def _edge_index(G, P):
    src, dst = [], []
    for u, v in G.edges():
        src += [u, v] if u != v else [u]
        dst += [v, u] if u != v else [u]
    have = {(s, d) for s, d in zip(src, dst)}
    for i in range(P):                      # add_remaining_self_loops
        if (i, i) not in have:
            src.append(i)
            dst.append(i)
    return np.asarray(src), np.asarray(dst)


def gcn_conv(x, W, bias, G, P):
    h = x @ W.T
    src, dst = _edge_index(G, P)
    deg = np.zeros(P)
    np.add.at(deg, dst, 1.0)
    dinv = deg ** -0.5
    norm = dinv[src] * dinv[dst]
    out = np.zeros((P, W.shape[0]))
    np.add.at(out, dst, norm[:, None] * h[src])
    return out + bias


def _leaky(x, slope=0.01):
    return np.where(x >= 0, x, slope * x)


def _layer_norm(x, w, b, eps=1e-5):
    mu = x.mean(-1, keepdims=True)
    var = x.var(-1, keepdims=True)
    return (x - mu) / np.sqrt(var + eps) * w + b


def hypernetwork(sd, features, graph_list, maxima, same_mode, eps=1e-5):
    """(alpha, tau, rho, eta) [B, H] in fp64 from node features [B, P, 2n].

    sd: the module's state_dict as float64 numpy arrays; maxima: (alpha_max, ..., eta_max)."""
    B, P, _ = features.shape
    outs = []
    for i in range(B):
        x = np.asarray(features[i], np.float64)
        for l in range(1, 6):
            x = gcn_conv(x, sd[f"encoder.conv{l}.lin.weight"], sd[f"encoder.conv{l}.bias"],
                         graph_list[i], P)
            x = _leaky(x)
            rm, rv = sd[f"encoder.bn{l}.running_mean"], sd[f"encoder.bn{l}.running_var"]
            x = (x - rm) / np.sqrt(rv + eps) * sd[f"encoder.bn{l}.weight"] + sd[f"encoder.bn{l}.bias"]
        x = _layer_norm(x, sd["encoder.norm.weight"], sd["encoder.norm.bias"])
        h = x.reshape(-1)
        for lin, ln in ((0, 2), (4, 6), (8, 10)):
            h = h @ sd[f"decoder.{lin}.weight"].T + sd[f"decoder.{lin}.bias"]
            h = _layer_norm(h, sd[f"decoder.{ln}.weight"], sd[f"decoder.{ln}.bias"])
            h = _leaky(h)
        h = h @ sd["fc.weight"].T + sd["fc.bias"]
        outs.append(h)
    h = np.clip(1.0 / (1.0 + np.exp(-np.stack(outs))), 1e-4, 0.9999)
    H = 1 if same_mode else P
    h = h.reshape(B, 4, H)
    am, tm, rm_, em = maxima
    return (h[:, 0] * am, np.minimum(h[:, 1] * tm, 0.9999), np.minimum(h[:, 2] * rm_, 0.9999),
            np.minimum(h[:, 3] * em, 0.9999))
