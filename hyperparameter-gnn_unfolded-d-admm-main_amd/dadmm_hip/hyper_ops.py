"""Inference-mode hypernetwork of DLASSO_GNNHyp3_Progressive on the HIP library (the
``dadmm_hyper_*`` entry points of include/dadmm.h).

``model.eval()`` under ``torch.no_grad()`` (the drivers' validation loop,
gnn_dlasso_progressive.py:240-265): Dropout is the identity and BatchNorm uses its running
statistics, so the whole GNNHypernetwork3 -> decoder -> fc -> head chain of one iteration
(gnn_dlasso_models_progressive.py:165-196) is 5 GCN-layer launches (f32 MFMA GEMM + normalised
adjacency mix + bias + leaky_relu + BatchNorm), one LayerNorm, three (split-K linear, LayerNorm +
LeakyReLU) pairs and one head launch that writes hyp_k [B, 4, H] — 13 launches for all B samples.
Training (autograd, Dropout draws, per-sample BatchNorm statistics) stays on the torch
composition in gnn_dlasso_models_progressive.py.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import _lib
from .ops import _ptr, _stream

LEAKY_SLOPE = 0.01   # F.leaky_relu / nn.LeakyReLU default negative_slope (reference :52-68, :97)


def supported(model, n: int) -> bool:
    """Whether ``model`` (a DLASSO_GNNHyp3_Progressive) can run its hypernetwork through the
    fused kernels: eval mode, standard BatchNorm / LayerNorm modules, every feature width a
    multiple of 4 (16-byte operand rows) and LayerNorm widths <= 2048."""
    if model.training:
        return False
    enc = model.encoder
    bns = (enc.bn1, enc.bn2, enc.bn3, enc.bn4, enc.bn5)
    if any(not (bn.track_running_stats and bn.affine and bn.running_mean is not None) for bn in bns):
        return False
    lns = [enc.norm] + [model.decoder[i] for i in (2, 6, 10)]
    if any(not isinstance(ln, nn.LayerNorm) or not ln.elementwise_affine or len(ln.normalized_shape) != 1
           for ln in lns):
        return False
    widths = [n, enc.conv1.lin.out_features, enc.conv2.lin.out_features, enc.conv3.lin.out_features,
              model.decoder[4].out_features, model.decoder[8].out_features]
    if any(w % 4 for w in widths):
        return False
    return all(ln.normalized_shape[0] <= 2048 for ln in lns)


class HyperBuffers:
    """Activation buffers of one forward (reused by every iteration), including the split-K
    partial sums of the three decoder linears."""

    def __init__(self, B, P, h4, dec_widths, H, device):
        L = _lib.load()
        self.x = [torch.empty((B * P, h4), device=device) for _ in range(2)]
        self.d = [torch.empty((B, w), device=device) for w in dec_widths]
        ins = [P * h4] + list(dec_widths[:-1])
        self.scratch = [torch.empty(max(L.dadmm_hyper_linear_ln_scratch_bytes(B, k, w), 16) // 4,
                                    device=device) for k, w in zip(ins, dec_widths)]
        self.hyp = torch.empty((B, 4, H), device=device)


def hypernetwork_eval(model, AtAy, Atb, n, ahat, per_sample, bufs: HyperBuffers):
    """(alpha, tau, rho, eta) of one iteration, each [B, H, 1, 1] (views of one [B, 4, H]
    tensor), from AtAy / Atb [B, P, n_store] (n columns used) and the normalised adjacency
    ``ahat`` [B or 1, P, P]."""
    L = _lib.load()
    B, P, ns = AtAy.shape
    dev = AtAy.device
    stream = _stream(dev)
    enc = model.encoder
    convs = (enc.conv1, enc.conv2, enc.conv3, enc.conv4, enc.conv5)
    bns = (enc.bn1, enc.bn2, enc.bn3, enc.bn4, enc.bn5)
    if n % 16 == 0:   # cat(AtAy, Atb) (:165) read in place from the two buffers
        x1, ld1, K1, x2, ld2, K = AtAy, ns, n, Atb, ns, 2 * n
    else:
        xc = torch.cat([AtAy[..., :n], Atb[..., :n]], dim=2).reshape(B * P, 2 * n).contiguous()
        x1, ld1, K1, x2, ld2, K = xc, 2 * n, 2 * n, None, 0, 2 * n
    with torch.cuda.device(dev):
        for i, (conv, bn) in enumerate(zip(convs, bns)):
            N = conv.lin.out_features
            y = bufs.x[i & 1]
            _lib.check("dadmm_hyper_gcn", L.dadmm_hyper_gcn(
                B, P, K, N, _ptr(x1), ld1, K1, _ptr(x2), ld2, _ptr(conv.lin.weight),
                _ptr(conv.bias), _ptr(ahat), int(per_sample), _ptr(bn.running_mean),
                _ptr(bn.running_var), _ptr(bn.weight), _ptr(bn.bias), float(bn.eps), LEAKY_SLOPE,
                _ptr(y), y.shape[1], stream))
            x1, ld1, K1, x2, ld2, K = y, y.shape[1], N, None, 0, N
        # self.norm (:69), in place on the last layer's output
        ln = enc.norm
        _lib.check("dadmm_hyper_rownorm", L.dadmm_hyper_rownorm(
            B * P, K, _ptr(x1), _ptr(ln.weight), _ptr(ln.bias), float(ln.eps), 0, 0.0, _ptr(x1),
            stream))
        # decoder (:93-105): Linear -> (Dropout) -> LayerNorm -> LeakyReLU, three times, on the
        # flattened [B, P * 4h] encoder output
        x, width = x1, P * K
        for blk, out in zip(range(3), bufs.d):
            lin, lnd = model.decoder[4 * blk], model.decoder[4 * blk + 2]
            N = lin.out_features
            _lib.check("dadmm_hyper_linear_ln", L.dadmm_hyper_linear_ln(
                B, width, N, _ptr(x), width, _ptr(lin.weight), _ptr(lin.bias), _ptr(lnd.weight),
                _ptr(lnd.bias), float(lnd.eps), 1, float(model.decoder[4 * blk + 3].negative_slope),
                _ptr(out), _ptr(bufs.scratch[blk]), stream))
            x, width = out, N
        H = bufs.hyp.shape[2]
        _lib.check("dadmm_hyper_head", L.dadmm_hyper_head(
            B, width, H, _ptr(x), width, _ptr(model.fc.weight), _ptr(model.fc.bias),
            float(model.alpha_max), float(model.tau_max), float(model.rho_max),
            float(model.eta_max), _ptr(bufs.hyp), stream))
    h = bufs.hyp
    return tuple(h[:, c].view(B, H, 1, 1) for c in range(4))
