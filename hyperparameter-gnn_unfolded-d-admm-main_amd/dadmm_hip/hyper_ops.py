"""The hypernetwork of DLASSO_GNNHyp3_Progressive on the HIP library (the ``dadmm_hyper_*``
entry points of include/dadmm.h), in inference and in training mode.

``model.eval()`` under ``torch.no_grad()`` (the drivers' validation loop,
gnn_dlasso_progressive.py:240-265): Dropout is the identity and BatchNorm uses its running
statistics, so the whole GNNHypernetwork3 -> decoder -> fc -> head chain of one iteration
(gnn_dlasso_models_progressive.py:165-196) is 5 GCN-layer launches (f32 MFMA GEMM + normalised
adjacency mix + bias + leaky_relu + BatchNorm), one LayerNorm, three (split-K linear, LayerNorm +
LeakyReLU) pairs and one head launch that writes hyp_k [B, 4, H] — 13 launches for all B samples.

``model.train()`` (the drivers' training loop, gnn_dlasso_progressive.py:193-214): HyperTrainFn
(``hypernetwork_train``) runs the same GEMMs with training epilogues (per-sample BatchNorm batch
statistics, Dropout) and HIP backward kernels. Dropout is counter-based: element (row, col) of
site s is kept iff hash(seed, s, row, col) >= p 2^32, with one 62-bit seed per hypernetwork call
drawn from torch's CPU generator (``draw_dropout_seed``; torch.manual_seed fixes it, and
dist.seed_rank_streams gives every data-parallel rank its own). The backward regenerates the
masks from the seed instead of storing them.
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


# ---- training mode (model.train()) ------------------------------------------------------------

def supported_train(model, n: int) -> bool:
    """Whether the training-mode hypernetwork can run on the HIP kernels: train mode, the
    standard modules of the reference (Dropout, BatchNorm1d with affine + running statistics,
    LayerNorm), P >= 2 (batch statistics over the nodes) and 4-aligned feature widths."""
    if not model.training or model.P < 2:
        return False
    enc = model.encoder
    bns = (enc.bn1, enc.bn2, enc.bn3, enc.bn4, enc.bn5)
    if any(not (bn.affine and bn.track_running_stats and bn.momentum is not None) for bn in bns):
        return False
    drops = [enc.dropout] + [model.decoder[i] for i in (1, 5, 9)]
    if any(not isinstance(d, nn.Dropout) for d in drops):
        return False
    lns = [enc.norm] + [model.decoder[i] for i in (2, 6, 10)]
    if any(not isinstance(ln, nn.LayerNorm) or not ln.elementwise_affine or len(ln.normalized_shape) != 1
           or ln.normalized_shape[0] > 2048 for ln in lns):
        return False
    widths = [n, enc.conv1.lin.out_features, enc.conv2.lin.out_features, enc.conv3.lin.out_features,
              enc.conv5.lin.out_features, model.decoder[0].out_features, model.decoder[4].out_features,
              model.decoder[8].out_features]
    return all(w % 4 == 0 for w in widths)


def _hyper_params(model):
    """The hypernetwork's parameters in the order HyperTrainFn takes them."""
    enc = model.encoder
    out = []
    for conv, bn in zip((enc.conv1, enc.conv2, enc.conv3, enc.conv4, enc.conv5),
                        (enc.bn1, enc.bn2, enc.bn3, enc.bn4, enc.bn5)):
        out += [conv.lin.weight, conv.bias, bn.weight, bn.bias]
    out += [enc.norm.weight, enc.norm.bias]
    for blk in range(3):
        lin, ln = model.decoder[4 * blk], model.decoder[4 * blk + 2]
        out += [lin.weight, lin.bias, ln.weight, ln.bias]
    out += [model.fc.weight, model.fc.bias]
    return out


_RS_WEIGHTS = {}


def _rs_weights(T, m, device):
    """m (1 - m)^(T-1-t), t = 0 .. T-1 (float64; cached per length, momentum and device)."""
    key = (T, float(m), str(device))
    w = _RS_WEIGHTS.get(key)
    if w is None:
        if len(_RS_WEIGHTS) > 64:
            _RS_WEIGHTS.clear()
        w = m * (1.0 - m) ** torch.arange(T - 1, -1, -1, device=device, dtype=torch.float64)
        _RS_WEIGHTS[key] = w
    return w


def _update_running_stats(bn, mean, var, P):
    """bn's running statistics after the reference's sequential per-sample calls (train mode),
    in closed form: r <- (1 - m) r + m s_t for t = 0 .. T-1 (unbiased variance). mean / var are
    [T, N]: the B samples of one call, or those of several calls stacked in call order."""
    T = mean.shape[0]
    m = bn.momentum
    w = _rs_weights(T, m, mean.device)
    decay = (1.0 - m) ** T
    w = w[:, None]   # weighted sums over the calls as multiply + reduce (a float64 GEMV is slow)
    bn.running_mean.copy_((decay * bn.running_mean.double() + (w * mean.double()).sum(0)).float())
    bn.running_var.copy_((decay * bn.running_var.double() + (w * (var.double() * (P / (P - 1)))).sum(0)).float())
    bn.num_batches_tracked += T


def flush_running_stats(model):
    """Apply the BatchNorm running-statistics updates that training-mode hypernetwork calls with
    ``defer=True`` queued on ``model`` — one closed-form update per layer over every queued call,
    in call order (what the per-call updates give, without their per-iteration launches)."""
    pending = getattr(model, "_bn_pending", None)
    if not pending:
        return
    model._bn_pending = []
    with torch.no_grad():
        for i in range(len(pending[0][0])):
            bn = pending[0][0][i][0]
            P = pending[0][1]
            mean = torch.cat([call[0][i][1] for call in pending])
            var = torch.cat([call[0][i][2] for call in pending])
            _update_running_stats(bn, mean, var, P)


class HyperTrainFn(torch.autograd.Function):
    """hyp_k [B, 4, H] = the training-mode hypernetwork of one iteration
    (gnn_dlasso_models_progressive.py:165-196 with :52-72 in train mode) on the HIP kernels;
    differentiable w.r.t. AtAy_k and every hypernetwork parameter. Forward: the GCN layers as
    f32 MFMA GEMMs with the mix / leaky_relu / batch-statistics BatchNorm / Dropout epilogue
    (dadmm_hyper_gcn_train), LayerNorm, the decoder blocks (dadmm_hyper_linear_ln_train) and the
    head. Backward: dadmm_hyper_head_act / dadmm_hyper_rownorm_bwd / dadmm_hyper_gcn_train_bwd
    for everything but the linears' plain GEMMs (dW = dZ^T X, dX = dZ W: hipBLASLt via torch)."""

    @staticmethod
    def forward(ctx, AtAy, Atb, ahat, model, n, per_sample, seed, defer, *params):
        L = _lib.load()
        B, P, ns = AtAy.shape
        dev = AtAy.device
        stream = _stream(dev)
        enc = model.encoder
        convs = (enc.conv1, enc.conv2, enc.conv3, enc.conv4, enc.conv5)
        bns = (enc.bn1, enc.bn2, enc.bn3, enc.bn4, enc.bn5)
        p_enc = float(enc.dropout.p)
        rows = B * P
        if n % 16 == 0:   # cat(AtAy, Atb) (:165) read in place
            x1, ld1, K1, x2, ld2, K = AtAy, ns, n, Atb, ns, 2 * n
        else:
            xc = torch.cat([AtAy[..., :n], Atb[..., :n]], dim=2).reshape(rows, 2 * n).contiguous()
            x1, ld1, K1, x2, ld2, K = xc, 2 * n, 2 * n, None, 0, 2 * n
        saved = []          # per GCN layer: (M, mean, var)
        stats = []          # per GCN layer: (bn, mean, var) for the running statistics
        xs = []             # per GCN layer: its input rows (None for layer 1: rebuilt from AtAy / Atb)
        with torch.cuda.device(dev):
            for i, (conv, bn) in enumerate(zip(convs, bns)):
                N = conv.lin.out_features
                y = torch.empty((rows, N), device=dev)
                M = torch.empty((rows, N), device=dev)
                mean = torch.empty((B, N), device=dev)
                var = torch.empty((B, N), device=dev)
                _lib.check("dadmm_hyper_gcn_train", L.dadmm_hyper_gcn_train(
                    B, P, K, N, _ptr(x1), ld1, K1, _ptr(x2), ld2, _ptr(conv.lin.weight),
                    _ptr(conv.bias), _ptr(ahat), int(per_sample), _ptr(bn.weight), _ptr(bn.bias),
                    float(bn.eps), LEAKY_SLOPE, p_enc if i < 4 else 0.0, seed, i, _ptr(y), N, _ptr(M),
                    _ptr(mean), _ptr(var), stream))
                if defer:
                    stats.append((bn, mean, var))
                else:
                    with torch.no_grad():
                        _update_running_stats(bn, mean, var, P)
                saved.append((M, mean, var))
                xs.append(None if i == 0 else x1)
                x1, ld1, K1, x2, ld2, K = y, N, N, None, 0, N
            # self.norm (:69) over 4h per node, then the flattened decoder input
            ln = enc.norm
            x5 = x1
            e = torch.empty_like(x5)
            _lib.check("dadmm_hyper_rownorm", L.dadmm_hyper_rownorm(
                rows, K, _ptr(x5), _ptr(ln.weight), _ptr(ln.bias), float(ln.eps), 0, 0.0, _ptr(e), stream))
            x, width = e.view(B, P * K), P * K
            dec_in, dec_xd = [], []
            for blk in range(3):
                lin, lnd = model.decoder[4 * blk], model.decoder[4 * blk + 2]
                N = lin.out_features
                out = torch.empty((B, N), device=dev)
                xd = torch.empty((B, N), device=dev)
                scratch = torch.empty(max(L.dadmm_hyper_linear_ln_scratch_bytes(B, width, N), 16) // 4,
                                      device=dev)
                _lib.check("dadmm_hyper_linear_ln_train", L.dadmm_hyper_linear_ln_train(
                    B, width, N, _ptr(x), width, _ptr(lin.weight), _ptr(lin.bias), _ptr(lnd.weight),
                    _ptr(lnd.bias), float(lnd.eps), 1, float(model.decoder[4 * blk + 3].negative_slope),
                    float(model.decoder[4 * blk + 1].p), seed, 4 + blk, _ptr(out), _ptr(xd),
                    _ptr(scratch), stream))
                dec_in.append(x)
                dec_xd.append(xd)
                x, width = out, N
            H = model.fc.out_features // 4
            z = torch.empty((B, 4 * H), device=dev)
            _lib.check("dadmm_hyper_linear", L.dadmm_hyper_linear(
                B, width, 4 * H, _ptr(x), width, width, None, 0, _ptr(model.fc.weight),
                _ptr(model.fc.bias), _ptr(z), 4 * H, stream))
            hyp = torch.empty((B, 4, H), device=dev)
            mx = [float(model.alpha_max), float(model.tau_max), float(model.rho_max), float(model.eta_max)]
            _lib.check("dadmm_hyper_head_act", L.dadmm_hyper_head_act(
                0, B, H, _ptr(z), None, *mx, _ptr(hyp), stream))
        if defer:
            if not hasattr(model, "_bn_pending"):
                model._bn_pending = []
            model._bn_pending.append((stats, P))
        ctx.model, ctx.n, ctx.per_sample, ctx.seed, ctx.mx = model, n, per_sample, seed, mx
        ctx.saved = saved
        ctx.xs, ctx.x5, ctx.dec_in, ctx.dec_xd, ctx.x3, ctx.z = xs, x5, dec_in, dec_xd, x, z
        ctx.AtAy, ctx.Atb, ctx.ahat = AtAy, Atb, ahat
        return hyp

    @staticmethod
    def backward(ctx, dhyp):
        L = _lib.load()
        model, n = ctx.model, ctx.n
        AtAy, Atb = ctx.AtAy, ctx.Atb
        B, P, ns = AtAy.shape
        rows = B * P
        dev = AtAy.device
        stream = _stream(dev)
        enc = model.encoder
        convs = (enc.conv1, enc.conv2, enc.conv3, enc.conv4, enc.conv5)
        bns = (enc.bn1, enc.bn2, enc.bn3, enc.bn4, enc.bn5)
        p_enc = float(enc.dropout.p)
        H = model.fc.out_features // 4
        g = {}
        with torch.cuda.device(dev):
            dhyp = dhyp.contiguous()
            dz = torch.empty((B, 4 * H), device=dev)
            _lib.check("dadmm_hyper_head_act", L.dadmm_hyper_head_act(
                1, B, H, _ptr(ctx.z), _ptr(dhyp), *ctx.mx, _ptr(dz), stream))
            g["fc.w"] = dz.t() @ ctx.x3
            g["fc.b"] = dz.sum(0)
            dx = dz @ model.fc.weight
            for blk in (2, 1, 0):
                lin, lnd = model.decoder[4 * blk], model.decoder[4 * blk + 2]
                N = lin.out_features
                dv = torch.empty((B, N), device=dev)
                part = torch.empty(max(L.dadmm_hyper_rownorm_bwd_part_bytes(B, N), 16) // 4, device=dev)
                _lib.check("dadmm_hyper_rownorm_bwd", L.dadmm_hyper_rownorm_bwd(
                    B, N, _ptr(dx.contiguous()), _ptr(ctx.dec_xd[blk]), _ptr(lnd.weight), _ptr(lnd.bias),
                    float(lnd.eps), 1, float(model.decoder[4 * blk + 3].negative_slope),
                    float(model.decoder[4 * blk + 1].p), ctx.seed, 4 + blk, _ptr(dv), _ptr(part), stream))
                pw = part[:L.dadmm_hyper_rownorm_bwd_part_bytes(B, N) // 4].view(-1, 2, N).sum(0)
                g[f"ln{blk}.w"], g[f"ln{blk}.b"] = pw[0], pw[1]
                g[f"lin{blk}.w"] = dv.t() @ ctx.dec_in[blk]
                g[f"lin{blk}.b"] = dv.sum(0)
                dx = dv @ lin.weight
            # self.norm backward (no dropout, no activation): input x5 [rows, 4h]
            C = ctx.x5.shape[1]
            dx = dx.reshape(rows, C).contiguous()
            de = torch.empty((rows, C), device=dev)
            part = torch.empty(max(L.dadmm_hyper_rownorm_bwd_part_bytes(rows, C), 16) // 4, device=dev)
            ln = enc.norm
            _lib.check("dadmm_hyper_rownorm_bwd", L.dadmm_hyper_rownorm_bwd(
                rows, C, _ptr(dx), _ptr(ctx.x5), _ptr(ln.weight), _ptr(ln.bias), float(ln.eps), 0, 0.0,
                0.0, ctx.seed, 99, _ptr(de), _ptr(part), stream))
            pw = part[:L.dadmm_hyper_rownorm_bwd_part_bytes(rows, C) // 4].view(-1, 2, C).sum(0)
            g["norm.w"], g["norm.b"] = pw[0], pw[1]
            dx = de
            for i in (4, 3, 2, 1, 0):
                conv, bn = convs[i], bns[i]
                N = conv.lin.out_features
                M, mean, var = ctx.saved[i]
                dZ = torch.empty((rows, N), device=dev)
                part = torch.empty((3, B, N), device=dev)
                _lib.check("dadmm_hyper_gcn_train_bwd", L.dadmm_hyper_gcn_train_bwd(
                    B, P, N, _ptr(dx.contiguous()), _ptr(M), _ptr(mean), _ptr(var), _ptr(bn.weight),
                    float(bn.eps), _ptr(ctx.ahat), int(ctx.per_sample), LEAKY_SLOPE,
                    p_enc if i < 4 else 0.0, ctx.seed, i, _ptr(dZ), _ptr(part), stream))
                ps = part.sum(1)
                g[f"bn{i}.w"], g[f"bn{i}.b"], g[f"conv{i}.b"] = ps[0], ps[1], ps[2]
                xin = ctx.xs[i]
                if xin is None:
                    xin = torch.cat([AtAy[..., :n], Atb[..., :n]], dim=2).reshape(rows, 2 * n)
                g[f"conv{i}.w"] = dZ.t() @ xin
                dx = dZ @ conv.lin.weight
            dAtAy = torch.zeros_like(AtAy)
            dAtAy[..., :n] = dx.reshape(B, P, 2 * n)[..., :n]
        grads = []
        for i in range(5):
            grads += [g[f"conv{i}.w"], g[f"conv{i}.b"], g[f"bn{i}.w"], g[f"bn{i}.b"]]
        grads += [g["norm.w"], g["norm.b"]]
        for blk in range(3):
            grads += [g[f"lin{blk}.w"], g[f"lin{blk}.b"], g[f"ln{blk}.w"], g[f"ln{blk}.b"]]
        grads += [g["fc.w"], g["fc.b"]]
        ctx.saved = ctx.xs = ctx.dec_in = ctx.dec_xd = None
        return (dAtAy, None, None, None, None, None, None, None, *grads)


def draw_dropout_seed() -> int:
    """The dropout stream of one training-mode hypernetwork call, from torch's CPU generator."""
    return int(torch.randint(0, 2 ** 62, (1,)).item())


def hypernetwork_train(model, AtAy, Atb, n, ahat, per_sample, seed=None, defer=False):
    """hyp_k [B, 4, H] of one iteration in training mode (HyperTrainFn); ``seed`` names the
    dropout stream (default: drawn from torch's CPU generator, so torch.manual_seed fixes it).
    defer: queue the BatchNorm running-statistics update on ``model`` for flush_running_stats
    (the model's forward flushes once after its K iterations)."""
    if seed is None:
        seed = draw_dropout_seed()
    return HyperTrainFn.apply(AtAy, Atb, ahat, model, n, per_sample, seed, defer, *_hyper_params(model))
