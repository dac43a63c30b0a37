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

import ctypes
import os
import weakref

import torch
import torch.nn as nn

from . import _lib
from .ops import _ptr, _stream

LEAKY_SLOPE = 0.01   # F.leaky_relu / nn.LeakyReLU default negative_slope (reference :52-68, :97)


def supported(model, n: int) -> bool:
    """Whether ``model`` (a DLASSO_GNNHyp3_Progressive) can run its hypernetwork through the
    fused kernels: eval mode, standard BatchNorm / LayerNorm modules, every hidden feature width
    a multiple of 4 (16-byte operand rows) and LayerNorm widths <= 2048. Any n: layer 1's input
    cat(AtAy, Atb) of width 2n is zero-padded to a multiple of 4 (``layer1_input``)."""
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
    widths = [enc.conv1.lin.out_features, enc.conv2.lin.out_features, enc.conv3.lin.out_features,
              model.decoder[4].out_features, model.decoder[8].out_features]
    if any(w % 4 for w in widths):
        return False
    return all(ln.normalized_shape[0] <= 2048 for ln in lns)


def layer1_input(model, AtAy, Atb, n):
    """Layer 1's operands when cat(AtAy, Atb) (:165) cannot be read in place (n % 16 != 0):
    (x [B*P, Kp], W1 [N, Kp], Kp) with Kp = 2n rounded up to a multiple of 4 (16-byte rows, what
    the GEMM kernels read); the padding columns of x and of the weight copy are zero, so
    x W1^T is the unpadded product (the extra terms are exact zeros). The weight copy is one
    buffer per model, refreshed from conv1's weight on every call (captured HIP graphs included)."""
    B, P, _ = AtAy.shape
    K = 2 * n
    Kp = (K + 3) & ~3
    x = torch.cat([AtAy[..., :n], Atb[..., :n]], dim=2).reshape(B * P, K)
    w = model.encoder.conv1.lin.weight
    if Kp == K:
        return x.contiguous(), w, K
    x = torch.nn.functional.pad(x, (0, Kp - K))
    ent = _cache(model)
    wp = ent.get("w1_padded")
    if wp is None or wp.shape != (w.shape[0], Kp) or wp.device != w.device:
        wp = ent["w1_padded"] = torch.zeros((w.shape[0], Kp), device=w.device, dtype=w.dtype)
    with torch.no_grad():
        wp[:, :K].copy_(w)
    return x, wp, Kp


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
        self.c1 = None          # layer 1's Atb half, A_hat (Atb W1[:, n:]^T) (hypernetwork_eval_prepare)


def hypernetwork_eval_prepare(model, Atb, n, ahat, per_sample, bufs: HyperBuffers):
    """Once per forward: layer 1's input is cat(AtAy_k, Atb) (:165) and Atb does not change between
    iterations, so its half of the GCNConv, A_hat (Atb W1[:, n:]^T), is formed here once (raw
    dadmm_hyper_gcn_ex) and every iteration's layer 1 runs its GEMM over AtAy_k alone (half the
    K depth) with this term added before the bias. Needs n % 16 == 0 (the in-place cat layout)."""
    if n % 16 or os.environ.get("DADMM_HYPER_ATB_HOIST", "1") == "0":   # (the env switch: A/B timing)
        bufs.c1 = None
        return
    L = _lib.load()
    B, P, ns = Atb.shape
    conv = model.encoder.conv1
    N = conv.lin.out_features
    if bufs.c1 is None or bufs.c1.shape != (B * P, N):
        bufs.c1 = torch.empty((B * P, N), device=Atb.device)
    w = conv.lin.weight
    with torch.cuda.device(Atb.device):
        _lib.check("dadmm_hyper_gcn_ex", L.dadmm_hyper_gcn_ex(
            B, P, n, N, _ptr(Atb), ns, w.data_ptr() + 4 * n, w.shape[1], None, 0, None, _ptr(ahat),
            int(per_sample), None, None, None, None, 0.0, 0.0, 1, _ptr(bufs.c1), N, _stream(Atb.device)))


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
    w1 = model.encoder.conv1.lin.weight
    if n % 16 == 0:   # cat(AtAy, Atb) (:165) read in place from the two buffers
        x1, ld1, K1, x2, ld2, K = AtAy, ns, n, Atb, ns, 2 * n
    else:
        xc, w1, Kp = layer1_input(model, AtAy, Atb, n)
        x1, ld1, K1, x2, ld2, K = xc, Kp, Kp, None, 0, Kp
    with torch.cuda.device(dev):
        for i, (conv, bn) in enumerate(zip(convs, bns)):
            N = conv.lin.out_features
            y = bufs.x[i & 1]
            if i == 0 and bufs.c1 is not None and K1 < K:
                # the AtAy half only; the Atb half comes from hypernetwork_eval_prepare
                w = conv.lin.weight
                _lib.check("dadmm_hyper_gcn_ex", L.dadmm_hyper_gcn_ex(
                    B, P, K1, N, _ptr(x1), ld1, _ptr(w), w.shape[1], _ptr(bufs.c1), N, _ptr(conv.bias),
                    _ptr(ahat), int(per_sample), _ptr(bn.running_mean), _ptr(bn.running_var),
                    _ptr(bn.weight), _ptr(bn.bias), float(bn.eps), LEAKY_SLOPE, 0, _ptr(y), y.shape[1], stream))
                x1, ld1, K1, x2, ld2, K = y, y.shape[1], N, None, 0, N
                continue
            _lib.check("dadmm_hyper_gcn", L.dadmm_hyper_gcn(
                B, P, K, N, _ptr(x1), ld1, K1, _ptr(x2), ld2, _ptr(w1 if i == 0 else conv.lin.weight),
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
    """Whether the differentiable hypernetwork can run on the HIP training kernels: the standard
    modules of the reference (Dropout, BatchNorm1d with affine + running statistics, LayerNorm),
    P >= 2 and 4-aligned feature widths. In train mode the BatchNorms use the samples' batch
    statistics and the Dropouts their p; in eval mode (a backward through model.eval(), e.g.
    torch.autograd.grad of a validation loss) the same kernels run with the running statistics
    and no dropout (the network torch's eval mode computes)."""
    if model.P < 2:
        return False
    enc = model.encoder
    bns = (enc.bn1, enc.bn2, enc.bn3, enc.bn4, enc.bn5)
    if any(not (bn.affine and bn.track_running_stats and bn.momentum is not None
                and bn.running_mean is not None) for bn in bns):
        return False
    drops = [enc.dropout] + [model.decoder[i] for i in (1, 5, 9)]
    if any(not isinstance(d, nn.Dropout) for d in drops):
        return False
    lns = [enc.norm] + [model.decoder[i] for i in (2, 6, 10)]
    if any(not isinstance(ln, nn.LayerNorm) or not ln.elementwise_affine or len(ln.normalized_shape) != 1
           or ln.normalized_shape[0] > 2048 for ln in lns):
        return False
    # (any n: layer 1's 2n-wide input is zero-padded to a multiple of 4 by layer1_input)
    widths = [enc.conv1.lin.out_features, enc.conv2.lin.out_features, enc.conv3.lin.out_features,
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
    if mean.dim() == 3:   # [iterations, B, N] blocks of a whole forward: the calls in order
        mean, var = mean.reshape(-1, mean.shape[2]), var.reshape(-1, var.shape[2])
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
            mean = torch.cat([call[0][i][1].reshape(-1, call[0][i][1].shape[-1]) for call in pending])
            var = torch.cat([call[0][i][2].reshape(-1, call[0][i][2].shape[-1]) for call in pending])
            _update_running_stats(bn, mean, var, P)


class HyperTrainFn(torch.autograd.Function):
    """hyp_k [B, 4, H] = the training-mode hypernetwork of one iteration
    (gnn_dlasso_models_progressive.py:165-196 with :52-72 in train mode) on the HIP kernels;
    differentiable w.r.t. AtAy_k and every hypernetwork parameter. Forward: the GCN layers as
    f32 MFMA GEMMs with the mix / leaky_relu / batch-statistics BatchNorm / Dropout epilogue
    (dadmm_hyper_gcn_train), LayerNorm, the decoder blocks (dadmm_hyper_linear_ln_train) and the
    head. Backward: dadmm_hyper_head_act / dadmm_hyper_rownorm_bwd / dadmm_hyper_gcn_train_bwd,
    and the linears' GEMMs on the library's own kernels too (dW = dZ^T X: dadmm_hyper_wgrad,
    csrc/dadmm_hyper_grad.hip; dX = dZ W: dadmm_hyper_linear with W^T) — no hipBLASLt."""

    @staticmethod
    def forward(ctx, AtAy, Atb, ahat, model, n, per_sample, seed, defer, *params):
        L = _lib.load()
        B, P, ns = AtAy.shape
        ctx.n_params = len(params)
        ctx.native = n % 16 == 0 and B > 0
        if ctx.native:   # the whole call in one library entry point (csrc/dadmm_hyper_net.cpp)
            return _native_forward(ctx, L, AtAy, Atb, ahat, model, n, per_sample, seed, defer)
        dev = AtAy.device
        stream = _stream(dev)
        enc = model.encoder
        convs = (enc.conv1, enc.conv2, enc.conv3, enc.conv4, enc.conv5)
        bns = (enc.bn1, enc.bn2, enc.bn3, enc.bn4, enc.bn5)
        train = model.training
        ctx.train = train
        # eval mode: Dropout is the identity and BatchNorm normalises with its running statistics
        p_enc = float(enc.dropout.p) if train else 0.0
        rows = B * P
        w1 = enc.conv1.lin.weight
        if n % 16 == 0:   # cat(AtAy, Atb) (:165) read in place
            x1, ld1, K1, x2, ld2, K = AtAy, ns, n, Atb, ns, 2 * n
        else:
            xc, w1, Kp = layer1_input(model, AtAy, Atb, n)
            x1, ld1, K1, x2, ld2, K = xc, Kp, Kp, None, 0, Kp
        x1in = (x1, ld1, K1, x2, ld2)   # layer 1's input, for its weight gradient
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
                    B, P, K, N, _ptr(x1), ld1, K1, _ptr(x2), ld2, _ptr(w1 if i == 0 else conv.lin.weight),
                    _ptr(conv.bias), _ptr(ahat), int(per_sample), _ptr(bn.weight), _ptr(bn.bias),
                    float(bn.eps), LEAKY_SLOPE, p_enc if i < 4 else 0.0, seed, i, _ptr(y), N, _ptr(M),
                    _ptr(mean), _ptr(var), None if train else _ptr(bn.running_mean),
                    None if train else _ptr(bn.running_var), stream))
                if train and defer:   # (eval mode: the running statistics are inputs, not updated)
                    stats.append((bn, mean, var))
                elif train:
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
                    float(model.decoder[4 * blk + 1].p) if train else 0.0, seed, 4 + blk, _ptr(out), _ptr(xd),
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
        if defer and train:
            if not hasattr(model, "_bn_pending"):
                model._bn_pending = []
            model._bn_pending.append((stats, P))
        ctx.model, ctx.n, ctx.per_sample, ctx.seed, ctx.mx = model, n, per_sample, seed, mx
        ctx.x1in = x1in
        ctx.saved = saved
        ctx.xs, ctx.x5, ctx.dec_in, ctx.dec_xd, ctx.x3, ctx.z = xs, x5, dec_in, dec_xd, x, z
        ctx.AtAy, ctx.Atb, ctx.ahat = AtAy, Atb, ahat
        return hyp

    @staticmethod
    def backward(ctx, dhyp):
        """The reverse of forward on the HIP kernels: head, decoder and encoder backward kernels,
        the parameter gradients of every linear by dadmm_hyper_wgrad (f32 MFMA, accumulated in
        place) and the partial sums by dadmm_hyper_colsum, all into the backward pass's flat
        gradient buffer (_GradAccumulator: one per loss.backward(), whose end callback hands the
        sums to the parameters' .grad); the input gradients dX = dZ W by dadmm_hyper_linear with
        the transposed weights. Returns only d AtAy: autograd adds nothing per call."""
        L = _lib.load()
        if ctx.native:
            return _native_backward(ctx, L, dhyp)
        model, n = ctx.model, ctx.n
        AtAy, Atb = ctx.AtAy, ctx.Atb
        B, P, ns = AtAy.shape
        rows = B * P
        dev = AtAy.device
        stream = _stream(dev)
        enc = model.encoder
        convs = (enc.conv1, enc.conv2, enc.conv3, enc.conv4, enc.conv5)
        bns = (enc.bn1, enc.bn2, enc.bn3, enc.bn4, enc.bn5)
        train = ctx.train
        p_enc = float(enc.dropout.p) if train else 0.0
        H = model.fc.out_features // 4
        acc = _GradAccumulator.current(model, dev)
        chk = _lib.check
        with torch.cuda.device(dev):
            dhyp = dhyp.contiguous()
            dz = torch.empty((B, 4 * H), device=dev)
            chk("dadmm_hyper_head_act", L.dadmm_hyper_head_act(
                1, B, H, _ptr(ctx.z), _ptr(dhyp), *ctx.mx, _ptr(dz), stream))
            fc = model.fc
            hid = fc.in_features
            acc.wgrad(B, 4 * H, hid, dz, 4 * H, ctx.x3, hid, hid, None, 0, fc.weight, fc.bias)
            dx = acc.input_grad(B, dz, 4 * H, fc.weight)            # [B, hid]
            for blk in (2, 1, 0):
                lin, lnd = model.decoder[4 * blk], model.decoder[4 * blk + 2]
                N, Kin = lin.out_features, lin.in_features
                dv = torch.empty((B, N), device=dev)
                nbytes = L.dadmm_hyper_rownorm_bwd_part_bytes(B, N)
                part = torch.empty(max(nbytes, 16) // 4, device=dev)
                chk("dadmm_hyper_rownorm_bwd", L.dadmm_hyper_rownorm_bwd(
                    B, N, _ptr(dx), _ptr(ctx.dec_xd[blk]), _ptr(lnd.weight), _ptr(lnd.bias),
                    float(lnd.eps), 1, float(model.decoder[4 * blk + 3].negative_slope),
                    float(model.decoder[4 * blk + 1].p) if train else 0.0, ctx.seed, 4 + blk, _ptr(dv),
                    _ptr(part), stream))
                acc.colsum(part, 1, nbytes // (4 * 2 * N), 2 * N, lnd.weight)   # -> ln.weight, ln.bias
                acc.wgrad(B, N, Kin, dv, N, ctx.dec_in[blk], Kin, Kin, None, 0, lin.weight, lin.bias)
                dx = acc.input_grad(B, dv, N, lin.weight)           # [B, Kin]
            # self.norm backward (no dropout, no activation): input x5 [rows, 4h]
            C = ctx.x5.shape[1]
            de = torch.empty((rows, C), device=dev)
            nbytes = L.dadmm_hyper_rownorm_bwd_part_bytes(rows, C)
            part = torch.empty(max(nbytes, 16) // 4, device=dev)
            ln = enc.norm
            chk("dadmm_hyper_rownorm_bwd", L.dadmm_hyper_rownorm_bwd(
                rows, C, _ptr(dx), _ptr(ctx.x5), _ptr(ln.weight), _ptr(ln.bias), float(ln.eps), 0, 0.0,
                0.0, ctx.seed, 99, _ptr(de), _ptr(part), stream))
            acc.colsum(part, 1, nbytes // (4 * 2 * C), 2 * C, ln.weight)        # -> norm.weight, .bias
            dx = de
            dAtAy = torch.zeros_like(AtAy) if ns != n else torch.empty_like(AtAy)
            for i in (4, 3, 2, 1, 0):
                conv, bn = convs[i], bns[i]
                N = conv.lin.out_features
                M, mean, var = ctx.saved[i]
                dZ = torch.empty((rows, N), device=dev)
                part = torch.empty((3, B, N), device=dev)
                chk("dadmm_hyper_gcn_train_bwd", L.dadmm_hyper_gcn_train_bwd(
                    B, P, N, _ptr(dx), _ptr(M), _ptr(mean), _ptr(var), _ptr(bn.weight),
                    float(bn.eps), _ptr(ctx.ahat), int(ctx.per_sample), LEAKY_SLOPE,
                    p_enc if i < 4 else 0.0, ctx.seed, i, _ptr(dZ), _ptr(part), int(not train), stream))
                acc.colsum(part, 3, B, N, bn.weight)          # -> bn.weight, bn.bias, conv.bias
                Kin = conv.lin.in_features
                if i == 0:
                    # layer 1's input cat(AtAy, Atb) (read in place, or zero-padded to Kp columns
                    # by layer1_input); only d AtAy is needed
                    x1, ld1, K1, x2, ld2 = ctx.x1in
                    if x2 is None and K1 != Kin:   # padded: dW1 = the first 2n columns
                        acc.wgrad_cols(rows, N, K1, dZ, N, x1, ld1, conv.lin.weight, Kin)
                    else:
                        acc.wgrad(rows, N, Kin, dZ, N, x1, ld1, K1, x2, ld2, conv.lin.weight, None)
                    acc.input_grad(rows, dZ, N, conv.lin.weight, cols=n, out=dAtAy, ldo=ns)
                else:
                    acc.wgrad(rows, N, Kin, dZ, N, ctx.xs[i], Kin, Kin, None, 0, conv.lin.weight, None)
                    dx = acc.input_grad(rows, dZ, N, conv.lin.weight)
        ctx.saved = ctx.xs = ctx.dec_in = ctx.dec_xd = None
        return (dAtAy, None, None, None, None, None, None, None) + (None,) * ctx.n_params


# ---- one library call per iteration (dadmm_hyper_train_forward / _backward) -------------------

_N_SAVED = 29   # pointers in dadmm_hyper_saved: y, m, mean, var [5] each, e, dec_y [3], dec_xd [3], z, hyp


# Per-model host caches (module tuples, the parameter list, the native plans), kept OUTSIDE the
# module so that copy.deepcopy / pickling of a model never sees them, and validated on every use
# against the model's live structure (a replaced submodule or Parameter rebuilds them).
_CACHE = weakref.WeakKeyDictionary()


def _structure_key(model):
    """ids of the hypernetwork's live submodules and Parameters, read from the modules' own
    dicts (no nn.Module.__getattr__, a few microseconds): ``model.fc = nn.Linear(...)`` or a new
    Parameter object anywhere in the encoder / decoder / fc changes it."""
    mm = model._modules
    key = [id(v) for v in mm.values()]
    for top in ("encoder", "decoder"):
        for v in mm[top]._modules.values():
            key.append(id(v))
            key += [id(p) for p in v._parameters.values()]
            for c in v._modules.values():            # GCNConv.lin
                key.append(id(c))
                key += [id(p) for p in c._parameters.values()]
    key += [id(p) for p in mm["fc"]._parameters.values()]
    return tuple(key)


def _cache(model):
    """The model's cache entry, emptied when its structure changed since it was filled."""
    key = _structure_key(model)
    ent = _CACHE.get(model)
    if ent is None or ent["key"] != key:
        ent = {"key": key, "plans": {}}
        _CACHE[model] = ent
    return ent


def _modules(model):
    """(convs, bns, decoder linears, decoder layernorms, decoder dropouts, decoder activations),
    cached per model structure (nn.Module attribute lookups dominate the per-iteration host
    cost)."""
    ent = _cache(model)
    mods = ent.get("mods")
    if mods is None:
        enc = model.encoder
        dec = model.decoder
        mods = ((enc.conv1, enc.conv2, enc.conv3, enc.conv4, enc.conv5),
                (enc.bn1, enc.bn2, enc.bn3, enc.bn4, enc.bn5),
                tuple(dec[4 * j] for j in range(3)), tuple(dec[4 * j + 2] for j in range(3)),
                tuple(dec[4 * j + 1] for j in range(3)), tuple(dec[4 * j + 3] for j in range(3)))
        ent["mods"] = mods
    return mods


class NativeHyperPlan:
    """The training hypernetwork of ``model`` for batches of B samples on one device, as the
    dadmm_hyper_net struct (parameter pointers, dimensions, constants), the layout of one
    iteration's saved activations (``per`` floats: the dadmm_hyper_saved slices, 16-byte aligned)
    and the shared work buffer. ``NativeHyperPlan.get`` rebuilds it when a parameter's storage, a
    dropout p or a maximum changes."""

    def __init__(self, model, B, P, n, ns, dev, key):
        self.L = L = _lib.load()
        self.key = key
        self.B, self.P, self.n, self.ns, self.dev = B, P, n, ns, dev
        convs, bns, lins, lns, drops, acts = _modules(model)
        enc = model.encoder
        net = _lib.HyperNet()
        net.P, net.n, net.ld = P, n, ns
        for i, (conv, bn) in enumerate(zip(convs, bns)):
            net.width[i] = conv.lin.out_features
            net.conv_w[i], net.conv_b[i] = conv.lin.weight.data_ptr(), conv.bias.data_ptr()
            net.bn_w[i], net.bn_b[i], net.bn_eps[i] = bn.weight.data_ptr(), bn.bias.data_ptr(), float(bn.eps)
        net.norm_w, net.norm_b, net.norm_eps = enc.norm.weight.data_ptr(), enc.norm.bias.data_ptr(), float(enc.norm.eps)
        for j in range(3):
            net.dec_width[j] = lins[j].out_features
            net.dec_w[j], net.dec_b[j] = lins[j].weight.data_ptr(), lins[j].bias.data_ptr()
            net.ln_w[j], net.ln_b[j], net.ln_eps[j] = lns[j].weight.data_ptr(), lns[j].bias.data_ptr(), float(lns[j].eps)
            net.dec_slope[j] = float(acts[j].negative_slope)
            net.dec_drop[j] = float(drops[j].p) if model.training else 0.0
        net.H = model.fc.out_features // 4
        net.fc_w, net.fc_b = model.fc.weight.data_ptr(), model.fc.bias.data_ptr()
        net.drop_enc = float(enc.dropout.p) if model.training else 0.0
        for c, v in enumerate((model.alpha_max, model.tau_max, model.rho_max, model.eta_max)):
            net.maxv[c] = float(v)
        # eval mode (model.eval() under autograd): BatchNorm on the running statistics, no dropout
        net.bn_eval = 0 if model.training else 1
        for i, bn in enumerate(bns):
            net.bn_rm[i], net.bn_rv[i] = bn.running_mean.data_ptr(), bn.running_var.data_ptr()
        self.train = model.training
        self.net = net
        self.bns = bns
        self.H = H = net.H
        rows = B * P
        W = [net.width[i] for i in range(5)]
        DW = [net.dec_width[j] for j in range(3)]
        self.W = W
        sizes = ([rows * w for w in W] * 2 + [B * w for w in W] * 2 + [rows * W[4]] + [B * d for d in DW] * 2
                 + [B * 4 * H, B * 4 * H])
        assert len(sizes) == _N_SAVED
        offs, o = [], 0
        for sz in sizes:
            offs.append(o)
            o += (sz + 3) & ~3
        self.offs = offs            # float offsets of the 29 slices in one iteration's block
        self.per = o                # floats per iteration
        self.offs_b = torch.tensor(offs, dtype=torch.int64) * 4
        nbytes = L.dadmm_hyper_train_work_bytes(ctypes.byref(net), B)
        if nbytes == 0:
            raise ValueError("dadmm_hyper_train_work_bytes: hypernetwork dimensions not supported")
        self.work = torch.empty(nbytes // 4 + 4, device=dev)
        self.dAtAy = None
        self.wscratch = None
        self.bn_scratch = None
        self.c1 = None              # layer 1's Atb half (atb_mix), one buffer per plan
        self.dsave_per = L.dadmm_hyper_train_dsave_floats(ctypes.byref(net), B)   # floats, multiple of 4

    @staticmethod
    def get(model, B, P, n, ns, dev):
        convs, bns, lins, lns, drops, _ = _modules(model)
        params = param_list(model)
        key = (B, P, n, ns, dev, tuple(p.data_ptr() for p in params), float(model.encoder.dropout.p),
               tuple(float(d.p) for d in drops), model.training,
               tuple((bn.running_mean.data_ptr(), bn.running_var.data_ptr()) for bn in bns),
               (float(model.alpha_max), float(model.tau_max), float(model.rho_max), float(model.eta_max)))
        plans = _cache(model)["plans"]
        plan = plans.get((B, dev, model.training))
        if plan is None or plan.key != key:
            if len(plans) > 8:
                plans.clear()
            plan = NativeHyperPlan(model, B, P, n, ns, dev, key)
            plans[(B, dev, model.training)] = plan
        return plan

    def saved(self, arena, k=0):
        """dadmm_hyper_saved of iteration block k of ``arena`` (blocks of ``per`` floats)."""
        ptrs = self.offs_b + (arena.data_ptr() + 4 * k * self.per)
        return _lib.HyperSaved.from_buffer_copy(ptrs.numpy().tobytes())

    def hyp(self, arena, k=0):
        o = k * self.per + self.offs[28]
        return arena[o:o + self.B * 4 * self.H].view(self.B, 4, self.H)

    def stats(self, arena, iters):
        """[(bn, mean [iters, B, N], var [iters, B, N])] of the GCN blocks over ``iters`` blocks."""
        blocks = arena[:iters * self.per].view(iters, self.per)
        out = []
        for i, bn in enumerate(self.bns):
            n = self.B * self.W[i]
            mean = blocks[:, self.offs[10 + i]:self.offs[10 + i] + n].view(iters, self.B, self.W[i])
            var = blocks[:, self.offs[15 + i]:self.offs[15 + i] + n].view(iters, self.B, self.W[i])
            out.append((bn, mean, var))
        return out

    def update_running_stats(self, arena, iters, stream):
        """The GCN blocks' BatchNorm running statistics after the training-mode calls of ``iters``
        blocks of ``arena`` (iters * B per-sample calls in order): _update_running_stats's closed
        form in one dadmm_hyper_bn_running_update (two launches for all five layers, in place of
        ~16 torch launches per layer). Falls back to the torch form when the layers' momenta differ
        or one is None (cumulative averaging)."""
        moms = {bn.momentum for bn in self.bns}
        if len(moms) != 1 or None in moms or any(bn.num_batches_tracked is None for bn in self.bns):
            queue_running_stats(None, self.stats(arena, iters), self.P, False)
            return
        m = moms.pop()
        T = iters * self.B
        nl = len(self.bns)
        widths = (ctypes.c_int32 * nl)(*self.W[:nl])
        vp = ctypes.c_void_p * nl
        base = arena.data_ptr()
        nbytes = self.L.dadmm_hyper_bn_running_scratch_bytes(nl, widths, iters, self.B)
        if self.bn_scratch is None or 4 * self.bn_scratch.numel() < nbytes:
            self.bn_scratch = torch.empty((nbytes + 3) // 4, device=self.dev)
        _lib.check("dadmm_hyper_bn_running_update", self.L.dadmm_hyper_bn_running_update(
            nl, widths, vp(*[bn.running_mean.data_ptr() for bn in self.bns]),
            vp(*[bn.running_var.data_ptr() for bn in self.bns]),
            vp(*[bn.num_batches_tracked.data_ptr() for bn in self.bns]),
            vp(*[base + 4 * self.offs[10 + i] for i in range(nl)]),
            vp(*[base + 4 * self.offs[15 + i] for i in range(nl)]),
            self.per, iters, self.B, self.P, _ptr(_rs_weights(T, m, self.dev)), (1.0 - m) ** T,
            _ptr(self.bn_scratch), stream))

    def atb_mix(self, Atb, ahat, per_sample, stream):
        """Layer 1's Atb half A_hat (Atb W1[:, n:]^T), once per forward (dadmm_hyper_train_atb_mix),
        for forward(..., atb_mix=); None where the in-place two-segment layout does not apply."""
        if self.n % 16 or os.environ.get("DADMM_HYPER_ATB_HOIST", "1") == "0":   # (env: A/B timing)
            return None
        if self.c1 is None:
            self.c1 = torch.empty((self.B * self.P, self.W[0]), device=self.dev)
        _lib.check("dadmm_hyper_train_atb_mix", self.L.dadmm_hyper_train_atb_mix(
            ctypes.byref(self.net), self.B, _ptr(Atb), _ptr(ahat), int(per_sample), _ptr(self.c1), stream))
        return self.c1

    def forward(self, AtAy, Atb, ahat, per_sample, seed, sv, stream, atb_mix=None):
        _lib.check("dadmm_hyper_train_forward_ex", self.L.dadmm_hyper_train_forward_ex(
            ctypes.byref(self.net), self.B, _ptr(AtAy), _ptr(Atb), _ptr(atb_mix), _ptr(ahat), int(per_sample),
            seed, ctypes.byref(sv), _ptr(self.work), stream))

    def backward(self, AtAy, Atb, ahat, per_sample, seed, sv, dhyp, g, stream):
        """d AtAy (a buffer of the plan, overwritten by the next call) from d hyp; the parameter
        gradients are added into ``g``'s accumulators."""
        if self.dAtAy is None:   # columns n .. ns stay zero: the kernels write the first n
            self.dAtAy = torch.zeros((self.B, self.P, self.ns), device=self.dev)
        _lib.check("dadmm_hyper_train_backward", self.L.dadmm_hyper_train_backward(
            ctypes.byref(self.net), self.B, _ptr(AtAy), _ptr(Atb), _ptr(ahat), int(per_sample), seed,
            ctypes.byref(sv), _ptr(dhyp), ctypes.byref(g), _ptr(self.dAtAy), _ptr(self.work), stream))
        return self.dAtAy

    def backward_deferred(self, AtAy, Atb, ahat, per_sample, seed, sv, dhyp, g, dsave, k, stream, acc=None,
                          dz_ready=False):
        """backward with the parameter gradients deferred: their operands go to block k of
        ``dsave`` (blocks of ``dsave_per`` floats) for one ``wgrad`` call after the last iteration.
        ``acc`` [B, P, ns]: d AtAy is added into it (in the last linear's epilogue) and returned.
        ``dz_ready``: the head's logit gradient is already in block k (dhyp unused)."""
        if acc is None and self.dAtAy is None:
            self.dAtAy = torch.zeros((self.B, self.P, self.ns), device=self.dev)
        out = self.dAtAy if acc is None else acc
        assert out.is_contiguous() and out.shape == (self.B, self.P, self.ns)
        _lib.check("dadmm_hyper_train_backward_deferred", self.L.dadmm_hyper_train_backward_deferred(
            ctypes.byref(self.net), self.B, _ptr(AtAy), _ptr(Atb), _ptr(ahat), int(per_sample), seed,
            ctypes.byref(sv), _ptr(dhyp), ctypes.byref(g), _ptr(out), _ptr(self.work),
            ctypes.c_void_p(dsave.data_ptr() + 4 * k * self.dsave_per),
            (0 if acc is None else 1) | (2 if dz_ready else 0), stream))
        return out

    def wgrad(self, iters, As, Atb, arena, dsave, g, stream):
        """Add the parameter gradients of ``iters`` deferred iterations (As [iters, B, P, ns], the
        saved blocks of ``arena``, the operand blocks of ``dsave``) into ``g``'s accumulators."""
        assert As.is_contiguous() and As.shape[0] >= iters
        nbytes = self.L.dadmm_hyper_train_wgrad_scratch_bytes(ctypes.byref(self.net), self.B, iters)
        if nbytes and (self.wscratch is None or 4 * self.wscratch.numel() < nbytes):
            self.wscratch = torch.empty(nbytes // 4, device=self.dev)   # row-split partials, grown
        scr = self.wscratch if nbytes else None
        _lib.check("dadmm_hyper_train_wgrad", self.L.dadmm_hyper_train_wgrad(
            ctypes.byref(self.net), self.B, iters, _ptr(As), As[0].numel(), _ptr(Atb),
            ctypes.byref(self.saved(arena, 0)), self.per, _ptr(dsave), self.dsave_per, ctypes.byref(g),
            _ptr(scr), stream))


def _native_forward(ctx, L, AtAy, Atb, ahat, model, n, per_sample, seed, defer):
    B, P, ns = AtAy.shape
    dev = AtAy.device
    plan = NativeHyperPlan.get(model, B, P, n, ns, dev)
    arena = torch.empty(plan.per, device=dev)
    sv = plan.saved(arena)
    with torch.cuda.device(dev):
        # layer 1's Atb half as the whole-forward node forms it (there once per forward; here per
        # call), so that both paths give the same bits
        c1 = plan.atb_mix(Atb, ahat, per_sample, _stream(dev))
        plan.forward(AtAy, Atb, ahat, per_sample, seed, sv, _stream(dev), atb_mix=c1)
    if plan.train and defer:   # eval mode: the running statistics were inputs
        queue_running_stats(model, plan.stats(arena, 1), P, defer)
    elif plan.train:
        with torch.cuda.device(dev):
            plan.update_running_stats(arena, 1, _stream(dev))
    ctx.model, ctx.n, ctx.per_sample, ctx.seed = model, n, per_sample, seed
    ctx.arena, ctx.sv, ctx.plan = arena, sv, plan
    ctx.AtAy, ctx.Atb, ctx.ahat = AtAy, Atb, ahat
    return plan.hyp(arena)


def _native_backward(ctx, L, dhyp):
    AtAy = ctx.AtAy
    dev = AtAy.device
    acc = _GradAccumulator.current(ctx.model, dev)
    with torch.cuda.device(dev):
        d = ctx.plan.backward(AtAy, ctx.Atb, ctx.ahat, ctx.per_sample, ctx.seed, ctx.sv, dhyp.contiguous(),
                              acc.grads_struct(), _stream(dev))
    ctx.arena = ctx.sv = None
    return (d.clone(), None, None, None, None, None, None, None) + (None,) * ctx.n_params


def queue_running_stats(model, stats, P, defer):
    """The BatchNorm running-statistics updates of training-mode calls: applied now, or queued on
    ``model`` for flush_running_stats (stats: [(bn, mean [T, B, N] or [B, N], var)])."""
    if defer:
        if not hasattr(model, "_bn_pending"):
            model._bn_pending = []
        model._bn_pending.append((stats, P))
    else:
        with torch.no_grad():
            for bn, mean, var in stats:
                _update_running_stats(bn, mean, var, P)


class _GradAccumulator:
    """The hypernetwork's parameter gradients of ONE backward pass, in one flat float32 buffer laid
    out so that every group the kernels produce together is contiguous: per GCN layer
    [lin.weight | bn.weight | bn.bias | conv.bias] (dadmm_hyper_gcn_train_bwd's [3][B][N]
    partials reduce in one dadmm_hyper_colsum), LayerNorm [weight | bias], Linear [weight | bias].
    Created by the first HyperTrainFn.backward of a pass; the autograd engine's end-of-backward
    callback adds the sums to the parameters' .grad (set when None, accumulated otherwise) — in
    place of autograd's per-call, per-parameter accumulation kernels. Also caches the transposed
    weights of the input-gradient GEMMs (the weights do not change during a backward pass)."""

    def __init__(self, model, dev):
        self.model = model
        self.L = _lib.load()
        self.stream = _stream(dev)
        self.dev = dev
        enc = model.encoder
        order = []
        for conv, bn in zip((enc.conv1, enc.conv2, enc.conv3, enc.conv4, enc.conv5),
                            (enc.bn1, enc.bn2, enc.bn3, enc.bn4, enc.bn5)):
            order += [conv.lin.weight, bn.weight, bn.bias, conv.bias]   # [3][N] partials: contiguous
        order += [enc.norm.weight, enc.norm.bias]
        for blk in range(3):
            lin, ln = model.decoder[4 * blk], model.decoder[4 * blk + 2]
            order += [lin.weight, lin.bias, ln.weight, ln.bias]
        order += [model.fc.weight, model.fc.bias]
        self.off = {}
        o = 0
        for p in order:
            self.off[id(p)] = o
            o += (p.numel() + 3) & ~3              # 16-byte aligned (widths are multiples of 4)
        self.params = order
        self.flat = torch.zeros(o, device=dev)
        self.wt = {}
        self.scratch = torch.empty(0, device=dev)

    @staticmethod
    def current(model, dev):
        """The accumulator of the running backward pass (keyed by autograd's graph-task id, so a
        pass that ended in an exception never leaks its partial sums into the next one)."""
        task = torch._C._current_graph_task_id()
        acc = getattr(model, "_grad_acc", None)
        if acc is None or acc.task != task:
            acc = _GradAccumulator(model, dev)
            acc.task = task
            model._grad_acc = acc
            torch.autograd.Variable._execution_engine.queue_callback(acc.finalize)
        return acc

    def ptr(self, p):
        return self.flat.data_ptr() + 4 * self.off[id(p)]

    def view(self, p):
        o = self.off[id(p)]
        return self.flat[o:o + p.numel()].view_as(p)

    def wgrad(self, R, N, K, dz, ldz, x1, ld1, K1, x2, ld2, weight, bias):
        nb = self.L.dadmm_hyper_wgrad_scratch_bytes(R, N, K)
        if nb > 4 * self.scratch.numel():
            self.scratch = torch.empty(nb // 4 + 4, device=self.dev)
        gb = ctypes.c_void_p(self.ptr(bias)) if bias is not None else None
        _lib.check("dadmm_hyper_wgrad", self.L.dadmm_hyper_wgrad(
            R, N, K, _ptr(dz), ldz, _ptr(x1), ld1, K1, _ptr(x2), ld2, ctypes.c_void_p(self.ptr(weight)),
            gb, 1, _ptr(self.scratch), self.stream))

    def wgrad_cols(self, R, N, Kp, dz, ldz, x, ldx, weight, K):
        """dW (+)= (dZ^T X)[:, :K] for an input zero-padded to Kp > K columns (layer1_input):
        the padded product into a scratch tile, its first K columns added to weight's slot."""
        nb = self.L.dadmm_hyper_wgrad_scratch_bytes(R, N, Kp)
        if nb > 4 * self.scratch.numel():
            self.scratch = torch.empty(nb // 4 + 4, device=self.dev)
        tmp = torch.empty((N, Kp), device=self.dev)
        _lib.check("dadmm_hyper_wgrad", self.L.dadmm_hyper_wgrad(
            R, N, Kp, _ptr(dz), ldz, _ptr(x), ldx, Kp, None, 0, _ptr(tmp), None, 0,
            _ptr(self.scratch), self.stream))
        self.view(weight).add_(tmp[:, :K])

    def colsum(self, part, G, R, C, first):
        _lib.check("dadmm_hyper_colsum", self.L.dadmm_hyper_colsum(
            _ptr(part), G, R, C, ctypes.c_void_p(self.ptr(first)), 1, self.stream))

    def input_grad(self, R, dz, N, weight, cols=None, out=None, ldo=None):
        """dX [R][cols] = dZ [R][N] W [N][cols] (the first ``cols`` input columns)."""
        wt = self.transposed(weight)
        cols = wt.shape[0] if cols is None else cols
        if out is None:
            out = torch.empty((R, cols), device=self.dev)
            ldo = cols
        _lib.check("dadmm_hyper_linear", self.L.dadmm_hyper_linear(
            R, N, cols, _ptr(dz), N, N, None, 0, _ptr(wt), None, _ptr(out), ldo, self.stream))
        return out

    def transposed(self, weight):
        wt = self.wt.get(id(weight))
        if wt is None:
            Nw, Kw = weight.shape
            wt = torch.empty((Kw, Nw), device=self.dev)
            _lib.check("dadmm_hyper_transpose", self.L.dadmm_hyper_transpose(
                Nw, Kw, _ptr(weight), _ptr(wt), self.stream))
            self.wt[id(weight)] = wt
        return wt

    def grads_struct(self):
        """dadmm_hyper_grads: this pass's accumulators and the transposed weights (built once)."""
        g = getattr(self, "_gstruct", None)
        if g is not None:
            return g
        model = self.model
        enc = model.encoder
        g = _lib.HyperGrads()
        for i, (conv, bn) in enumerate(zip((enc.conv1, enc.conv2, enc.conv3, enc.conv4, enc.conv5),
                                           (enc.bn1, enc.bn2, enc.bn3, enc.bn4, enc.bn5))):
            g.conv_w[i] = self.ptr(conv.lin.weight)
            g.bn_wbc[i] = self.ptr(bn.weight)
            g.conv_wt[i] = self.transposed(conv.lin.weight).data_ptr()
        g.norm_wb = self.ptr(enc.norm.weight)
        for j in range(3):
            lin, ln = model.decoder[4 * j], model.decoder[4 * j + 2]
            g.dec_w[j], g.dec_b[j], g.ln_wb[j] = self.ptr(lin.weight), self.ptr(lin.bias), self.ptr(ln.weight)
            g.dec_wt[j] = self.transposed(lin.weight).data_ptr()
        g.fc_w, g.fc_b = self.ptr(model.fc.weight), self.ptr(model.fc.bias)
        g.fc_wt = self.transposed(model.fc.weight).data_ptr()
        self._gstruct = g
        return g

    def finalize(self):
        if getattr(self.model, "_grad_acc", None) is self:
            self.model._grad_acc = None
        with torch.no_grad():
            for p in self.params:
                if not p.requires_grad:
                    continue
                g = self.view(p)
                if p.grad is None:
                    p.grad = g
                else:
                    p.grad.add_(g)


def param_list(model):
    """_hyper_params(model), cached per model structure (the Parameter objects outlive .to() /
    optimiser steps, which replace or update their storage in place; a replaced Parameter or
    submodule rebuilds the list)."""
    ent = _cache(model)
    params = ent.get("params")
    if params is None:
        params = ent["params"] = _hyper_params(model)
    return params


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
    return HyperTrainFn.apply(AtAy, Atb, ahat, model, n, per_sample, seed, defer, *param_list(model))
