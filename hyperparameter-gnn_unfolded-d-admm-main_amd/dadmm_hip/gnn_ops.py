"""Per-iteration HIP path of the GNN-hypernetwork model (C ABI: the dadmm_gnn_* entry points of
include/dadmm.h) and its autograd plumbing.

Every D-ADMM operation — A^T A y, A^T b, the gradient assembly and clamps, the primal / consensus /
dual updates and the reference's batch-global guards — runs in libdadmm.so; so does the
hypernetwork between iterations (dadmm_hip.hyper_ops). GnnTrainFn runs a whole training-mode
forward (K iterations) as one autograd node.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from .graph import GraphBatch
from .ops import PreparedOperator, _dev_check, _pad_n, _ptr, _stream


class GnnRun:
    """Device state of one forward of DLASSO_GNNHyp3_Progressive: guard flags, Atb, the iterate
    table (y0, y_1 .. y_K) and its device pointer array."""

    def __init__(self, op: PreparedOperator, b: torch.Tensor, graphs: GraphBatch, K: int, H: int,
                 variant: int, y0, U0, d0, grad: bool, begin: bool = True):
        _dev_check(b, y0, U0, d0, graphs.deg)
        B, P, m = b.shape
        ns = op.n_store
        dev = b.device
        self.op, self.graphs, self.K, self.H, self.variant, self.grad = op, graphs, K, H, variant, grad
        self.B, self.P, self.dev = B, P, dev
        self.d = op.dims(B=B, K=K, variant=variant, hyp_rows=H, graph_shared=graphs.shared)
        self.L = _lib.load()
        self.y0 = _pad_n(y0.float(), ns).contiguous()
        self.U0 = _pad_n(U0.float(), ns).contiguous()
        self.d0 = _pad_n(d0.float(), ns).contiguous()
        self.b = b.contiguous().float()
        if grad:
            self.ys = [self.y0] + [torch.empty((B, P, ns), device=dev) for _ in range(K)]
            self.Y = None
        else:
            self.Y = torch.empty((K, B, P, ns), device=dev)
            self.ys = [self.y0] + list(self.Y.unbind(0))
        # from pinned memory, asynchronously: a pageable copy would make the host wait for the
        # stream to drain (the previous train step's backward) before enqueueing this forward
        self.yptr = torch.tensor([t.data_ptr() for t in self.ys], dtype=torch.int64,
                                 pin_memory=True).to(dev, non_blocking=True)
        self.flags = torch.empty(max(self.L.dadmm_gnn_flag_bytes(K) // 4, 1), dtype=torch.int32,
                                 device=dev)
        self.Atb = torch.empty((B, P, ns), device=dev)
        self.G = torch.empty((B, P, ns), device=dev)
        self.status = torch.zeros(1, dtype=torch.int32, device=dev)
        if begin:
            self.begin()

    def begin(self):
        """Zero the guard flags, the k = 0 guards, Atb = A^T b (dadmm_gnn_begin); enqueued."""
        with torch.cuda.device(self.dev):
            _lib.check("dadmm_gnn_begin", self.L.dadmm_gnn_begin(
                ctypes.byref(self.d), _ptr(self.op.workspace), _ptr(self.b), _ptr(self.y0),
                _ptr(self.U0), _ptr(self.Atb), _ptr(self.flags), _stream(self.dev)))

    def gram(self, k: int, x: torch.Tensor = None, out: torch.Tensor = None) -> torch.Tensor:
        """A^T A y_k (guard-resolved y_k) or, with ``x``, A^T A x; into ``out`` if given."""
        if out is None:
            out = torch.empty((self.B, self.P, self.op.n_store), device=self.dev)
        if x is not None:
            x = _pad_n(x.float(), self.op.n_store).contiguous()
        with torch.cuda.device(self.dev):
            _lib.check("dadmm_gnn_gram", self.L.dadmm_gnn_gram(
                ctypes.byref(self.d), _ptr(self.op.workspace), k, _ptr(self.yptr), _ptr(self.flags),
                _ptr(x), _ptr(out), _stream(self.dev)))
        return out

    def gram_acc(self, x: torch.Tensor, out: torch.Tensor, addend: torch.Tensor = None) -> torch.Tensor:
        """out += A^T A x in one launch (== out.add_(self.gram(0, x=x)), bit for bit), then
        out += addend when given (the same bits as a separate add after)."""
        x = _pad_n(x.float(), self.op.n_store).contiguous()
        if addend is not None:
            addend = addend.contiguous()
            assert addend.shape == out.shape
        with torch.cuda.device(self.dev):
            _lib.check("dadmm_gnn_gram_acc", self.L.dadmm_gnn_gram_acc(
                ctypes.byref(self.d), _ptr(self.op.workspace), _ptr(x), _ptr(out), _ptr(addend),
                _stream(self.dev)))
        return out

    def step(self, k: int, AtAy, hyp_k, U, D):
        """One iteration; returns (y_{k+1}, U_{k+1}, delta_{k+1})."""
        g = self.graphs
        U_next = torch.empty_like(U)
        D_next = torch.empty_like(D)
        with torch.cuda.device(self.dev):
            _lib.check("dadmm_gnn_step", self.L.dadmm_gnn_step(
                ctypes.byref(self.d), k, _ptr(g.vptr), _ptr(g.vq), _ptr(g.deg), _ptr(hyp_k),
                _ptr(self.yptr), _ptr(AtAy), _ptr(self.Atb), _ptr(U), _ptr(D), _ptr(U_next),
                _ptr(D_next), _ptr(self.G), _ptr(self.flags), _stream(self.dev)))
        return self.ys[k + 1], U_next, D_next

    def finish(self) -> torch.Tensor:
        with torch.cuda.device(self.dev):
            _lib.check("dadmm_gnn_finish", self.L.dadmm_gnn_finish(
                ctypes.byref(self.d), _ptr(self.yptr), _ptr(self.flags), _ptr(self.status),
                _stream(self.dev)))
        return self.status

    def step_backward(self, k, y_k, AtAy, hyp_k, U, D, gy1, gU1, gd1, head=None):
        """The step's adjoint; ``head`` (a _lib.HeadBwd) runs the hyper-parameter head's backward
        in the same launch (dadmm_gnn_step_backward_ex)."""
        g = self.graphs
        mk = lambda t: None if t is None else t.contiguous()
        gy1, gU1, gd1 = mk(gy1), mk(gU1), mk(gd1)
        gy, gU, gd, gA = (torch.empty_like(U) for _ in range(4))
        ghyp = torch.empty((self.B, 4, self.H), device=self.dev)
        with torch.cuda.device(self.dev):
            _lib.check("dadmm_gnn_step_backward_ex", self.L.dadmm_gnn_step_backward_ex(
                ctypes.byref(self.d), k, _ptr(g.vptr), _ptr(g.vq), _ptr(g.deg), _ptr(hyp_k),
                _ptr(y_k), _ptr(AtAy), _ptr(self.Atb), _ptr(U), _ptr(D), _ptr(gy1), _ptr(gU1),
                _ptr(gd1), _ptr(gy), _ptr(gU), _ptr(gd), _ptr(gA), _ptr(ghyp),
                None if head is None else ctypes.byref(head), _stream(self.dev)))
        return gy, gU, gd, gA, ghyp


def _stage_status(run: GnnRun):
    """After the forward's finish: the status word copied to pinned host memory behind an event,
    so that the backward can read it without draining the stream (_check_guards). The copy and
    the event go on run.dev's current stream (the one the forward ran on), whichever device is
    current for the caller."""
    run.status_host = torch.empty(1, dtype=torch.int32, pin_memory=True)
    with torch.cuda.device(run.dev):
        run.status_host.copy_(run.status, non_blocking=True)
        run.status_event = torch.cuda.Event()
        run.status_event.record(torch.cuda.current_stream(run.dev))


def _check_guards(run: GnnRun):
    """Once per backward pass: the adjoint assumes no guard fired. With a staged status word
    (_stage_status) this waits only for the forward; else one host sync."""
    if getattr(run, "_checked", False):
        return
    # (any adjacency: the step adjoint applies compute_delta through the forward's visit lists,
    # and that map is symmetric for directed graphs too; oracle.laplacians)
    if getattr(run, "status_event", None) is not None:
        run.status_event.synchronize()
        st = int(run.status_host[0])
    else:
        st = int(run.status.item())
    run._checked = True
    if st:
        from .autograd import GuardAdjointError
        from .ops import describe_status
        raise GuardAdjointError(
            "backward through a forward in which the reference's NaN/Inf guards fired ("
            + "; ".join(describe_status(st)) + ") is not supported")


class GramFn(torch.autograd.Function):
    """AtAy_k = A^T A y_k (gnn_dlasso_models_progressive.py:158-162); backward: A^T A g."""

    @staticmethod
    def forward(ctx, y_k, run, k):
        ctx.run = run
        return run.gram(k)

    @staticmethod
    def backward(ctx, g):
        _check_guards(ctx.run)
        return ctx.run.gram(0, x=g), None, None


class StepFn(torch.autograd.Function):
    """(y_{k+1}, U_{k+1}, delta_{k+1}) = one D-ADMM iteration (:205-237)."""

    @staticmethod
    def forward(ctx, y_k, U, D, AtAy, hyp_k, run, k):
        y1, U1, D1 = run.step(k, AtAy, hyp_k, U, D)
        ctx.run, ctx.k = run, k
        ctx.save_for_backward(y_k, U, D, AtAy, hyp_k)
        return y1, U1, D1

    @staticmethod
    def backward(ctx, gy1, gU1, gd1):
        _check_guards(ctx.run)
        y_k, U, D, AtAy, hyp_k = ctx.saved_tensors
        gy, gU, gd, gA, ghyp = ctx.run.step_backward(ctx.k, y_k, AtAy, hyp_k, U, D, gy1, gU1, gd1)
        return gy, gU, gd, gA, ghyp, None, None


class GnnTrainFn(torch.autograd.Function):
    """The K iterations of a training-mode forward of DLASSO_GNNHyp3_Progressive
    (gnn_dlasso_models_progressive.py:227-243 with the hypernetwork of :165-196 in train mode) as
    ONE autograd node: per iteration A^T A y_k (dadmm_gnn_gram), the hypernetwork
    (dadmm_hyper_train_forward, one library call) and the D-ADMM step (dadmm_gnn_step); the
    backward walks the iterations in reverse with dadmm_gnn_step_backward,
    dadmm_hyper_train_backward_deferred (the parameter gradients' operands saved per iteration) and
    A^T A for the gram's input gradient, then ONE dadmm_hyper_train_wgrad call adds the parameter
    gradients of all K iterations into the pass's flat buffer (hyper_ops._GradAccumulator). Replaces K x (GramFn,
    HyperTrainFn, StepFn) nodes and the engine's per-iteration gradient sums — the training step
    is then bound by the GPU, not by the host.

    Inputs: the GnnRun (iterate table Y [K, B, P, ns] layout), the model, its
    hyper_ops.NativeHyperPlan, a_hat, per-sample flag, the K dropout seeds and the hypernetwork's
    parameters (hyper_ops.param_list order). Outputs: Y [K, B, P, ns] and hyp_{K-1} [B, 4, H]. The
    BatchNorm running statistics of the K iterations are updated in the forward, in call order.
    The backward RETURNS the parameter gradients (views of the pass's flat accumulator), so
    autograd delivers them: ``.grad`` accumulation, ``torch.autograd.grad`` and parameter hooks
    behave as with torch modules. A second backward through the same node (retain_graph=True)
    raises: the saved activations are released by the first."""

    @staticmethod
    def forward(ctx, run, model, plan, a_hat, per_sample, seeds, *params):
        from . import hyper_ops
        K, dev = run.K, run.dev
        stream = _stream(dev)
        arena = torch.empty(K * plan.per, device=dev)
        svs = [plan.saved(arena, k) for k in range(K)]
        U, D = run.U0, run.d0
        Us, Ds = [U], [D]
        # the K gram outputs in one [K, B, P, ns] block: the deferred weight gradient of the first
        # GCN layer reads them at a fixed stride
        As = torch.empty((K, run.B, run.P, run.op.n_store), device=dev)
        with torch.cuda.device(dev):
            c1 = plan.atb_mix(run.Atb, a_hat, per_sample, stream)
            for k in range(K):
                AtAy = run.gram(k, out=As[k])
                plan.forward(AtAy, run.Atb, a_hat, per_sample, seeds[k], svs[k], stream, atb_mix=c1)
                _, U, D = run.step(k, AtAy, plan.hyp(arena, k), U, D)
                Us.append(U)
                Ds.append(D)
        run.finish()
        _stage_status(run)
        if plan.train:   # eval mode (a backward through model.eval()): running statistics are inputs
            with torch.cuda.device(dev):
                plan.update_running_stats(arena, K, hyper_ops._stream(dev))
        ctx.run, ctx.model, ctx.plan, ctx.a_hat, ctx.per_sample, ctx.seeds = run, model, plan, a_hat, per_sample, seeds
        ctx.arena, ctx.svs, ctx.As, ctx.Us, ctx.Ds = arena, svs, As, Us, Ds
        ctx.params = params
        return run.Y, plan.hyp(arena, K - 1)

    @staticmethod
    def backward(ctx, gY, ghyp_last):
        from . import hyper_ops
        run, plan = ctx.run, ctx.plan
        if ctx.arena is None:
            raise RuntimeError("GnnTrainFn: a second backward through the same training forward "
                               "(retain_graph=True) is not supported; its saved activations were "
                               "released by the first backward")
        K, dev = run.K, run.dev
        stream = _stream(dev)
        # this node's own accumulator: its sums are returned to autograd below
        acc = hyper_ops._GradAccumulator(ctx.model, dev)
        g = acc.grads_struct()
        # parameter gradients deferred: each iteration's operands go to a block of dsave and one
        # dadmm_hyper_train_wgrad call sums all K iterations' (one launch per parameter, not K)
        dsave = torch.empty(K * plan.dsave_per, device=dev)
        gY = gY.contiguous() if gY is not None else None
        gy1 = gY[K - 1] if gY is not None else None
        gU1 = gd1 = None
        if ghyp_last is not None:
            ghyp_last = ghyp_last.contiguous()
        head = _lib.HeadBwd()
        head.maxv[:] = [float(v) for v in plan.net.maxv]
        with torch.cuda.device(dev):
            for k in range(K - 1, -1, -1):
                hyp_k = plan.hyp(ctx.arena, k)
                # in the step adjoint's epilogue: the head's backward (d logits into the
                # iteration's dsave block, ghyp_last added first)
                head.z = ctx.svs[k].z
                head.ghyp_add = ghyp_last.data_ptr() if (k == K - 1 and ghyp_last is not None) else None
                head.dz = dsave.data_ptr() + 4 * k * plan.dsave_per
                gy, gU, gd, gA, ghyp = run.step_backward(k, run.ys[k], ctx.As[k], hyp_k, ctx.Us[k], ctx.Ds[k],
                                                         gy1, gU1, gd1, head=head)
                # gA += d AtAy from the hypernetwork (in its last linear's epilogue); at k = 0 the
                # sum is not used (y_0, U_0, delta_0 are the random inits: no gradient)
                plan.backward_deferred(ctx.As[k], run.Atb, ctx.a_hat, ctx.per_sample, ctx.seeds[k],
                                       ctx.svs[k], None, g, dsave, k, stream, acc=gA, dz_ready=True)
                if k == 0:
                    break
                # gy += A^T A gA, then + the loss's own gradient on y_k (gY[k - 1]), one launch
                run.gram_acc(gA, gy, addend=gY[k - 1] if gY is not None else None)
                gy1, gU1, gd1 = gy, gU, gd
            plan.wgrad(K, ctx.As, run.Atb, ctx.arena, dsave, g, stream)
        ctx.arena = ctx.svs = ctx.As = ctx.Us = ctx.Ds = None
        # the guard check after the enqueue (the forward's status, staged behind an event, is
        # ready by now in the common case: no stall between the forward and this backward); if a
        # guard fired the gradients just computed are discarded with the error
        _check_guards(run)
        grads = tuple(acc.view(p) if p.requires_grad else None for p in ctx.params)
        ctx.params = None
        return (None,) * 6 + grads
