"""Drop-in ``unfolded_DLASSO`` module: ``DLASSO_unfolded`` and ``seq_hyperparam``.

Mirrors the reference's public interface (unfolded_DLASSO.py:9-168): constructor ``(A, args)``,
``forward(b, graph_list, K=None) -> (Y [K',B,P,n,1], hyp [H,4,1])`` with ``K' = min(K, self.K)``,
state_dict ``{'seq_hyp.param': [K, P|1, 4]}``, and ``seq_hyp(k)``. On CUDA tensors the K-step
recurrence runs in one fused HIP launch (``dadmm_hip``, C ABI ``include/dadmm.h``); CPU tensors
(the reference's default device) run its op sequence in torch eager ops (``dadmm_cpu``).
"""
from __future__ import annotations

import torch
import torch.nn as nn

import dadmm_cpu
from dadmm_hip import _lib
from dadmm_hip.autograd import check_status, dadmm_unfolded_apply, tag_status
from dadmm_hip.ops import describe_status
from dadmm_hip.graph import ingest, n_graphs
from dadmm_hip.ops import PreparedOperator


class DLASSO_unfolded(nn.Module):
    """Unfolded D-ADMM for distributed LASSO (reference: unfolded_DLASSO.py:9-146)."""

    def __init__(self, A, args):
        super().__init__()
        # A [1, P, m, n] — a plain attribute, as in the reference (:13): not a buffer
        self.A = A
        _, self.P, self.m, self.n = self.A.shape
        self.K = args.GHN_iter_num
        self.DADMM_mode = args.DADMM_mode
        if args.DADMM_mode == 'same':
            hyp_shape = [self.K, 1, 4]
        else:
            hyp_shape = [self.K, self.P, 4]
        max_param = torch.tensor([args.alpha_max, args.tau_max, args.rho_max, args.eta_max],
                                 device=A.device)
        self.seq_hyp = seq_hyperparam(hyp_shape, max_param, args)
        self.max_param = max_param.unsqueeze(0)
        self.args = args
        self._op = None
        self._op_key = None
        # device int32 [1]: DADMM_STATUS_* bits of the guards the last forward applied
        # (include/dadmm.h); read it with guard_warnings() (synchronises)
        self.last_status = None
        self._table = None
        self._table_key = None

    # The reference precomputes AtA eagerly (:16). The HIP path never forms it; it is kept as a
    # lazily computed attribute for callers that read it.
    @property
    def AtA(self):
        A = self.A
        return torch.matmul(A.transpose(-1, -2), A)

    def operator(self) -> PreparedOperator:
        """The prepared operator for the current ``self.A`` (re-prepared if A changed)."""
        A = self.A
        key = (A.data_ptr(), A.device, tuple(A.shape), A._version)
        if self._op is None or self._op_key != key:
            self._op = PreparedOperator(A)
            self._op_key = key
        return self._op

    def hyp_table(self, K: int) -> torch.Tensor:
        """[K, H, 4] rows seq_hyp(0..K-1), differentiable w.r.t. seq_hyp.param. Outside autograd
        the table is memoised on (param version, K, train/eval mode)."""
        param = self.seq_hyp.param
        if torch.is_grad_enabled() and param.requires_grad:
            return self.seq_hyp.table(K)
        key = (param.data_ptr(), param._version, param.device, K, self.seq_hyp.training)
        if self._table_key != key:
            with torch.no_grad():
                self._table = self.seq_hyp.table(K)
            self._table_key = key
        return self._table

    def forward(self, b, graph_list, K=None, *, inits=None):
        """b [B,P,m,1]; graph_list: B networkx graphs on agents 0..P-1 (may repeat one object),
        or a ``dadmm_hip.graph.GraphBatch`` from an earlier ``ingest`` of them.

        ``inits`` (keyword-only, optional): (y0, U0, d0) each [B,P,n,1] or [B,P,n]; by default
        they are drawn like the reference (:49-51): randn * 1e-2 on b.device, in that order.
        """
        batch_size = max(len(b), n_graphs(graph_list, len(b)))
        device = b.device
        if K is None:
            K = self.K
        else:
            K = min(K, self.K)
        if K <= 0:
            # the reference's loop would not run and `hyp` would be unbound (NameError)
            raise RuntimeError(f"forward needs at least one iteration, got K={K}")
        if b.dim() != 4 or b.shape[1] != self.P or b.shape[2] != self.m:
            raise RuntimeError(f"b must be [B,{self.P},{self.m},1], got {tuple(b.shape)}")
        bb = b[..., 0]
        if len(b) != batch_size:
            if len(b) != 1:
                raise RuntimeError(
                    f"The size of tensor a ({len(b)}) must match the size of tensor b "
                    f"({batch_size}) at non-singleton dimension 0")
            bb = bb.expand(batch_size, -1, -1)
        graphs = ingest(graph_list, self.P, batch_size, device)

        if device.type == "cpu":
            # CPU tensors (the reference's default device): its op sequence in torch eager ops
            # (dadmm_cpu); CUDA tensors never take this path
            if inits is None:
                y0, U0, d0 = (torch.randn((batch_size, self.P, self.n, 1), device=device) * 1e-2
                              for _ in range(3))                            # :49-51, in order
            else:
                y0, U0, d0 = inits
            table = self.seq_hyp.table(K)
            Y, st = dadmm_cpu.unfolded_forward(self.A, bb, graphs, table, K, (y0, U0, d0))
            self.last_status = torch.tensor([st], dtype=torch.int32)
            return tag_status(Y.unsqueeze(-1), self.last_status), table[K - 1].unsqueeze(-1)

        if inits is None:
            # drawn by the forward's prologue launch: == torch.randn((B,P,n,1)) * 1e-2 x 3 value
            # for value, same generator stream (tests/test_gpu_parity.py::
            # test_prologue_draws_match_torch)
            y0 = U0 = d0 = None
        else:
            y0, U0, d0 = (x.reshape(batch_size, self.P, self.n) for x in inits)

        table = self.hyp_table(K)                       # [K, H, 4]
        Y, self.last_status = dadmm_unfolded_apply(self.operator(), bb, graphs, table, y0, U0,
                                                   d0, _lib.VARIANT_UNFOLDED)
        hyp = table[K - 1].unsqueeze(-1)                # seq_hyp(K-1): [H, 4, 1]
        return tag_status(Y.unsqueeze(-1), self.last_status), hyp

    def guard_warnings(self):
        """The reference's NaN/Inf warnings (unfolded_DLASSO.py:56-104) for the last forward
        (synchronises with the device)."""
        if self.last_status is None:
            return []
        return describe_status(check_status(self.last_status))

    # kept for API parity with the reference (:111-146); not used by the HIP forward
    def compute_sum_neighbors(self, graph_list, device):
        g = ingest(graph_list, self.P, len(graph_list), device)
        deg = g.deg if not g.shared else g.deg.expand(len(graph_list), -1)
        return deg.reshape(len(graph_list), self.P, 1, 1).float()

    def compute_Atx(self, x):
        A = self.A.to(x.device)
        return torch.einsum('pmn,bpmc->bpnc', A[0], x)

    def compute_delta(self, graph_list, y1, y2=None, device=None):
        if y2 is None:
            y2 = y1
        delta = torch.zeros_like(y1, device=device)
        for b in range(len(graph_list)):
            graph = graph_list[b]
            for p in range(self.P):
                y_p = y1[b, p]
                for j in graph.neighbors(p):
                    diff = y_p - y2[b, j]
                    delta[b, p] += diff
                    delta[b, j] -= diff
        return delta

    def compute_loss(self, y_k, label):
        loss = 0.0
        for p in range(self.P):
            loss += torch.nn.functional.mse_loss(y_k[:, p], label)
        return loss / self.P


class seq_hyperparam(nn.Module):
    """Per-iteration (alpha, tau, rho, eta) table (reference: unfolded_DLASSO.py:148-168)."""

    def __init__(self, hyp_shape, max_param, args=None):
        super().__init__()
        self.param = nn.Parameter(torch.zeros(hyp_shape))
        self.max_param = max_param.unsqueeze(0)
        self.args = args

    def _finish(self, hyp):
        # hyp [..., H, 4]; training-mode penalty (:161-165), then clamp (:167)
        if self.training and self.args is not None:
            mean = hyp.sum(dim=(-2, -1)) / (hyp.shape[-2] * hyp.shape[-1])
            scale = torch.where(mean > self.args.max_penalty_threshold,
                                torch.as_tensor(self.args.penalty_reduction_factor,
                                                dtype=hyp.dtype, device=hyp.device),
                                torch.ones((), dtype=hyp.dtype, device=hyp.device))
            hyp = hyp * scale[..., None, None]
        return torch.clamp(hyp, min=1e-4, max=0.99)

    def forward(self, k):
        hyp = torch.sum(self.param[:k + 1], dim=0)
        hyp = torch.sigmoid(hyp) * self.max_param.to(hyp.device)
        return self._finish(hyp).unsqueeze(-1)

    def table(self, K):
        """All rows 0..K-1 at once: [K, H, 4] (cumulative sums instead of K prefix sums)."""
        hyp = torch.cumsum(self.param[:K], dim=0)
        hyp = torch.sigmoid(hyp) * self.max_param.to(hyp.device)
        return self._finish(hyp)
