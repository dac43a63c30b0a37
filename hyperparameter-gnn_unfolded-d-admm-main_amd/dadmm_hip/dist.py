"""Batch-axis data parallelism for the unfolded D-ADMM path.

Samples are independent problems, so the batch shards over ranks with NO collective inside the
forward or the adjoint. One process per GPU (``torch.distributed``, backend ``nccl`` = RCCL over
xGMI on MI355X; ``gloo`` for the CPU tests). The only collectives are the ones the reference's
training loop implies once its batch is split:

* the loss of a batch (``compute_loss``, reference gnn_dlasso_utils.py:27-88) is a mean over
  samples, so the global value is the shard losses weighted by shard size: one ``all_reduce`` of
  [sum_r B_r loss_mean_r, sum_r B_r loss_final_r, sum_r B_r] (12 bytes, latency-bound);
* the gradient of that global loss w.r.t. the replicated parameters (``seq_hyp.param``, 2 KB at
  the headline shape) is sum_r (B_r / B) grad_r: one bucketed ``all_reduce`` of all parameter
  gradients, flattened into a single buffer (one collective per step, no per-tensor calls).

The reference's batch-global NaN/Inf guards (unfolded_DLASSO.py:55-61) become per shard.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def world():
    """(rank, world_size); (0, 1) when torch.distributed is not initialised."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def shard_range(B: int, rank: int, world_size: int):
    """Contiguous slice [lo, hi) of a B-sample batch for ``rank``; the first B % world ranks
    take one extra sample (every rank gets work when B >= world)."""
    if world_size < 1 or not (0 <= rank < world_size):
        raise ValueError(f"bad rank {rank} / world {world_size}")
    q, r = divmod(B, world_size)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def shard(t: torch.Tensor, rank: int = None, world_size: int = None):
    """This rank's contiguous slice of ``t`` along dim 0."""
    if rank is None:
        rank, world_size = world()
    lo, hi = shard_range(t.shape[0], rank, world_size)
    return t[lo:hi]


def global_losses(loss_mean: torch.Tensor, loss_final: torch.Tensor, n_local: int,
                  timed_out: bool = None):
    """(loss_mean, loss_final) of the whole batch from this rank's shard losses: shard-size
    weighted mean, one all_reduce of 3 values. Returns detached 0-dim tensors (host-side logging
    / scheduler use, like the reference's ``.item()`` sums, unfolded_train_new.py:82).

    ``timed_out`` (this rank's forward had a guard-recomputation timeout, autograd.timed_out):
    the flag rides in the same all_reduce, and EVERY rank raises GuardTimeoutError after the
    collective when any rank set it (a rank raising before the collective would leave the others
    blocked in it)."""
    vals = [loss_mean.detach().double() * n_local, loss_final.detach().double() * n_local,
            torch.tensor(float(n_local), dtype=torch.float64, device=loss_mean.device)]
    if timed_out is not None:
        vals.append(torch.tensor(1.0 if timed_out else 0.0, dtype=torch.float64,
                                 device=loss_mean.device))
    buf = torch.stack(vals)
    if world()[1] > 1:
        dist.all_reduce(buf)
    if timed_out is not None and float(buf[3]) > 0:
        from .autograd import GuardTimeoutError
        raise GuardTimeoutError(
            f"the guarded recomputation timed out on {int(float(buf[3]))} rank(s): "
            "stepwise grid barrier timed out, Y is invalid (device shared with other work)")
    return buf[0] / buf[2], buf[1] / buf[2]


def allreduce_gradients(params, n_local: int, n_global: int):
    """Replace each parameter's .grad (of the SHARD loss) by the gradient of the GLOBAL batch loss:
    sum_r (B_r / B) grad_r, in one flattened all_reduce. Parameters without a gradient contribute
    zeros (every rank must pass the same parameter list)."""
    params = [p for p in params if p.requires_grad]
    if not params:
        return
    dev = params[0].device
    flat = torch.cat([(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1)
                      for p in params]).to(dev)
    flat.mul_(n_local / n_global)
    if world()[1] > 1:
        dist.all_reduce(flat)
    off = 0
    for p in params:
        k = p.numel()
        g = flat[off:off + k].view_as(p)
        if p.grad is None:
            p.grad = g.clone()
        else:
            p.grad.copy_(g)
        off += k


def init_from_env(backend: str = None):
    """Initialise torch.distributed from torchrun's environment (RANK / WORLD_SIZE / LOCAL_RANK /
    MASTER_ADDR / MASTER_PORT). Backend: ``backend``, else $DADMM_DIST_BACKEND, else nccl (RCCL)
    with a GPU and gloo without. Returns (rank, world, local_rank); no-op for WORLD_SIZE <= 1."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if ws > 1 and not dist.is_initialized():
        if backend is None:
            backend = os.environ.get("DADMM_DIST_BACKEND") or (
                "nccl" if torch.cuda.is_available() else "gloo")
        kw = {}
        if backend == "nccl":
            kw["device_id"] = torch.device("cuda", local)
        dist.init_process_group(backend, **kw)
    return rank, ws, local


def seed_rank_streams(seed: int, rank: int) -> None:
    """Give every rank its own random streams after the replicated model init: torch's CPU
    generator (the HIP training hypernetwork draws its dropout seed from it,
    hyper_ops.draw_dropout_seed) and the device generators (the random inits y0, U0, delta0).
    Without it, local sample i of every rank would draw the same dropout masks."""
    torch.manual_seed(int(seed) * 1009 + int(rank))

