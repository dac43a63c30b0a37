#!/usr/bin/env python3
"""Training driver for DLASSO_unfolded on the HIP path — the counterpart of the reference's
unfolded_train_new.py:18-184, with batch-axis data parallelism.

    python train_unfolded.py --device cuda:0 --P 5 --m 64 --n 256 --GHN_iter_num 25 \
        --batch_size 4096 --train_size 16384 --test_size 4096 --num_epochs 10 --lr 2e-3
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
        train_unfolded.py ...          # one process per GPU, each batch split over the ranks

Same loop as the reference: set_A -> set_Data (train / valid) -> DLASSO_unfolded -> Adam ->
ReduceLROnPlateau(factor 0.8, patience 3, min_lr 1e-6) -> per batch: one ER graph replicated
over the batch, forward, compute_loss, loss_final.backward(), step -> validation under no_grad
-> early stopping (patience 70) -> losses.csv, model.pt (state_dict {'seq_hyp.param'}), A.pt,
args.json. Differences, all deliberate: everything is seeded (--seed; the reference seeds
nothing), the best state is actually restored (the reference's aliasing makes its
restore a no-op, unfolded_train_new.py:134), args are saved as JSON instead of a pickle, and no
plots are drawn.

With WORLD_SIZE > 1 every rank builds the same A, datasets, shuffle order and graph from the
seed, runs the forward and adjoint on its contiguous slice of each batch, and the only
collectives are dadmm_hip.dist's loss and gradient all_reduces.
"""
from __future__ import annotations

import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)

import networkx as nx  # noqa: E402
import torch  # noqa: E402
from torch.optim.lr_scheduler import ReduceLROnPlateau  # noqa: E402

import configurations  # noqa: E402
import gnn_dlasso_utils  # noqa: E402
import unfolded_DLASSO  # noqa: E402
from dadmm_hip import dist as D  # noqa: E402
from dadmm_hip.autograd import timed_out  # noqa: E402


def _dataset(A, size, args, gen):
    """(b [N,P,m,1], x* [N,n,1]) with gnn_data.set_Data's distribution, from ``gen``."""
    _, P, m, n = A.shape
    x = 2 * torch.randn(size, n, 1, generator=gen)
    x = x * (torch.rand(size, n, 1, generator=gen) <= 0.25)
    b = torch.einsum("pmn,snc->spmc", A[0].cpu(), x)
    return b, x


def _batches(N, bs, gen, shuffle):
    order = torch.randperm(N, generator=gen) if shuffle else torch.arange(N)
    for i in range(N // bs):                      # drop_last=True (gnn_data.py:15)
        yield order[i * bs:(i + 1) * bs]


def _inits(args, bs, lo, hi, device):
    """None (the module draws its shard's inits) or this rank's slice of the whole batch's."""
    if args.init_draw == "local":
        return None
    shape = (bs, args.P, args.n, 1)
    return tuple(torch.empty(shape, device=device).normal_(0.0, 1e-2)[lo:hi] for _ in range(3))


def validate(model, b_va, x_va, graph, args, bs, gen, rank, world, device):
    """The epoch's validation loss (global over ranks) and the last batch's hyp. A timed-out
    guard recomputation (NaN losses, compute_loss) raises GuardTimeoutError here instead of
    reaching the scheduler and the checkpoint test as NaN (the float() syncs anyway); the flag
    goes through the loss all_reduce, so all ranks raise together."""
    model.eval()
    hyp = None
    with torch.no_grad():
        tot, nb = 0.0, 0
        for idx in _batches(args.test_size, bs, gen, shuffle=True):
            lo, hi = D.shard_range(bs, rank, world)
            sel = idx[lo:hi].to(device)
            Y, hyp = model(b_va[sel], [graph] * (hi - lo), inits=_inits(args, bs, lo, hi, device))
            loss_mean, loss_final = gnn_dlasso_utils.compute_loss(Y, x_va[sel])
            # the timeout flag rides in the loss all_reduce: every rank raises together
            tot += float(D.global_losses(loss_mean, loss_final, hi - lo,
                                         timed_out=timed_out(loss_final))[1])
            nb += 1
    return tot / max(nb, 1), hyp


def main(argv=None):
    ap = configurations.build_parser()
    ap.add_argument("--out", default=None, help="output directory (default: save_dir/<time>)")
    ap.add_argument("--patience", type=int, default=70)
    ap.add_argument("--init-draw", choices=["local", "global"], default="local",
                    help="random inits y0/U0/delta0 (unfolded_DLASSO.py:49-51): 'local' = each "
                         "rank draws its shard's (independent streams per rank); 'global' = every "
                         "rank draws the whole batch's and keeps its slice (bit-identical "
                         "per-sample forwards for any world size; costs B/shard x the draws)")
    args = ap.parse_args(argv)
    rank, world, local = D.init_from_env()
    if torch.cuda.is_available() and args.device.startswith("cuda"):
        # one process per GPU; ranks beyond the visible devices share them (gloo rehearsals)
        dev_idx = local % torch.cuda.device_count() if world > 1 else int(args.device.split(":")[1])
        device = torch.device("cuda", dev_idx)
        torch.cuda.set_device(device)
    elif args.device == "cpu":
        # the reference's default device: DLASSO_unfolded runs its CPU path (dadmm_cpu)
        device = torch.device("cpu")
    else:
        raise SystemExit(f"--device {args.device}: use cuda:N (a ROCm GPU) or cpu")
    seed = int(args.seed)
    torch.manual_seed(seed)
    gen = torch.Generator().manual_seed(seed)

    A = gnn_dlasso_utils.set_A(args).to(device)
    if args.init_draw == "local":
        if device.type == "cuda":
            torch.cuda.manual_seed(seed * 1009 + rank)   # independent init noise per shard
    b_tr, x_tr = _dataset(A, args.train_size, args, gen)
    b_va, x_va = _dataset(A, args.test_size, args, gen)
    b_tr, x_tr, b_va, x_va = (t.to(device) for t in (b_tr, x_tr, b_va, x_va))
    graph = nx.erdos_renyi_graph(args.P, args.graph_prob, seed=seed)

    model = unfolded_DLASSO.DLASSO_unfolded(A=A, args=args).to(device)
    optimizer = torch.optim.Adam(model.parameters(), lr=args.lr, amsgrad=False)
    scheduler = ReduceLROnPlateau(optimizer, mode="min", factor=0.8, patience=3, min_lr=1e-6)

    bs = args.batch_size
    train_losses, valid_losses = [], []
    best, best_state, bad = float("inf"), None, 0
    t0 = time.time()
    for epoch in range(args.num_epochs):
        model.train()
        tot, nb = 0.0, 0
        for idx in _batches(args.train_size, bs, gen, shuffle=True):
            lo, hi = D.shard_range(bs, rank, world)
            sel = idx[lo:hi].to(device)
            b, label = b_tr[sel], x_tr[sel]
            Y, hyp = model(b, [graph] * (hi - lo), inits=_inits(args, bs, lo, hi, device))
            loss_mean, loss_final = gnn_dlasso_utils.compute_loss(Y, label)
            optimizer.zero_grad()
            loss_final.backward()
            D.allreduce_gradients(model.parameters(), hi - lo, bs)
            optimizer.step()
            tot += float(D.global_losses(loss_mean, loss_final, hi - lo)[1])
            nb += 1
        train_losses.append(tot / max(nb, 1))

        valid, hyp = validate(model, b_va, x_va, graph, args, bs, gen, rank, world, device)
        valid_losses.append(valid)
        scheduler.step(valid)
        if rank == 0:
            h = hyp[0, :, 0].tolist()
            print(f"epoch {epoch + 1}/{args.num_epochs} train {train_losses[-1]:.5f} "
                  f"valid {valid:.5f} alpha {h[0]:.5f} tau {h[1]:.5f} rho {h[2]:.5f} "
                  f"eta {h[3]:.5f} ({time.time() - t0:.1f} s)", flush=True)
        if valid < best:
            best, bad = valid, 0
            best_state = {k: v.detach().clone() for k, v in model.state_dict().items()}
        else:
            bad += 1
            if bad >= args.patience:
                break
    if best_state is not None:
        model.load_state_dict(best_state)

    if rank == 0:
        out = args.out or os.path.join(args.save_dir, time.strftime("%Y%m%d_%H%M%S") + "_unfolded_hip")
        os.makedirs(out, exist_ok=True)
        with open(os.path.join(out, "losses.csv"), "w") as f:
            f.write("epoch,train_loss,valid_loss\n")
            for i, (a, v) in enumerate(zip(train_losses, valid_losses)):
                f.write(f"{i + 1},{a},{v}\n")
        with open(os.path.join(out, "args.json"), "w") as f:
            json.dump(vars(args), f, indent=1)
        torch.save(A.cpu(), os.path.join(out, "A.pt"))
        torch.save(model.state_dict(), os.path.join(out, "model.pt"))
        print(f"saved to {out}")
    if world > 1:
        torch.distributed.destroy_process_group()
    return train_losses, valid_losses


if __name__ == "__main__":
    main()
