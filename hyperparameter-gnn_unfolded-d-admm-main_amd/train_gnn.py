#!/usr/bin/env python3
"""Training driver for DLASSO_GNNHyp3_Progressive on the HIP path — the counterpart of the
reference's gnn_dlasso_progressive.py:20-362, with batch-axis data parallelism.

    python train_gnn.py --device cuda:0 --P 5 --m 64 --n 256 --GHN_iter_num 15 \
        --batch_size 256 --train_size 2048 --test_size 256 --num_epochs 40 --lr 1e-4
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
        train_gnn.py ...               # one process per GPU, each batch split over the ranks

The reference's loop, piece by piece:
  * set_A -> set_Data (train / valid), DLASSO_GNNHyp3_Progressive (:22-36);
  * AdamW(lr, weight_decay 1e-5, betas (0.9, 0.999)), gradient-norm clip 100,
    ReduceLROnPlateau(factor 0.7, patience 15, min_lr 1e-6), early stopping patience 20 (:39-57);
  * progressive depth: iterations(epoch) = round(1 + (K - 1) * min(1, epoch / (0.75 E)) ** 1.5)
    (:79-85), and the learning rate scaled only at full depth by max(0.3, 0.8 - 0.5 *
    epochs_at_max / remaining) (:87-118) — ``iterations_for_epoch`` / ``lr_factor`` below;
  * per batch: a fresh connected ER graph per sample with edge probability max(graph_prob, 0.3)
    (:181-191), forward(b, graph_list, training_iterations), compute_loss, loss_final.backward(),
    clip, step (:207-214); validation under no_grad (:240-281); best / final checkpoints (:284-326).
Differences, all deliberate: everything is seeded (--seed; the reference seeds nothing); graphs
are generated on the device by default (--graphs device: dadmm_hip.generate_er, same model of
graph, no networkx; --graphs host: networkx exactly as the reference, then ingested); mixed
precision, tqdm and the plots are left out (the reference keeps AMP off, :65); checkpoints hold
state dicts and JSON args (no pickled namespace).

With WORLD_SIZE > 1 every rank builds the same A, datasets and shuffle order from the seed and
runs its contiguous slice of each batch (graphs are drawn per sample from (seed, epoch, batch,
sample), so a sample's graph does not depend on the world size). The only collectives are
dadmm_hip.dist's loss all_reduce and one flattened gradient all_reduce per step (~1.4 M floats at
h = 100), before the clip so every rank clips the same global gradient. BatchNorm running
statistics are updated from each rank's shard (SURVEY.md §8(e) caveat); rank 0's are saved.
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

import configurations  # noqa: E402
import gnn_dlasso_models_progressive  # noqa: E402
import gnn_dlasso_utils  # noqa: E402
from dadmm_hip import dist as D  # noqa: E402
from dadmm_hip.autograd import timed_out  # noqa: E402
from dadmm_hip.graph import generate_er, ingest  # noqa: E402

MIN_ITERATIONS = 1        # gnn_dlasso_progressive.py:73


def iterations_for_epoch(epoch: int, total_epochs: int, max_iterations: int) -> int:
    """Progressive depth (gnn_dlasso_progressive.py:79-85)."""
    progress = min(1.0, epoch / (total_epochs * 0.75))
    it = MIN_ITERATIONS + (max_iterations - MIN_ITERATIONS) * (progress ** 1.5)
    return max(MIN_ITERATIONS, min(max_iterations, round(it)))


def lr_factor(current_iterations: int, epoch: int, total_epochs: int, max_iterations: int) -> float:
    """Learning-rate factor (gnn_dlasso_progressive.py:87-118): 1 below full depth; at full
    depth max(0.3, 0.8 - 0.5 * epochs_at_max / remaining), 0.8 if no epochs remain."""
    if current_iterations < max_iterations:
        return 1.0
    max_iter_epoch = int(total_epochs * 0.75)
    epochs_at_max = epoch - max_iter_epoch + 1
    remaining = total_epochs - max_iter_epoch
    if remaining > 0:
        return max(0.3, 0.8 - (epochs_at_max / remaining) * 0.5)
    return 0.8


def _dataset(A, size, gen):
    """(b [N,P,m,1], x* [N,n,1]) with gnn_data.set_Data's distribution, from ``gen``."""
    _, P, m, n = A.shape
    x = 2 * torch.randn(size, n, 1, generator=gen)
    x = x * (torch.rand(size, n, 1, generator=gen) <= 0.25)
    b = torch.einsum("pmn,snc->spmc", A[0].cpu(), x)
    return b, x


def _host_graphs(P, prob, seeds):
    """The reference's per-sample graphs (:181-191) with networkx, seeded per sample."""
    out = []
    for sd in seeds:
        g = nx.erdos_renyi_graph(P, prob, seed=sd)
        if not nx.is_connected(g):
            comps = list(nx.connected_components(g))
            for i in range(len(comps) - 1):
                g.add_edge(list(comps[i])[0], list(comps[i + 1])[0])
        out.append(g)
    return out


def _graphs(args, batch_seed, lo, hi, device):
    """This rank's graphs for samples lo..hi-1 of one batch, drawn per sample."""
    prob = max(args.graph_prob, 0.3)
    if args.graphs == "host" or device.type == "cpu":   # (on the CPU: networkx, as the reference)
        return ingest(_host_graphs(args.P, prob, [batch_seed * 65536 + s for s in range(lo, hi)]),
                      args.P, hi - lo, device)
    # device: one generate_er call per shard; sample s of the batch uses hash stream
    # (batch_seed, s) whatever the shard boundaries (the generator indexes samples from 0, so
    # the shard is generated as the first hi samples and sliced)
    gb = generate_er(hi, args.P, prob, batch_seed, device)
    if lo == 0:
        return gb
    from dadmm_hip.graph import GraphBatch
    vptr = gb.vptr[lo * args.P:]
    base = int(vptr[0])
    return GraphBatch(gb.nbr[lo:], gb.deg[lo:], False,
                      gb.order[lo:] if gb.order is not None else None,
                      vptr - base, gb.vq[base:], gb.fused_ok, gb.symmetric)


def _batches(N, bs, gen):
    order = torch.randperm(N, generator=gen)
    for i in range(N // bs):                      # drop_last=True (gnn_data.py:15)
        yield order[i * bs:(i + 1) * bs]


def main(argv=None):
    ap = configurations.build_parser()
    ap.add_argument("--out", default=None, help="output directory (default: checkpoints/<time>)")
    ap.add_argument("--patience", type=int, default=20)
    ap.add_argument("--graphs", choices=["device", "host"], default="device",
                    help="per-sample graphs generated on the GPU (dadmm_hip.generate_er) or with "
                         "networkx as the reference does")
    args = ap.parse_args(argv)
    # the reference's parser reads --GHyp_hidden as float (configurations.py:118), which only
    # works at its int default: a value given on the command line would reach nn.Linear as 16.0
    args.GHyp_hidden = int(args.GHyp_hidden)
    if args.train_size < args.batch_size or args.test_size < args.batch_size:
        # drop_last batching (gnn_data.py:15) would leave an epoch without a single batch
        raise SystemExit(f"--train_size ({args.train_size}) and --test_size ({args.test_size}) must "
                         f"be at least --batch_size ({args.batch_size})")
    rank, world, local = D.init_from_env()
    if torch.cuda.is_available() and args.device.startswith("cuda"):
        dev_idx = local % torch.cuda.device_count() if world > 1 else int(args.device.split(":")[1])
        device = torch.device("cuda", dev_idx)
        torch.cuda.set_device(device)
    elif args.device == "cpu":
        # the reference's default device: DLASSO_GNNHyp3_Progressive runs its CPU path (dadmm_cpu)
        device = torch.device("cpu")
    else:
        raise SystemExit(f"--device {args.device}: use cuda:N (a ROCm GPU) or cpu")
    seed = int(args.seed)
    torch.manual_seed(seed)
    gen = torch.Generator().manual_seed(seed)

    A = gnn_dlasso_utils.set_A(args)
    b_tr, x_tr = _dataset(A, args.train_size, gen)
    b_va, x_va = _dataset(A, args.test_size, gen)
    A = A.to(device)
    b_tr, x_tr, b_va, x_va = (t.to(device) for t in (b_tr, x_tr, b_va, x_va))
    torch.manual_seed(seed)            # model init identical on every rank
    model = gnn_dlasso_models_progressive.DLASSO_GNNHyp3_Progressive(A=A, args=args).to(device)
    D.seed_rank_streams(seed, rank)     # dropout seeds and random inits: a stream per rank
    optimizer = torch.optim.AdamW(model.parameters(), lr=args.lr, weight_decay=1e-5,
                                  betas=(0.9, 0.999))
    scheduler = torch.optim.lr_scheduler.ReduceLROnPlateau(optimizer, mode="min", factor=0.7,
                                                           patience=15, min_lr=1e-6)
    max_grad_norm = 100.0
    E, Kmax, bs = args.num_epochs, args.GHN_iter_num, args.batch_size
    hist = {"train_mean": [], "train_final": [], "valid_mean": [], "valid_final": [],
            "iterations": []}
    best, best_state, bad = float("inf"), None, 0
    out = args.out or os.path.join("checkpoints", time.strftime("progressive_hip_%Y%m%d_%H%M%S"))
    t0 = time.time()
    batch_id = 0
    hyp = None
    for epoch in range(E):
        K = iterations_for_epoch(epoch, E, Kmax)
        f = lr_factor(K, epoch, E, Kmax)
        for g in optimizer.param_groups:
            g["lr"] = args.lr * f
        model.train()
        tm = tf = 0.0
        nb = 0
        for idx in _batches(args.train_size, bs, gen):
            lo, hi = D.shard_range(bs, rank, world)
            sel = idx[lo:hi].to(device)
            graphs = _graphs(args, seed * 1_000_003 + batch_id, lo, hi, device)
            batch_id += 1
            Y, hyp = model(b_tr[sel], graphs, training_iterations=K)
            loss_mean, loss_final = gnn_dlasso_utils.compute_loss(Y, x_tr[sel])
            optimizer.zero_grad()
            loss_final.backward()
            D.allreduce_gradients(model.parameters(), hi - lo, bs)
            torch.nn.utils.clip_grad_norm_(model.parameters(), max_grad_norm)
            optimizer.step()
            gm, gf = D.global_losses(loss_mean, loss_final, hi - lo)
            tm += float(gm)
            tf += float(gf)
            nb += 1
        hist["train_mean"].append(tm / max(nb, 1))
        hist["train_final"].append(tf / max(nb, 1))
        model.eval()
        with torch.no_grad():
            vm = vf = 0.0
            nb = 0
            for idx in _batches(args.test_size, bs, gen):
                lo, hi = D.shard_range(bs, rank, world)
                sel = idx[lo:hi].to(device)
                graphs = _graphs(args, seed * 1_000_003 + batch_id, lo, hi, device)
                batch_id += 1
                Y, _ = model(b_va[sel], graphs, training_iterations=K)
                loss_mean, loss_final = gnn_dlasso_utils.compute_loss(Y, x_va[sel])
                # a timed-out guard recomputation makes the losses NaN: stop here with the
                # error instead of feeding NaN to the scheduler and the checkpoint test (the
                # float() below synchronises anyway); the flag rides in the loss all_reduce, so
                # every rank raises together
                gm, gf = D.global_losses(loss_mean, loss_final, hi - lo,
                                         timed_out=timed_out(loss_final))
                vm += float(gm)
                vf += float(gf)
                nb += 1
        valid = vf / max(nb, 1)
        hist["valid_mean"].append(vm / max(nb, 1))
        hist["valid_final"].append(valid)
        hist["iterations"].append(K)
        scheduler.step(valid)
        if rank == 0:
            a0 = hyp[0][0, 0].item() if hyp is not None else float("nan")   # last training batch
            print(f"epoch {epoch + 1}/{E} iterations {K} lr x{f:.3f} train {hist['train_final'][-1]:.5f} "
                  f"valid {valid:.5f} alpha[0,0] {a0:.5f} ({time.time() - t0:.1f} s)", flush=True)
        if valid < best:
            best, bad = valid, 0
            best_state = {k: v.detach().clone() for k, v in model.state_dict().items()}
            if rank == 0:
                os.makedirs(out, exist_ok=True)
                torch.save({"epoch": epoch, "model_state_dict": best_state, "valid_loss": valid,
                            "current_iterations": K}, os.path.join(out, "best_model.pt"))
        else:
            bad += 1
            if bad >= args.patience:
                if rank == 0:
                    print(f"early stopping at epoch {epoch + 1}", flush=True)
                break

    if rank == 0:
        os.makedirs(out, exist_ok=True)
        with open(os.path.join(out, "losses.csv"), "w") as fh:
            fh.write("epoch,iterations,train_mean,train_final,valid_mean,valid_final\n")
            for i in range(len(hist["valid_final"])):
                fh.write(f"{i + 1},{hist['iterations'][i]},{hist['train_mean'][i]},"
                         f"{hist['train_final'][i]},{hist['valid_mean'][i]},{hist['valid_final'][i]}\n")
        torch.save({"epoch": len(hist["valid_final"]) - 1, "model_state_dict": model.state_dict(),
                    "final_valid_loss": hist["valid_final"][-1]}, os.path.join(out, "final_model.pt"))
        torch.save(A.cpu(), os.path.join(out, "A.pt"))
        with open(os.path.join(out, "args.json"), "w") as fh:
            json.dump(vars(args), fh, indent=1)
        print(f"saved to {out}; best valid {best:.5f}", flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()
    return hist


if __name__ == "__main__":
    main()
