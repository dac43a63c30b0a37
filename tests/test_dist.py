"""CPU, multi-process (gloo): the batch-sharded path of SURVEY.md §8(e) — shard ranges, the
shard-size weighted loss all_reduce and the flattened gradient all_reduce — reproduce the
full-batch loss and the full-batch gradient of seq_hyp.param.

The forward inside each rank is the oracle's differentiable fp64 replay of the reference's ops
(oracle/ref_torch.forward_autograd) standing in for the HIP forward (no GPU here); what is under
test is the host-side data-parallel logic (dadmm_hip/dist.py) around it."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from dadmm_hip import dist as D

MAXP = [0.1, 0.99, 0.99, 0.99]


def test_shard_range_covers_batch():
    for B in (1, 7, 8, 4096, 4099):
        for W in (1, 2, 3, 8):
            if B < W:
                continue
            spans = [D.shard_range(B, r, W) for r in range(W)]
            assert spans[0][0] == 0 and spans[-1][1] == B
            assert all(spans[i][1] == spans[i + 1][0] for i in range(W - 1))
            sizes = [hi - lo for lo, hi in spans]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        D.shard_range(8, 2, 2)


def _problem(seed=0):
    import oracle as O
    P, m, n, B, K = 4, 12, 32, 7, 6
    A, b, x = O.make_problem(P, m, n, B, seed=seed)
    graphs = [O.connected_er_graph(P, 0.5, seed=30 + s) for s in range(B)]
    rng = np.random.default_rng(1)
    y0, U0, d0 = (1e-2 * rng.standard_normal((3, B, P, n))).astype(np.float32)
    param = (0.3 * rng.standard_normal((K, P, 4))).astype(np.float64)
    return A, b, x, graphs, y0, U0, d0, param


def _loss_and_grad(sl, A, b, x, graphs, y0, U0, d0, param):
    """compute_loss of the forward on samples `sl`, and d loss_final / d param."""
    import argparse

    import gnn_dlasso_utils
    import unfolded_DLASSO
    from oracle import ref_torch
    K, P = param.shape[:2]
    args = argparse.Namespace(max_penalty_threshold=0.8, penalty_reduction_factor=0.95)
    seq = unfolded_DLASSO.seq_hyperparam([K, P, 4], torch.tensor(MAXP, dtype=torch.float64), args)
    seq.param = torch.nn.Parameter(torch.tensor(param))
    seq.train()
    table = seq.table(K)
    Y, _, _, _ = ref_torch.forward_autograd(A, b[sl], [graphs[i] for i in range(*sl.indices(len(graphs)))],
                                            table, y0[sl], U0[sl], d0[sl])
    label = torch.as_tensor(x[sl], dtype=torch.float64)[..., None]
    loss_mean, loss_final = gnn_dlasso_utils.compute_loss(Y[..., None], label)
    loss_final.backward()
    return loss_mean.detach(), loss_final.detach(), seq.param


def _worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    r, w, _ = D.init_from_env("gloo")
    assert (r, w) == (rank, world)
    A, b, x, graphs, y0, U0, d0, param = _problem()
    lo, hi = D.shard_range(b.shape[0], r, w)
    lm, lf, p = _loss_and_grad(slice(lo, hi), A, b, x, graphs, y0, U0, d0, param)
    gm, gf = D.global_losses(lm, lf, hi - lo)
    D.allreduce_gradients([p], hi - lo, b.shape[0])
    if r == 0:
        np.savez(out_path, loss_mean=gm.numpy(), loss_final=gf.numpy(), grad=p.grad.numpy())
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_loss_and_gradient_equal_full_batch(tmp_path, world):
    out = str(tmp_path / "r0.npz")
    mp.start_processes(_worker, args=(world, _free_port(), out), nprocs=world, join=True,
                       start_method="spawn")
    got = np.load(out)
    A, b, x, graphs, y0, U0, d0, param = _problem()
    lm, lf, p = _loss_and_grad(slice(0, b.shape[0]), A, b, x, graphs, y0, U0, d0, param)
    # compute_loss adds 1e-8 to each shard's loss; the weighted mean keeps exactly one 1e-8
    np.testing.assert_allclose(got["loss_mean"], lm.numpy(), rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(got["loss_final"], lf.numpy(), rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(got["grad"], p.grad.numpy(), rtol=1e-9,
                               atol=1e-12 * np.abs(p.grad.numpy()).max())


def _seed_worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    r, w, _ = D.init_from_env("gloo")
    from dadmm_hip import hyper_ops
    # train_gnn.main: the model init is replicated (same seed everywhere), then every rank
    # re-seeds its own streams; the HIP training hypernetwork draws its dropout seeds from them
    torch.manual_seed(5)
    init = torch.randn(4)
    D.seed_rank_streams(5, r)
    seeds = torch.tensor([hyper_ops.draw_dropout_seed() for _ in range(3)], dtype=torch.int64)
    gi = [torch.empty_like(init) for _ in range(w)]
    gs = [torch.empty_like(seeds) for _ in range(w)]
    torch.distributed.all_gather(gi, init)
    torch.distributed.all_gather(gs, seeds)
    if r == 0:
        np.savez(out_path, init=torch.stack(gi).numpy(), seeds=torch.stack(gs).numpy())
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


def test_dropout_seeds_differ_between_ranks(tmp_path):
    """each rank's dropout masks must come from its own stream (hash(seed, site, local
    row, col) with a shared seed would give local sample i the same masks on every rank)."""
    out = str(tmp_path / "seeds.npz")
    mp.start_processes(_seed_worker, args=(2, _free_port(), out), nprocs=2, join=True,
                       start_method="spawn")
    got = np.load(out)
    assert np.array_equal(got["init"][0], got["init"][1])          # replicated model init
    s0, s1 = got["seeds"]
    assert not set(s0.tolist()) & set(s1.tolist())                 # disjoint dropout seeds


def test_single_process_is_identity():
    p = torch.nn.Parameter(torch.ones(3))
    p.grad = torch.full((3,), 2.0)
    D.allreduce_gradients([p], 5, 5)
    assert torch.equal(p.grad, torch.full((3,), 2.0))
    gm, gf = D.global_losses(torch.tensor(0.5), torch.tensor(0.25), 5)
    assert float(gm) == 0.5 and float(gf) == 0.25


def _timeout_worker(rank, world, port, out_path):
    """Rank 1's forward timed out, rank 0's did not: both must raise after the collective."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    r, w, _ = D.init_from_env("gloo")
    from dadmm_hip import _lib
    from dadmm_hip.autograd import GuardTimeoutError, tag_status, timed_out
    bits = _lib.STATUS_BARRIER_TIMEOUT if r == 1 else 0
    lf = tag_status(torch.tensor(0.5), torch.tensor([bits], dtype=torch.int32))
    raised = False
    try:
        D.global_losses(torch.tensor(0.5), lf, 3, timed_out=timed_out(lf))
    except GuardTimeoutError:
        raised = True
    # both ranks reach this second collective only if neither was left blocked in the first
    flags = [torch.zeros(1) for _ in range(w)]
    torch.distributed.all_gather(flags, torch.tensor([1.0 if raised else 0.0]))
    if r == 0:
        np.save(out_path, torch.cat(flags).numpy())
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


def test_timeout_flag_raises_on_every_rank(tmp_path):
    """a guard-recomputation timeout on ONE rank must not leave the others
    blocked in the loss all_reduce: the flag rides in that collective and every rank raises."""
    out = str(tmp_path / "to.npy")
    mp.start_processes(_timeout_worker, args=(2, _free_port(), out), nprocs=2, join=True,
                       start_method="spawn")
    assert np.load(out).tolist() == [1.0, 1.0]
