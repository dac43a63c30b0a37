"""The GNN training driver (train_gnn.py), counterpart of gnn_dlasso_progressive.py.

CPU: the progressive-depth schedule and the learning-rate factor against values worked out by
hand from the reference's formulas (gnn_dlasso_progressive.py:79-118).
GPU: the driver trains end to end (device graphs and networkx graphs), single process and
batch-sharded over 2 ranks (gloo on the test box's one GPU; RCCL on a multi-GPU node)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import train_gnn


def test_progressive_schedule_known_answers():
    # E = 40, K = 15: progress = epoch / 30, iterations = round(1 + 14 progress^1.5)
    it = [train_gnn.iterations_for_epoch(e, 40, 15) for e in range(40)]
    assert it[0] == 1
    assert it[10] == round(1 + 14 * (10 / 30) ** 1.5) == 4
    assert it[20] == round(1 + 14 * (20 / 30) ** 1.5) == 9
    assert it[29] == round(1 + 14 * (29 / 30) ** 1.5) == 14
    assert all(v == 15 for v in it[30:])
    assert it == sorted(it)
    # lr factor: 1 below full depth; at depth, 0.8 - 0.5 * (epoch - 30 + 1) / 10, floor 0.3
    assert train_gnn.lr_factor(14, 29, 40, 15) == 1.0
    assert train_gnn.lr_factor(15, 30, 40, 15) == pytest.approx(0.75)
    assert train_gnn.lr_factor(15, 35, 40, 15) == pytest.approx(0.5)
    assert train_gnn.lr_factor(15, 39, 40, 15) == pytest.approx(0.3)
    # E = 1: full depth at once, int(0.75) = 0 -> 0.8 - 0.5 * 1 / 1
    assert train_gnn.lr_factor(3, 0, 1, 3) == pytest.approx(0.3)


def test_host_graphs_are_the_reference_patch():
    import networkx as nx
    gs = train_gnn._host_graphs(12, 0.3, range(30))
    assert all(nx.is_connected(g) for g in gs)


ARGS = ["--device", "cuda:0", "--P", "5", "--m", "16", "--n", "64", "--GHN_iter_num", "4",
        "--GHyp_hidden", "16", "--batch_size", "32", "--train_size", "128", "--test_size", "32",
        "--num_epochs", "4", "--lr", "3e-3", "--seed", "5"]


@pytest.mark.gpu
@pytest.mark.parametrize("graphs", ["device", "host"])
def test_driver_trains_and_saves(cuda, tmp_path, graphs):
    h = train_gnn.main(ARGS + ["--graphs", graphs, "--out", str(tmp_path)])
    assert h["iterations"] == [1, 2, 3, 4]          # E = 4, K = 4: round(1 + 3 (epoch / 3)^1.5)
    for k in ("train_final", "valid_final"):
        assert np.isfinite(h[k]).all(), h[k]
    for f in ("losses.csv", "best_model.pt", "final_model.pt", "A.pt", "args.json"):
        assert os.path.exists(tmp_path / f), f
    sd = torch.load(tmp_path / "final_model.pt", weights_only=True)["model_state_dict"]
    assert "fc.weight" in sd and any(k.startswith("encoder.conv1") for k in sd)


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), DADMM_DIST_BACKEND="gloo")
    h = train_gnn.main(ARGS + ["--num_epochs", "2", "--out", out])
    if rank == 0:
        np.save(os.path.join(out, "h.npy"), np.array(h["train_final"] + h["valid_final"]))


@pytest.mark.gpu
def test_two_rank_sharded_training_runs(cuda, tmp_path):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = str(tmp_path)
    mp.start_processes(_worker, args=(2, port, out), nprocs=2, join=True, start_method="spawn")
    got = np.load(os.path.join(out, "h.npy"))
    assert np.isfinite(got).all() and (got > 0).all()
