"""GPU: the training driver (train_unfolded.py, counterpart of the reference's
unfolded_train_new.py) end to end on the HIP forward + adjoint, single process and batch-sharded
over 2 ranks (gloo on the one GPU of the test box; the driver uses RCCL on a multi-GPU node)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ARGS = ["--device", "cuda:0", "--P", "5", "--m", "32", "--n", "128", "--GHN_iter_num", "10",
        "--batch_size", "64", "--train_size", "256", "--test_size", "64", "--num_epochs", "3",
        "--lr", "2e-2", "--seed", "3"]


def test_driver_trains_and_saves(cuda, tmp_path):
    import train_unfolded
    tr, va = train_unfolded.main(ARGS + ["--out", str(tmp_path)])
    assert len(tr) == 3 and np.isfinite(tr).all() and np.isfinite(va).all()
    assert tr[-1] < tr[0], tr
    for f in ("losses.csv", "model.pt", "A.pt", "args.json"):
        assert os.path.exists(tmp_path / f), f
    sd = torch.load(tmp_path / "model.pt", weights_only=True)
    assert list(sd) == ["seq_hyp.param"] and tuple(sd["seq_hyp.param"].shape) == (10, 5, 4)


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), DADMM_DIST_BACKEND="gloo")
    import train_unfolded
    tr, va = train_unfolded.main(ARGS + ["--num_epochs", "2", "--init-draw", "global", "--out", out])
    if rank == 0:
        np.save(os.path.join(out, "tr.npy"), np.array(tr + va))


def test_two_rank_sharded_training_matches_single_process(cuda, tmp_path):
    import train_unfolded
    tr1, va1 = train_unfolded.main(ARGS + ["--num_epochs", "2", "--init-draw", "global",
                                           "--out", str(tmp_path / "one")])
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = str(tmp_path / "two")
    os.makedirs(out)
    mp.start_processes(_worker, args=(2, port, out), nprocs=2, join=True, start_method="spawn")
    got = np.load(os.path.join(out, "tr.npy"))
    # per-sample forwards are bit-identical under sharding; only the loss / gradient sums are
    # grouped differently (fp32 rounding), so the curves agree to rounding
    np.testing.assert_allclose(got, np.array(tr1 + va1), rtol=1e-4)
