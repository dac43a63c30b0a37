"""Timing probe: the column-split forward (dadmm_forward_split) against the fused forward at a
small batch, HIP events over back-to-back forward_raw calls (draws + launch + gated stepwise).

    python scripts/time_split.py [B] [reps]      (P=5, n=256, m=64, K=25, shared ER graph)
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [ROOT, os.path.join(ROOT, "hyperparameter-gnn_unfolded-d-admm-main_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle as O  # noqa: E402
from dadmm_hip import PreparedOperator, forward_raw, ingest  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    P, m, n, K = 5, 64, 256, 25
    dev = torch.device("cuda", 0)
    A, b, _ = O.make_problem(P, m, n, B, seed=1)
    G = O.er_graph(P, 0.5, seed=7)
    hyp = torch.from_numpy(O.hyp_table(np.load(os.path.join(
        ROOT, "tests", "golden", "fixture_25_iter_general_learning_seq_hyp_param.npy")),
        [0.1, 0.99, 0.99, 0.99])).to(dev)
    op = PreparedOperator(torch.from_numpy(A).to(dev))
    g = ingest([G] * B, P, B, dev)
    bt = torch.from_numpy(b).to(dev)
    for path in ("split", "fused", "split", "fused"):
        f = lambda: forward_raw(op, bt, g, hyp, path=path if path == "fused" else "auto")  # noqa
        for _ in range(10):
            f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            Y, _, st = f()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        print(f"{path:6s} B={B}: {ms * 1e3:8.1f} us per forward, {B * K / (ms * 1e-3) / 1e6:7.1f} "
              f"M ADMM-iters/s, status {int(st.item())}", flush=True)


if __name__ == "__main__":
    main()
