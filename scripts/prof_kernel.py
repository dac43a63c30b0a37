#!/usr/bin/env python3
"""Launch the product fused kernel a few times at the headline shape (for rocprofv3 passes)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hyperparameter-gnn_unfolded-d-admm-main_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from dadmm_hip import PreparedOperator, forward_raw, ingest  # noqa: E402
import oracle as O  # noqa: E402  (input generator only)


def main():
    B, P, m, n, K = (int(x) for x in (sys.argv[1:6] if len(sys.argv) > 5 else (4096, 5, 64, 256, 25)))
    reps = int(os.environ.get("REPS", "3"))
    dev = torch.device("cuda:0")
    A, b, _ = O.make_problem(P, m, n, B, seed=1234)
    op = PreparedOperator(torch.from_numpy(A).to(dev))
    g = ingest([O.er_graph(P, 0.5, seed=7)] * B, P, B, dev)
    bt = torch.from_numpy(b).to(dev)
    y0, U0, d0 = (torch.randn(B, P, n, device=dev) * 1e-2 for _ in range(3))
    hyp = torch.full((K, P, 4), 0.05, device=dev)
    for _ in range(reps):
        forward_raw(op, bt, g, hyp, y0, U0, d0)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
