#!/usr/bin/env python3
"""GNN-hypernetwork model forward (eval, no_grad) for kernel-trace profiling:
    python scripts/prof_gnn.py [B P n m K reps]      (default: 1024 5 256 64 25 3)"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hyperparameter-gnn_unfolded-d-admm-main_amd")]
import torch  # noqa: E402

import oracle as O  # noqa: E402


def main():
    B, P, n, m, K, reps = (int(x) for x in (sys.argv[1:7] if len(sys.argv) > 6
                                            else (1024, 5, 256, 64, 25, 3)))
    backend = os.environ.get("HYPER_BACKEND", "auto")
    import gnn_dlasso_models_progressive as GM
    dev = torch.device("cuda:0")
    A, b, _ = O.make_problem(P, m, n, B, seed=55)
    args = argparse.Namespace(GHN_iter_num=K, GHyp_hidden=100, DADMM_mode="diff", alpha_max=0.1,
                              tau_max=0.99, rho_max=0.99, eta_max=0.99)
    g = GM.DLASSO_GNNHyp3_Progressive(torch.from_numpy(A)[None].to(dev), args).to(dev).eval()
    g.hyper_backend = backend
    graphs = [O.connected_er_graph(P, 0.5, seed=500 + s) for s in range(B)]
    if os.environ.get("PREINGEST", "1") != "0":   # time the GPU forward, not networkx ingestion
        from dadmm_hip.graph import ingest
        graphs = ingest(graphs, P, B, dev)
    bt = torch.from_numpy(b)[..., None].to(dev)
    with torch.no_grad():
        g(bt, graphs)
        torch.cuda.synchronize()
        first = int(g.last_status.item())
        t0 = time.perf_counter()
        for _ in range(reps):
            g(bt, graphs)
        torch.cuda.synchronize()
    print(f"B={B} P={P} n={n} m={m} K={K} backend={backend}: "
          f"{1e3 * (time.perf_counter() - t0) / reps:.2f} ms per forward, "
          f"guard status {first} / {int(g.last_status.item())}")


if __name__ == "__main__":
    main()
