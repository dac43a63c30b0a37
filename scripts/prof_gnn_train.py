#!/usr/bin/env python3
"""GNN model train steps (model.train(): dropout, per-sample BatchNorm statistics, autograd) as in
bench.py's gnn_train_step extra, for rocprofv3 kernel traces:
python scripts/prof_gnn_train.py [B K steps [P m n]]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hyperparameter-gnn_unfolded-d-admm-main_amd")]
import torch  # noqa: E402

import gnn_dlasso_models_progressive as GM  # noqa: E402
import gnn_dlasso_utils  # noqa: E402
import oracle as O  # noqa: E402
from dadmm_hip.graph import ingest  # noqa: E402

B, K, steps = (int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (256, 25, 3)))
P, m, n = (int(v) for v in (sys.argv[4:7] if len(sys.argv) > 6 else (5, 64, 256)))
dev = torch.device("cuda:0")
A, b, x = O.make_problem(P, m, n, B, seed=1234)
args = argparse.Namespace(GHN_iter_num=K, GHyp_hidden=100, DADMM_mode="diff", alpha_max=0.1,
                          tau_max=0.99, rho_max=0.99, eta_max=0.99)
gnn = GM.DLASSO_GNNHyp3_Progressive(torch.from_numpy(A)[None].to(dev), args).to(dev).train()
graphs = ingest([O.connected_er_graph(P, 0.5, seed=100 + s) for s in range(B)], P, B, dev)
bt = torch.from_numpy(b)[..., None].to(dev)
lab = torch.from_numpy(x)[..., None].to(dev)


def step():
    Y, _ = gnn(bt, graphs)
    _, lf = gnn_dlasso_utils.compute_loss(Y, lab)
    gnn.zero_grad()
    lf.backward()


step()
torch.cuda.synchronize()
if os.environ.get("CPROF"):   # host-side profile of the timed steps
    import cProfile
    import pstats
    pr = cProfile.Profile()
    pr.enable()
t0 = time.perf_counter()
for _ in range(steps):
    step()
t_enq = time.perf_counter()   # the host's enqueue time (the GPU may still be running)
torch.cuda.synchronize()
if os.environ.get("CPROF"):
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(35)
print(f"B={B} K={K} P={P} m={m} n={n}: {1e3 * (time.perf_counter() - t0) / steps:.2f} ms per train step "
      f"(graphs pre-ingested, backend {gnn.last_backend}; host enqueue {1e3 * (t_enq - t0) / steps:.2f} ms)")
