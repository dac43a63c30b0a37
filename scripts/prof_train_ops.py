#!/usr/bin/env python3
"""Which torch ops launch device kernels in the GNN train step (bench.py's gnn_train_step extra):
torch.profiler over a few steps, the aten ops that ran a device kernel with their call counts and
the Python source line that issued them. python scripts/prof_train_ops.py [B K steps]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hyperparameter-gnn_unfolded-d-admm-main_amd")]
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

import gnn_dlasso_models_progressive as GM  # noqa: E402
import gnn_dlasso_utils  # noqa: E402
import oracle as O  # noqa: E402
from dadmm_hip.graph import ingest  # noqa: E402

B, K, steps = (int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (256, 25, 2)))
P, m, n = 5, 64, 256
dev = torch.device("cuda:0")
A, b, x = O.make_problem(P, m, n, B, seed=1234)
args = argparse.Namespace(GHN_iter_num=K, GHyp_hidden=100, DADMM_mode="diff", alpha_max=0.1,
                          tau_max=0.99, rho_max=0.99, eta_max=0.99)
gnn = GM.DLASSO_GNNHyp3_Progressive(torch.from_numpy(A)[None].to(dev), args).to(dev).train()
graphs = ingest([O.connected_er_graph(P, 0.5, seed=100 + s) for s in range(B)], P, B, dev)
bt = torch.from_numpy(b)[..., None].to(dev)
lab = torch.from_numpy(x)[..., None].to(dev)
opt = torch.optim.AdamW(gnn.parameters(), lr=1e-4)


def step():
    Y, _ = gnn(bt, graphs)
    _, lf = gnn_dlasso_utils.compute_loss(Y, lab)
    opt.zero_grad()
    lf.backward()


step()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
print(prof.key_averages(group_by_stack_n=4).table(sort_by="device_time_total", row_limit=40,
                                                  max_name_column_width=60))
