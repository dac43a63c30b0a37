#!/usr/bin/env python3
"""Module train steps at the headline shape (forward + compute_loss + loss.backward()), for
rocprofv3 kernel traces."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hyperparameter-gnn_unfolded-d-admm-main_amd")]
import torch  # noqa: E402

import gnn_dlasso_utils  # noqa: E402
import oracle as O  # noqa: E402
import unfolded_DLASSO  # noqa: E402

P, m, n, B, K = 5, 64, 256, 4096, 25
dev = torch.device("cuda:0")
A, b, x = O.make_problem(P, m, n, B, seed=1234)
args = argparse.Namespace(GHN_iter_num=K, DADMM_mode="diff", alpha_max=0.1, tau_max=0.99,
                          rho_max=0.99, eta_max=0.99, max_penalty_threshold=0.8,
                          penalty_reduction_factor=0.95)
model = unfolded_DLASSO.DLASSO_unfolded(torch.from_numpy(A)[None].to(dev), args).to(dev)
model.train()
G = O.er_graph(P, 0.5, seed=7)
bt = torch.from_numpy(b)[..., None].to(dev)
label = torch.from_numpy(x)[..., None].to(dev)
opt = torch.optim.Adam(model.parameters(), lr=1e-3)
for _ in range(6):
    Y, _ = model(bt, [G] * B)
    lm, lf = gnn_dlasso_utils.compute_loss(Y, label)
    opt.zero_grad()
    lf.backward()
    opt.step()
torch.cuda.synchronize()
print("done")
