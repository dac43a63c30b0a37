#!/usr/bin/env python3
"""Which torch op launches a copy kernel in the headline forward (bench.py's inputs): torch.profiler
over three forwards, printing every aten op that ran a device kernel, with its input shapes."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hyperparameter-gnn_unfolded-d-admm-main_amd")]
import torch  # noqa: E402

import oracle as O  # noqa: E402
import unfolded_DLASSO  # noqa: E402

dev = torch.device("cuda:0")
P, n, m, K, B = 5, 256, 64, 25, 4096
A, _, _ = O.make_problem(P, m, n, 1, seed=1234)
gen = torch.Generator().manual_seed(4321)
x = 2 * torch.randn(B, n, generator=gen) * (torch.rand(B, n, generator=gen) <= 0.25)
b = torch.einsum("pmn,bn->bpm", torch.from_numpy(A), x)
print("A", A.dtype, "b", b.dtype, b.is_contiguous())
bt = b[..., None].to(dev)
G = O.er_graph(P, 0.5, seed=7)
args = argparse.Namespace(GHN_iter_num=K, DADMM_mode="diff", alpha_max=0.1, tau_max=0.99, rho_max=0.99,
                          eta_max=0.99, max_penalty_threshold=0.8, penalty_reduction_factor=0.95)
model = unfolded_DLASSO.DLASSO_unfolded(torch.from_numpy(A)[None].to(dev), args).to(dev)
import numpy as np  # noqa: E402
param = np.load(os.path.join(ROOT, "tests", "golden", "fixture_25_iter_general_learning_seq_hyp_param.npy"))
with torch.no_grad():   # as bench.py: the trained table, eval mode, ONE graph list object reused
    model.seq_hyp.param.copy_(torch.from_numpy(param))
model.eval()
graph_list = [G] * B
with torch.no_grad():
    for _ in range(3):
        model(bt, graph_list)
torch.cuda.synchronize()
from torch.profiler import profile, ProfilerActivity  # noqa: E402
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
    with torch.no_grad():
        for _ in range(3):
            model(bt, graph_list)
    torch.cuda.synchronize()
print(prof.key_averages(group_by_input_shape=True).table(sort_by="cuda_time_total", row_limit=40))
