#!/usr/bin/env python3
"""Host side of the headline module forward (bench.py's timed step: DLASSO_unfolded under no_grad,
B=4096 P=5 n=256 m=64 K=25, shared ER(0.5) graph list): per forward, the host's enqueue time
(no synchronisation inside the loop) against the wall time with the GPU, then a cProfile of the
enqueue (CPROF=1).   python scripts/time_module_host.py [steps]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hyperparameter-gnn_unfolded-d-admm-main_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle as O  # noqa: E402  (input generator only)
import unfolded_DLASSO  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
P, n, m, K, B = 5, 256, 64, 25, 4096
dev = torch.device("cuda:0")
A, _, _ = O.make_problem(P, m, n, 1, seed=1234)
gen = torch.Generator().manual_seed(4321)
x = 2 * torch.randn(B, n, generator=gen) * (torch.rand(B, n, generator=gen) <= 0.25)
bt = torch.einsum("pmn,bn->bpm", torch.from_numpy(A), x)[..., None].to(dev)
graph_list = [O.er_graph(P, 0.5, seed=7)] * B
args = argparse.Namespace(GHN_iter_num=K, DADMM_mode="diff", alpha_max=0.1, tau_max=0.99, rho_max=0.99,
                          eta_max=0.99, max_penalty_threshold=0.8, penalty_reduction_factor=0.95)
model = unfolded_DLASSO.DLASSO_unfolded(torch.from_numpy(A)[None].to(dev), args).to(dev).eval()
if os.environ.get("FIXTURE", "1") != "0":   # the bench's trained seq_hyp (FIXTURE=0: the random init)
    param = np.load(os.path.join(ROOT, "tests", "golden", "fixture_25_iter_general_learning_seq_hyp_param.npy"))
    with torch.no_grad():
        model.seq_hyp.param.copy_(torch.from_numpy(param))


def step():
    with torch.no_grad():
        return model(bt, graph_list)


for _ in range(5):
    step()
torch.cuda.synchronize()
for rnd in range(3):
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"round {rnd}: host enqueue {1e3 * (t1 - t0) / steps:.3f} ms/forward, wall {1e3 * (t2 - t0) / steps:.3f} ms/forward")
if os.environ.get("CPROF"):
    import cProfile
    import pstats
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(steps):
        step()
    pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)
