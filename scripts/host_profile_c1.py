#!/usr/bin/env python3
"""Host cost of one DLASSO_unfolded.forward at BASELINE configs[1] (B = 1024): enqueue time per
call (no synchronisation inside the loop) against the GPU time per call, and a cProfile of the
enqueue loop.    python scripts/host_profile_c1.py [B] [calls]"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hyperparameter-gnn_unfolded-d-admm-main_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle as O  # noqa: E402  (input generator only)
import unfolded_DLASSO  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
N = int(sys.argv[2]) if len(sys.argv) > 2 else 200
P, m, n, K = 5, 64, 256, 25
dev = torch.device("cuda:0")
A, b, _ = O.make_problem(P, m, n, B, seed=1)
G = O.er_graph(P, 0.5, seed=7)
args = argparse.Namespace(GHN_iter_num=K, DADMM_mode="diff", alpha_max=0.1, tau_max=0.99, rho_max=0.99,
                          eta_max=0.99, max_penalty_threshold=0.8, penalty_reduction_factor=0.95)
model = unfolded_DLASSO.DLASSO_unfolded(torch.from_numpy(A).to(dev)[None], args).to(dev).eval()
bt = torch.from_numpy(b).to(dev)[..., None]
graphs = [G] * B


def f():
    with torch.no_grad():
        model(bt, graphs)


for _ in range(20):
    f()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
t0 = time.perf_counter()
e0.record()
for _ in range(N):
    f()
e1.record()
t1 = time.perf_counter()
torch.cuda.synchronize()
print(f"B={B}: host enqueue {1e6 * (t1 - t0) / N:.1f} us per call, GPU {1e3 * e0.elapsed_time(e1) / N:.1f} us per call")
pr = cProfile.Profile()
pr.enable()
for _ in range(N):
    f()
pr.disable()
torch.cuda.synchronize()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(30)
print(s.getvalue())
