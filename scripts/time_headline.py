#!/usr/bin/env python3
"""A/B timing of the fused forward's two work divisions at one shape (default: the headline,
B=4096 P=5 n=256 m=64 K=25, shared ER(0.5) graph, trained hyper-parameters).

For each division (DADMM_FUSED_DIVISION=agents | rows) and several interleaved rounds: the fused
launch alone (HIP events around dadmm_forward on its stream, explicit inits) and the module
forward (DLASSO_unfolded under no_grad: prologue draws + fused kernel + gate), plus an output
checksum so a division that changes results is visible. One JSON line per (round, division).

    python scripts/time_headline.py [B P n m K rounds reps]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hyperparameter-gnn_unfolded-d-admm-main_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle as O  # noqa: E402  (input generator only)
import unfolded_DLASSO  # noqa: E402
from dadmm_hip import PreparedOperator, forward_raw, ingest  # noqa: E402

av = [int(x) for x in sys.argv[1:8]] + [None] * 7
B, P, n, m, K, rounds, reps = (v if v is not None else d for v, d in
                               zip(av, (4096, 5, 256, 64, 25, 3, 20)))
dev = torch.device("cuda:0")
A, _, _ = O.make_problem(P, m, n, 1, seed=1234)
gen = torch.Generator().manual_seed(4321)
x = 2 * torch.randn(B, n, generator=gen) * (torch.rand(B, n, generator=gen) <= 0.25)
b = torch.einsum("pmn,bn->bpm", torch.from_numpy(A), x).float()
G = O.er_graph(P, 0.5, seed=7)
param = np.load(os.path.join(ROOT, "tests", "golden", "fixture_25_iter_general_learning_seq_hyp_param.npy"))
if param.shape != (K, P, 4):
    param = (0.3 * np.random.default_rng(0).standard_normal((K, P, 4))).astype(np.float32)
hyp = torch.from_numpy(O.hyp_table(param, [0.1, 0.99, 0.99, 0.99])).to(dev)
op = PreparedOperator(torch.from_numpy(A).to(dev))
g = ingest([G] * B, P, B, dev)
bt = b.to(dev)
y0, U0, d0 = (1e-2 * torch.randn(3, B, P, n, generator=gen)).to(dev)
args = argparse.Namespace(GHN_iter_num=K, DADMM_mode="diff", alpha_max=0.1, tau_max=0.99, rho_max=0.99,
                          eta_max=0.99, max_penalty_threshold=0.8, penalty_reduction_factor=0.95)
model = unfolded_DLASSO.DLASSO_unfolded(torch.from_numpy(A)[None].to(dev), args).to(dev).eval()
if param.shape == (K, P, 4):
    with torch.no_grad():
        model.seq_hyp.param.copy_(torch.from_numpy(param))
graph_list = [G] * B


def timed(fn, reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        out = fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps, out


for rnd in range(rounds):
    for div in os.environ.get("DIVISIONS", "agents,rows").split(","):
        os.environ["DADMM_FUSED_DIVISION"] = div
        ms_k, out = timed(lambda: forward_raw(op, bt, g, hyp, y0, U0, d0, path="fused"), reps)
        Y, _, st = out
        with torch.no_grad():
            ms_f, (Ym, _) = timed(lambda: model(bt[..., None], graph_list), reps)
            # host time to enqueue one module forward (no sync inside the loop): when it nears the
            # GPU time, the step becomes host-bound
            import time as _time
            torch.cuda.synchronize()
            t0 = _time.perf_counter()
            for _ in range(reps):
                model(bt[..., None], graph_list)
            host_ms = (_time.perf_counter() - t0) * 1e3 / reps
            torch.cuda.synchronize()
        print(json.dumps({"lib": os.path.basename(os.environ.get("DADMM_LIB_VARIANT", "libdadmm.so")),
                          "round": rnd, "division": div, "cfg": [B, P, n, m, K],
                          "kernel_ms": ms_k, "module_forward_ms": ms_f, "host_enqueue_ms": host_ms,
                          "M_iters_per_s": B * K / ms_f / 1e3, "status": int(st.item()),
                          "Ysum": float(Y.double().sum())}),
              flush=True)
