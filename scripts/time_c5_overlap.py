#!/usr/bin/env python3
"""Feasibility probe for pipelining the GNN forward over batch halves: the configs[4] shard
(P=50, n=1024, m=32, K, h=100, eval + no_grad, graphed) as one B-sample forward, as two B/2
forwards one after the other, and as two B/2 forwards on two streams at once (two model copies,
so no cached buffer is shared). HIP events around each form, median of 3.
    python scripts/time_c5_overlap.py [B K]"""
import argparse
import copy
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hyperparameter-gnn_unfolded-d-admm-main_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import gnn_dlasso_models_progressive as GM  # noqa: E402
import oracle as O  # noqa: E402  (input generator only)
from dadmm_hip.graph import generate_er  # noqa: E402

B, K = (int(v) for v in (sys.argv[1:3] if len(sys.argv) > 2 else (1024, 10)))
P, n, m = 50, 1024, 32
dev = torch.device("cuda:0")
A, b, _ = O.make_problem(P, m, n, B, seed=55)
args = argparse.Namespace(GHN_iter_num=K, GHyp_hidden=100, DADMM_mode="diff", alpha_max=0.1,
                          tau_max=0.99, rho_max=0.99, eta_max=0.99)
g0 = GM.DLASSO_GNNHyp3_Progressive(torch.from_numpy(A)[None].to(dev), args).to(dev).eval()
g1 = copy.deepcopy(g0)
g2 = copy.deepcopy(g0)
bt = torch.from_numpy(b)[..., None].to(dev)
H = B // 2
gball = generate_er(B, P, 0.5, 3, dev)
ga = generate_er(H, P, 0.5, 3, dev)
gbb = generate_er(B - H, P, 0.5, 4, dev)
ba, bb = bt[:H].contiguous(), bt[H:].contiguous()
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def full():
    g0(bt, gball)


def seq():
    g1(ba, ga)
    g2(bb, gbb)


def conc():
    cur = torch.cuda.current_stream()
    s1.wait_stream(cur)
    s2.wait_stream(cur)
    with torch.cuda.stream(s1):
        g1(ba, ga)
    with torch.cuda.stream(s2):
        g2(bb, gbb)
    cur.wait_stream(s1)
    cur.wait_stream(s2)


def stag(cycles):
    def f():
        cur = torch.cuda.current_stream()
        s1.wait_stream(cur)
        s2.wait_stream(cur)
        with torch.cuda.stream(s1):
            g1(ba, ga)
        with torch.cuda.stream(s2):
            torch.cuda._sleep(cycles)      # half B starts later: its phases offset from half A's
            g2(bb, gbb)
        cur.wait_stream(s1)
        cur.wait_stream(s2)
    return f


def sleep_only(cycles):
    return lambda: torch.cuda._sleep(cycles)


def ms(fn, reps=3):
    with torch.no_grad():
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
    return float(np.median(ts))


out = {"B": B, "K": K}
for name, fn in (("full", full), ("seq_halves", seq), ("concurrent_halves", conc),
                 ("sleep_1M", sleep_only(1000000)), ("staggered_1M", stag(1000000)),
                 ("sleep_2M", sleep_only(2000000)), ("staggered_2M", stag(2000000)),
                 ("sleep_4M", sleep_only(4000000)), ("staggered_4M", stag(4000000)), ("full_again", full)):
    out[name + "_ms"] = round(ms(fn), 3)
print(json.dumps(out))
