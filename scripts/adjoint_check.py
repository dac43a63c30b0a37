#!/usr/bin/env python3
"""Adjoint accuracy and timing at the headline shape (diagnostic, GPU).

Prints the adjoint's error along its own trajectory (vs oracle.backward_np64, relative to the
largest entry) at a 64-sample slice, then HIP-event times of the recording forward, the plain
forward and the adjoint at B=4096, P=5, n=256, m=64, K=25."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hyperparameter-gnn_unfolded-d-admm-main_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle as O  # noqa: E402
from dadmm_hip import PreparedOperator, forward_raw, ingest  # noqa: E402
from dadmm_hip.ops import backward_raw  # noqa: E402

dev = torch.device("cuda:0")
TR = np.load(os.path.join(ROOT, "tests", "golden", "fixture_25_iter_general_learning_seq_hyp_param.npy"))
hyp = O.hyp_table(TR, [0.1, 0.99, 0.99, 0.99])
P, m, n, K = 5, 64, 256, 25
out = {}
for B, per in ((64, False), (64, True)):
    A, b, _ = O.make_problem(P, m, n, B, seed=11)
    graphs = ([O.connected_er_graph(P, 0.5, seed=s) for s in range(B)] if per
              else [O.er_graph(P, 0.5, seed=7)] * B)
    rng = np.random.default_rng(0)
    y0, U0, d0 = (1e-2 * rng.standard_normal((3, B, P, n))).astype(np.float32)
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)
    op = PreparedOperator(t(A))
    g = ingest(graphs, P, B, dev)
    Y, _, st, tr = forward_raw(op, t(b), g, t(hyp), t(y0), t(U0), t(d0), record=True)
    gY = rng.standard_normal((K, B, P, n)).astype(np.float32)
    dh = backward_raw(op, g, tr, t(gY)).cpu().numpy().astype(np.float64)
    want = O.backward_np64(A, graphs, hyp, y0, d0, Y.cpu().numpy(), tr.Grec.cpu().numpy(),
                           tr.Urec.cpu().numpy(), gY)
    out[f"rel_err_B{B}_{'per_sample' if per else 'shared'}"] = float(
        np.abs(dh - want).max() / np.abs(want).max())

B = 4096
A, b, _ = O.make_problem(P, m, n, B, seed=1234)
t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)
op = PreparedOperator(t(A))
G = O.er_graph(P, 0.5, seed=7)
g = ingest([G] * B, P, B, dev)
bt, ht = t(b), t(hyp)
y0, U0, d0 = (torch.randn(3, B, P, n, device=dev) * 1e-2).unbind(0)
gY = torch.randn(K, B, P, n, device=dev)


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


res = {}
res["forward_ms"] = timeit(lambda: forward_raw(op, bt, g, ht, y0, U0, d0))
res["forward_record_ms"] = timeit(lambda: forward_raw(op, bt, g, ht, y0, U0, d0, record=True))
_, _, _, tr = forward_raw(op, bt, g, ht, y0, U0, d0, record=True)
res["backward_ms"] = timeit(lambda: backward_raw(op, g, tr, gY))
out.update(res)
print(json.dumps(out))
