#!/usr/bin/env python3
"""Time one BASELINE config's forward (HIP events, median of N) with the library that
DADMM_LIB_VARIANT names (default: the in-tree build). Prints one JSON line.

    DADMM_LIB_VARIANT=build/var/libdadmm_x.so python scripts/time_config.py [P n m B K prob per_sample path]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hyperparameter-gnn_unfolded-d-admm-main_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle as O  # noqa: E402
from dadmm_hip import PreparedOperator, forward_raw, ingest  # noqa: E402

args = sys.argv[1:]
P, n, m, B, K = (int(v) for v in (args[:5] if len(args) >= 5 else (16, 512, 64, 4096, 25)))
prob = float(args[5]) if len(args) > 5 else 0.3
per_sample = bool(int(args[6])) if len(args) > 6 else True
path = args[7] if len(args) > 7 else "auto"
dev = torch.device("cuda:0")
A, b, _ = O.make_problem(P, m, n, B, seed=77)
graphs = ([O.connected_er_graph(P, prob, seed=s) for s in range(B)] if per_sample
          else [O.er_graph(P, prob, seed=7)] * B)
rng = np.random.default_rng(0)
hyp = O.hyp_table((0.3 * rng.standard_normal((K, P, 4))).astype(np.float32), [0.1, 0.99, 0.99, 0.99])
op = PreparedOperator(torch.from_numpy(A).to(dev))
g = ingest(graphs, P, B, dev)
bt, ht = torch.from_numpy(b).to(dev), torch.from_numpy(hyp).to(dev)
gen = torch.Generator().manual_seed(99)
y0, U0, d0 = (1e-2 * torch.randn(B, P, n, generator=gen)).to(dev), \
    (1e-2 * torch.randn(B, P, n, generator=gen)).to(dev), (1e-2 * torch.randn(B, P, n, generator=gen)).to(dev)
ref = None
ts = []
for it in range(12):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    out = forward_raw(op, bt, g, ht, y0, U0, d0, path=path)
    e1.record()
    torch.cuda.synchronize()
    if it >= 2:
        ts.append(e0.elapsed_time(e1))
    Y = out[0] if isinstance(out, tuple) else out
    if ref is None:
        ref = Y.clone()
    elif not torch.equal(ref, Y) and not os.environ.get("DADMM_ABLATION"):
        raise SystemExit("nondeterministic output")
print(json.dumps({"lib": os.path.basename(os.environ.get("DADMM_LIB_VARIANT", "libdadmm.so")),
                  "cfg": [P, n, m, B, K, prob, per_sample, path], "median_ms": float(np.median(ts)),
                  "min_ms": float(np.min(ts)), "Ysum": float(Y.double().sum())}))
