#!/usr/bin/env python3
"""Time the two adjoint paths on one recorded trajectory (HIP events, median of 10):
the fused adjoint (dadmm_backward, state on chip) and the general one (dadmm_adjoint, state in
HBM), and check that they agree.   python scripts/time_adjoint.py [P n m B K]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hyperparameter-gnn_unfolded-d-admm-main_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle as O  # noqa: E402  (input generator only)
from dadmm_hip import PreparedOperator, ingest  # noqa: E402
from dadmm_hip.ops import backward_raw, forward_raw  # noqa: E402

P, n, m, B, K = (int(v) for v in (sys.argv[1:6] if len(sys.argv) > 5 else (5, 256, 64, 4096, 25)))
dev = torch.device("cuda:0")
A, b, _ = O.make_problem(P, m, n, B, seed=3)
op = PreparedOperator(torch.from_numpy(A).to(dev))
g = ingest([O.er_graph(P, 0.5, seed=7)] * B, P, B, dev)
rng = np.random.default_rng(0)
hyp = torch.from_numpy(O.hyp_table((0.3 * rng.standard_normal((K, P, 4))).astype(np.float32),
                                   [0.1, 0.99, 0.99, 0.99])).to(dev)
bt = torch.from_numpy(b).to(dev)
out = {"cfg": [P, n, m, B, K]}
for path in ("stepwise", "auto"):
    Y, _, _, tr = forward_raw(op, bt, g, hyp, record=True, path=path)
    gY = torch.randn(Y.shape, device=dev, generator=torch.Generator(device=dev).manual_seed(1))
    res = {}
    for bp in (("fused", "general") if tr.fused else ("general",)):
        ts = []
        for it in range(12):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            d = backward_raw(op, g, tr, gY, path=bp)
            e1.record()
            torch.cuda.synchronize()
            if it >= 2:
                ts.append(e0.elapsed_time(e1))
        res[bp] = (float(np.median(ts)), d.clone())
    out[path] = {k: v[0] for k, v in res.items()}
    if len(res) == 2:
        a, c = res["fused"][1].double(), res["general"][1].double()
        out[path]["max_rel_diff"] = float(((a - c).abs().max() / a.abs().max()).item())
print(json.dumps(out))
