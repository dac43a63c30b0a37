#!/usr/bin/env python3
"""Run one BASELINE config's forward a few times (for rocprofv3 kernel traces / PMC passes).

    python scripts/prof_config.py [P n m B K prob per_sample(0/1) path]   default: configs[2]"""
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
for _ in range(4):
    forward_raw(op, bt, g, ht, path=path)
torch.cuda.synchronize()
print("done", P, n, m, B, K, path)
