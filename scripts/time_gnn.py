#!/usr/bin/env python3
"""Time the GNN model's eval forward (graphed inference path, pre-ingested device graphs) with
the library DADMM_LIB_VARIANT names; one JSON line with the median and an output checksum.
    python scripts/time_gnn.py [B P n m K reps]      (default: configs[4]'s shard 1024 50 1024 32 50 3)"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hyperparameter-gnn_unfolded-d-admm-main_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle as O  # noqa: E402  (input generator only)

B, P, n, m, K, reps = (int(x) for x in (sys.argv[1:7] if len(sys.argv) > 6 else (1024, 50, 1024, 32, 50, 3)))
import gnn_dlasso_models_progressive as GM  # noqa: E402
from dadmm_hip.graph import generate_er  # noqa: E402
dev = torch.device("cuda:0")
A, b, _ = O.make_problem(P, m, n, B, seed=55)
torch.manual_seed(0)
args = argparse.Namespace(GHN_iter_num=K, GHyp_hidden=100, DADMM_mode="diff", alpha_max=0.1,
                          tau_max=0.99, rho_max=0.99, eta_max=0.99)
g = GM.DLASSO_GNNHyp3_Progressive(torch.from_numpy(A)[None].to(dev), args).to(dev).eval()
gb = generate_er(B, P, 0.5, 5, dev)
bt = torch.from_numpy(b)[..., None].to(dev)
gen = torch.Generator(device=dev).manual_seed(1)
inits = tuple(1e-2 * torch.randn((B, P, n), device=dev, generator=gen) for _ in range(3))
ts = []
with torch.no_grad():
    for it in range(reps + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        Y, _ = g(bt, gb, inits=inits)
        e1.record()
        torch.cuda.synchronize()
        if it >= 1:
            ts.append(e0.elapsed_time(e1))
print(json.dumps({"lib": os.path.basename(os.environ.get("DADMM_LIB_VARIANT", "libdadmm.so")),
                  "cfg": [B, P, n, m, K], "median_ms": float(np.median(ts)), "min_ms": float(np.min(ts)),
                  "status": int(g.last_status.item()), "Ysum": float(Y.double().sum())}))
