#!/usr/bin/env python3
"""Time one inference GCN layer (dadmm_hyper_gcn) in isolation with HIP events (median of 20), with the
library DADMM_LIB_VARIANT names; prints one JSON line with TFLOP/s (GEMM flops only, 2 rows K N).
    python scripts/time_gcn_layer.py [B P K N]   (default: configs[4]'s 400-wide layer 1024 50 400 400)"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hyperparameter-gnn_unfolded-d-admm-main_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from dadmm_hip import _lib  # noqa: E402
from dadmm_hip.graph import generate_er  # noqa: E402
import gnn_dlasso_models_progressive as G  # noqa: E402

B, P, K, N = (int(v) for v in (sys.argv[1:5] if len(sys.argv) > 4 else (1024, 50, 400, 400)))
dev = torch.device("cuda:0")
L = _lib.load()
gb = generate_er(B, P, 0.5, 5, dev)
ahat = G.normalized_adjacency(gb.nbr, P, adj=gb.adj).contiguous()
gen = torch.Generator(device=dev).manual_seed(0)
x = torch.randn(B * P, K, device=dev, generator=gen)
W = torch.randn(N, K, device=dev, generator=gen) / np.sqrt(K)
bias, rm, bw, bb = (torch.randn(N, device=dev, generator=gen) for _ in range(4))
rv = torch.rand(N, device=dev, generator=gen) + 0.5
y = torch.empty(B * P, N, device=dev)
p = lambda t: ctypes.c_void_p(t.data_ptr())
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
def run():
    rc = L.dadmm_hyper_gcn(B, P, K, N, p(x), K, K, None, 0, p(W), p(bias), p(ahat), 1, p(rm), p(rv), p(bw), p(bb),
                           1e-5, 0.01, p(y), N, s)
    assert rc == 0, L.dadmm_last_error()
ts = []
for it in range(25):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); run(); e1.record(); torch.cuda.synchronize()
    if it >= 5:
        ts.append(e0.elapsed_time(e1))
ms = float(np.median(ts))
print(json.dumps({"lib": os.path.basename(os.environ.get("DADMM_LIB_VARIANT", "libdadmm.so")),
                  "gcn32": os.environ.get("DADMM_GCN32", "1"), "cfg": [B, P, K, N], "median_us": ms * 1e3,
                  "gemm_TFLOPs": 2.0 * B * P * K * N / (ms * 1e-3) / 1e12, "ysum": float(y.double().sum())}))
