#!/usr/bin/env python3
"""Time one weight gradient (dadmm_hyper_wgrad: G += dZ^T X, with the bias column sums) in isolation
with HIP events (median of 20), with the library DADMM_LIB_VARIANT names; prints one JSON line with
TFLOP/s (2 R N K) and a checksum of G.
    python scripts/time_wgrad.py [R N K]   (default: the B = 4096 train step's batched 400 x 400 GCN
    gradient over 25 iterations: 512000 400 400)"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hyperparameter-gnn_unfolded-d-admm-main_amd")]
import torch  # noqa: E402

from dadmm_hip import _lib  # noqa: E402

R, N, K = (int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (512000, 400, 400)))
dev = torch.device("cuda:0")
L = _lib.load()
gen = torch.Generator(device=dev).manual_seed(0)
dz = torch.randn(R, N, device=dev, generator=gen)
x = torch.randn(R, K, device=dev, generator=gen)
G = torch.zeros(N, K, device=dev)
gb = torch.zeros(N, device=dev)
scratch = torch.empty(max(L.dadmm_hyper_wgrad_scratch_bytes(R, N, K), 16) // 4 + 4, device=dev)
p = lambda t: ctypes.c_void_p(t.data_ptr())
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def run():
    rc = L.dadmm_hyper_wgrad(R, N, K, p(dz), N, p(x), K, K, None, 0, p(G), p(gb), 0, p(scratch), s)
    assert rc == 0, L.dadmm_last_error()


ts = []
for it in range(25):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    run()
    e1.record()
    torch.cuda.synchronize()
    if it >= 5:
        ts.append(e0.elapsed_time(e1))
ts.sort()
ms = ts[len(ts) // 2]
print(json.dumps({"lib": os.path.basename(_lib.LIB_PATH), "R": R, "N": N, "K": K, "median_ms": ms,
                  "tflops": 2.0 * R * N * K / ms / 1e9, "Gsum": float(G.double().sum()),
                  "splits_bytes": L.dadmm_hyper_wgrad_scratch_bytes(R, N, K)}))
