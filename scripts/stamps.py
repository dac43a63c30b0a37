#!/usr/bin/env python3
"""Per-phase cycle shares of the fused kernel from the -DDADMM_STAMPS diagnostic build
(build/ablate/libdadmm_stamps.so). Shares only: the stamps themselves cost cycles."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hyperparameter-gnn_unfolded-d-admm-main_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from dadmm_hip import _lib  # noqa: E402

PHASES = ["gemm1", "barrier1", "gemm2", "elementwise+stores", "barrier2"]


def main():
    B, P, m, n, K = 4096, 5, 64, 256, 25
    dev = torch.device("cuda:0")
    L = ctypes.CDLL(os.path.join(ROOT, "build", "ablate", "libdadmm_stamps.so"))
    L.dadmm_forward.argtypes = [ctypes.POINTER(_lib.Dims)] + [ctypes.c_void_p] * 13
    L.dadmm_prepare_operator.argtypes = [ctypes.POINTER(_lib.Dims)] + [ctypes.c_void_p] * 3
    L.dadmm_operator_bytes.restype = ctypes.c_size_t
    L.dadmm_operator_bytes.argtypes = [ctypes.POINTER(_lib.Dims)]
    L.dadmm_debug_set_stamps.argtypes = [ctypes.c_void_p]
    g = torch.Generator().manual_seed(0)
    A = torch.randn(P, m, n, generator=g).to(dev) * 0.1
    b = torch.randn(B, P, m, generator=g).to(dev)
    y0, U0, d0 = (torch.randn(B, P, n, generator=g).to(dev) * 1e-2 for _ in range(3))
    hyp = torch.full((K, P, 4), 0.05, device=dev)
    nbr = torch.tensor([0b00110, 0b01001, 0b10001, 0b00010, 0b00100], dtype=torch.int64, device=dev)
    deg = torch.tensor([2.0, 2, 2, 1, 1], device=dev)
    Y = torch.empty(K, B, P, n, device=dev)
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    d = _lib.Dims(B=B, P=P, m=m, n=n, K=K, variant=0, hyp_rows=P, graph_shared=1)
    ws = torch.empty(L.dadmm_operator_bytes(ctypes.byref(d)) // 4, device=dev)
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    assert L.dadmm_prepare_operator(ctypes.byref(d), p(A), p(ws), None) == 0
    stamps = torch.zeros((B // 16) * 8 * 8, dtype=torch.int64, device=dev)
    assert L.dadmm_debug_set_stamps(p(stamps)) == 0
    for _ in range(3):
        assert L.dadmm_forward(ctypes.byref(d), p(ws), p(b), p(nbr), None, p(deg), p(hyp), p(y0),
                               p(U0), p(d0), p(Y), None, p(st), None) == 0
    torch.cuda.synchronize()
    s = stamps.view(B // 16, 8, 8)[:, :, :5].cpu().numpy().astype(np.float64)
    tot = s.sum(axis=2)
    out = {}
    for half, sl in (("waves0-3", slice(0, 4)), ("waves4-7", slice(4, 8))):
        v = s[:, sl, :].reshape(-1, 5)
        out[half] = {ph: float(v[:, i].mean() / tot[:, sl].mean()) for i, ph in enumerate(PHASES)}
        out[half]["total_cycles_mean"] = float(tot[:, sl].mean())
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
