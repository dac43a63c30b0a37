#!/usr/bin/env python3
"""Time the hypernetwork's GEMM launches at the GNN train step's small batch (default B = 256, P = 5):
the plain linear (bias epilogue), the inference GCN layer and the training GCN layer (per-sample
BatchNorm statistics + dropout), each as 20 back-to-back launches between HIP events (the train
step runs them back to back), median of 7 rounds, per launch. The library DADMM_LIB_VARIANT names.
    python scripts/time_gcn_train.py [B P]"""
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

B, P = (int(v) for v in (sys.argv[1:3] if len(sys.argv) > 2 else (256, 5)))
dev = torch.device("cuda:0")
L = _lib.load()
gb = generate_er(B, P, 0.5, 5, dev)
ahat = G.normalized_adjacency(gb.nbr, P, adj=gb.adj).contiguous()
gen = torch.Generator(device=dev).manual_seed(0)
p = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
R = B * P


_warm = [False]


def timeit(fn, n=20, rounds=7):
    fn()
    torch.cuda.synchronize()
    if not _warm[0]:   # the GPU clock ramps over the first ~0.5 s of work
        import time
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.6:
            for _ in range(50):
                fn()
            torch.cuda.synchronize()
        _warm[0] = True
    ts = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / n)
    return float(np.median(ts))


out = {"lib": os.path.basename(os.environ.get("DADMM_LIB_VARIANT", "libdadmm.so")), "B": B, "P": P,
       "kw": os.environ.get("DADMM_HYPER_KW", "1")}
SHAPES = [tuple(int(v) for v in t.split('x')) for t in os.environ.get('SHAPES', '400x400,200x400,100x200,256x100').split(',')]
for K, N in SHAPES:
    x = torch.randn(R, K, device=dev, generator=gen)
    W = torch.randn(N, K, device=dev, generator=gen) / np.sqrt(K)
    bias, rm, bw, bb = (torch.randn(N, device=dev, generator=gen) for _ in range(4))
    rv = torch.rand(N, device=dev, generator=gen) + 0.5
    y = torch.empty(R, N, device=dev)
    mo = torch.empty(R, N, device=dev)
    mean, var = torch.empty(B, N, device=dev), torch.empty(B, N, device=dev)
    dz = torch.empty(R, N, device=dev)
    part = torch.empty(3 * B, N, device=dev)

    def lin():
        assert L.dadmm_hyper_linear(R, K, N, p(x), K, K, None, 0, p(W), p(bias), p(y), N, s) == 0, L.dadmm_last_error()

    def gcn():
        rc = L.dadmm_hyper_gcn(B, P, K, N, p(x), K, K, None, 0, p(W), p(bias), p(ahat), 1, p(rm), p(rv), p(bw),
                               p(bb), ctypes.c_float(1e-5), ctypes.c_float(0.01), p(y), N, s)
        assert rc == 0, L.dadmm_last_error()

    def gcn_train():
        rc = L.dadmm_hyper_gcn_train(B, P, K, N, p(x), K, K, None, 0, p(W), p(bias), p(ahat), 1, p(bw), p(bb),
                                     ctypes.c_float(1e-5), ctypes.c_float(0.01), ctypes.c_float(0.1),
                                     ctypes.c_uint64(7), 3, p(y), N, p(mo), p(mean), p(var), None, None, s)
        assert rc == 0, L.dadmm_last_error()

    def gcn_bwd():
        rc = L.dadmm_hyper_gcn_train_bwd(B, P, N, p(y), p(mo), p(mean), p(var), p(bw), ctypes.c_float(1e-5),
                                         p(ahat), 1, ctypes.c_float(0.01), ctypes.c_float(0.1), ctypes.c_uint64(7), 3,
                                         p(dz), p(part), 0, s)
        assert rc == 0, L.dadmm_last_error()

    Wt = W.t().contiguous()   # [K][N]: the input-gradient GEMM dx = dy W (x = dy [R][N] -> [R][K])
    dzk = torch.empty(R, K, device=dev)
    dyN = torch.randn(R, N, device=dev, generator=gen)
    mK, meanK, varK = torch.randn(R, K, device=dev), torch.randn(B, K, device=dev), torch.rand(B, K, device=dev) + 0.5
    bwK = torch.randn(K, device=dev, generator=gen)
    partK = torch.empty(3 * B, K, device=dev)

    def lin_gcn_bwd():
        rc = L.dadmm_hyper_linear_gcn_bwd(B, P, N, K, p(dyN), N, p(Wt), p(mK), p(meanK), p(varK), p(bwK),
                                          ctypes.c_float(1e-5), p(ahat), 1, ctypes.c_float(0.01),
                                          ctypes.c_float(0.1), ctypes.c_uint64(7), 3, p(dzk), p(partK), 0, s)
        assert rc == 0, L.dadmm_last_error()

    gcn_train()
    r = {"linear_us": timeit(lin), "gcn_us": timeit(gcn), "gcn_train_us": timeit(gcn_train),
         "gcn_bwd_us": timeit(gcn_bwd), "linear_gcn_bwd_us": timeit(lin_gcn_bwd)}
    gcn_train()
    torch.cuda.synchronize()
    r["ysum"] = float(y.double().sum())
    out[f"{K}x{N}"] = {k: round(v, 3) for k, v in r.items()}
print(json.dumps(out))
