#!/usr/bin/env python3
"""Time ablation builds of the fused kernel (build/ablate/libdadmm_*.so, `make -C csrc ablate`)
on the headline workload, interleaved in one process (MI355X_MICROARCH §5.4 rule 24).
Timing only: the ablated builds compute wrong results by construction."""
import ctypes
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hyperparameter-gnn_unfolded-d-admm-main_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from dadmm_hip import _lib  # noqa: E402


def main():
    B, P, m, n, K = (int(x) for x in (sys.argv[1:6] if len(sys.argv) > 5 else (4096, 5, 64, 256, 25)))
    rounds = 7
    dev = torch.device("cuda:0")
    libs = {}
    for path in sorted(glob.glob(os.path.join(ROOT, "build", "ablate", "libdadmm_*.so"))):
        if "stamps" in path:          # diagnostic build: needs its stamp buffer (scripts/stamps.py)
            continue
        L = ctypes.CDLL(path)
        L.dadmm_forward.argtypes = [ctypes.POINTER(_lib.Dims)] + [ctypes.c_void_p] * 13
        L.dadmm_prepare_operator.argtypes = [ctypes.POINTER(_lib.Dims)] + [ctypes.c_void_p] * 3
        L.dadmm_operator_bytes.restype = ctypes.c_size_t
        L.dadmm_operator_bytes.argtypes = [ctypes.POINTER(_lib.Dims)]
        libs[os.path.basename(path)[9:-3]] = L
    g = torch.Generator().manual_seed(0)
    A = torch.randn(P, m, n, generator=g).to(dev) * 0.1
    b = torch.randn(B, P, m, generator=g).to(dev)
    y0, U0, d0 = (torch.randn(B, P, n, generator=g).to(dev) * 1e-2 for _ in range(3))
    hyp = torch.full((K, P, 4), 0.05, device=dev)
    nbr = torch.tensor([0b00110, 0b01001, 0b10001, 0b00010, 0b00100], dtype=torch.int64, device=dev)[:P]
    deg = torch.tensor([2.0, 2, 2, 1, 1], device=dev)[:P]
    Y = torch.empty(K, B, P, n, device=dev)
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    d = _lib.Dims(B=B, P=P, m=m, n=n, K=K, variant=0, hyp_rows=P, graph_shared=1)
    ops = {}
    for name, L in libs.items():
        ws = torch.empty(L.dadmm_operator_bytes(ctypes.byref(d)) // 4, device=dev)
        assert L.dadmm_prepare_operator(ctypes.byref(d), ctypes.c_void_p(A.data_ptr()),
                                        ctypes.c_void_p(ws.data_ptr()), None) == 0
        ops[name] = ws
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    times = {k: [] for k in libs}
    for r in range(rounds):
        for name, L in libs.items():
            s = torch.cuda.current_stream()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            for it in range(3):
                if it == 2:
                    e0.record(s)
                rc = L.dadmm_forward(ctypes.byref(d), p(ops[name]), p(b), p(nbr), None, p(deg),
                                     p(hyp), p(y0), p(U0), p(d0), p(Y), None, p(st),
                                     ctypes.c_void_p(s.cuda_stream))
                assert rc == 0, rc
            e1.record(s)
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1))
    out = {k: {"median_ms": float(np.median(v)), "min_ms": float(np.min(v))} for k, v in times.items()}
    print(json.dumps({"B": B, "P": P, "m": m, "n": n, "K": K, "ablations": out}, indent=1))


if __name__ == "__main__":
    main()
