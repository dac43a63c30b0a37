#!/usr/bin/env python3
"""Time ablation builds of the hypernetwork GEMM (build/hyabl/libdadmm_*.so): dadmm_hyper_gcn /
dadmm_hyper_linear at the GNN model's layer shapes. Timing only (ablated builds are wrong)."""
import ctypes
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hyperparameter-gnn_unfolded-d-admm-main_amd")]
import torch  # noqa: E402

from dadmm_hip import _lib  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    i32, vp, f32 = ctypes.c_int32, ctypes.c_void_p, ctypes.c_float
    libs = {}
    for path in sorted(glob.glob(os.path.join(ROOT, "build", "hyabl", "libdadmm_*.so"))):
        L = ctypes.CDLL(path)
        L.dadmm_hyper_gcn.argtypes = [i32] * 4 + [vp, i32, i32, vp, i32] + [vp] * 3 + [i32] + \
            [vp] * 4 + [f32, f32, vp, i32, vp]
        L.dadmm_hyper_linear.argtypes = [i32] * 3 + [vp, i32, i32, vp, i32, vp, vp, vp, i32, vp]
        libs[os.path.basename(path)[9:-3]] = L
    p = lambda t: vp(t.data_ptr())
    shapes = [("gcn P5 B1024 400x400", 1024, 5, 400, 400), ("gcn P50 B1024 400x400", 1024, 50, 400, 400),
              ("gcn P5 B1024 512x100", 1024, 5, 512, 100), ("lin 1024 2000x400", 1024, 1, 2000, 400)]
    out = {}
    for name, B, P, K, N in shapes:
        rows = B * P
        x = torch.randn(rows, K, device=dev)
        W = torch.randn(N, K, device=dev)
        v = torch.randn(N, device=dev)
        ah = torch.rand(1, P, P, device=dev)
        y = torch.empty(rows, N, device=dev)
        res = {}
        for lname, L in libs.items():
            def run():
                if P > 1:
                    rc = L.dadmm_hyper_gcn(B, P, K, N, p(x), K, K, None, 0, p(W), p(v), p(ah), 0, p(v), p(v),
                                           p(v), p(v), 1e-5, 0.01, p(y), N, None)
                else:
                    rc = L.dadmm_hyper_linear(rows, K, N, p(x), K, K, None, 0, p(W), p(v), p(y), N, None)
                assert rc == 0
            for _ in range(3):
                run()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                run()
            e1.record()
            torch.cuda.synchronize()
            us = 1e3 * e0.elapsed_time(e1) / 20
            res[lname] = {"us": us, "TFLOPs": 2.0 * rows * K * N / (us * 1e-6) / 1e12}
        out[name] = res
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
