#!/usr/bin/env python3
"""Diagnostic: per-parameter gradient error of the GNN train node vs the torch backend at odd/even B."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "hyperparameter-gnn_unfolded-d-admm-main_amd")]
import torch  # noqa: E402
import gnn_dlasso_utils as U  # noqa: E402
import test_gpu_hyper_train as T  # noqa: E402

cuda = torch.device("cuda:0")
for B in [int(v) for v in sys.argv[1:]] or [50, 51, 52, 13, 12]:
    for hook in (False, True):
        P, n, hidden, K = 5, 32, 8, 4
        model, ref, graphs, inits, bt, label = T._train_pair(cuda, P, n, hidden, "diff", False, B=B)
        if hook:
            model.on_hyp = lambda *a: None
        Y1, _ = model(bt, graphs, K, inits=inits)
        U.compute_loss(Y1, label)[1].backward()
        Y2, _ = ref(bt, graphs, K, inits=inits)
        U.compute_loss(Y2, label)[1].backward()
        bad = []
        for (name, p1), (_, p2) in zip(model.named_parameters(), ref.named_parameters()):
            e = float((p1.grad - p2.grad).abs().max() / p2.grad.abs().max().clamp_min(1e-30))
            if e > 5e-3:
                bad.append(f"{name}:{e:.2e}")
        print(f"B={B} hook={hook} backend={model.last_backend} Ydiff={float((Y1 - Y2).abs().max()):.2e} bad={bad}")
