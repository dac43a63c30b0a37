#!/usr/bin/env python3
"""Time the forward prologue (the three torch.randn * 1e-2 inits in one launch) at the headline
shape with the library DADMM_LIB_VARIANT names: python scripts/time_prologue.py [B P n reps]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hyperparameter-gnn_unfolded-d-admm-main_amd")]
import torch  # noqa: E402

from dadmm_hip.ops import draw_inits  # noqa: E402

B, P, n, reps = (int(v) for v in (sys.argv[1:5] if len(sys.argv) > 4 else (4096, 5, 256, 50)))
dev = torch.device("cuda:0")
torch.manual_seed(0)
y0, _, _ = draw_inits((B, P, n), dev)
ref = torch.randn((B, P, n), device=dev)   # warm torch's own kernel too
torch.cuda.synchronize()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
ev[0].record()
for _ in range(reps):
    draw_inits((B, P, n), dev)
ev[1].record()
ev[2].record()
for _ in range(reps):
    for _ in range(3):
        torch.randn((B, P, n), device=dev).mul_(1e-2)
ev[3].record()
torch.cuda.synchronize()
torch.manual_seed(1)
a = draw_inits((B, P, n), dev)
torch.manual_seed(1)
b = [torch.randn((B, P, n), device=dev) * 1e-2 for _ in range(3)]
same = all(torch.equal(x, y) for x, y in zip(a, b))
print(json.dumps({"lib": os.path.basename(os.environ.get("DADMM_LIB_VARIANT", "libdadmm.so")),
                  "prologue_ms": ev[0].elapsed_time(ev[1]) / reps,
                  "torch_3randn_ms": ev[2].elapsed_time(ev[3]) / reps, "bit_identical": same}))
