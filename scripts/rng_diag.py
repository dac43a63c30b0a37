import sys, os
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "hyperparameter-gnn_unfolded-d-admm-main_amd")]
import torch
from dadmm_hip.ops import draw_inits
cuda = torch.device("cuda:0")
shape = (7, 3, 62)
torch.manual_seed(4321)
ref = [torch.randn(shape + (1,), device=cuda)[..., 0] * 1e-2 for _ in range(3)]
torch.manual_seed(4321)
got = draw_inits(shape, cuda, 64)
for r, g in zip(ref, got):
    g = g[..., :62]
    d = (g - r)
    ne = (g != r)
    print("mismatch frac", ne.float().mean().item(), "max abs", d.abs().max().item(), "max rel", (d.abs() / r.abs().clamp_min(1e-30)).max().item())
    idx = ne.nonzero()[:5]
    for i in idx:
        i = tuple(i.tolist())
        print(i, r[i].item(), g[i].item(), (r[i]/1e-2).item())
# raw normals (mean 0 std 1)
torch.manual_seed(4321)
r1 = torch.randn(1000, device=cuda)
torch.manual_seed(4321)
from dadmm_hip import _lib
import ctypes
L = _lib.load()
gen = torch.cuda.default_generators[0]
seed, off = gen.initial_seed(), gen.get_offset()
out = [torch.empty(1000, device=cuda) for _ in range(3)]
L.dadmm_prologue(seed, off, 1000, 1000, 1000, 0.0, 1.0, ctypes.c_void_p(out[0].data_ptr()), ctypes.c_void_p(out[1].data_ptr()), ctypes.c_void_p(out[2].data_ptr()), None, 0, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
torch.cuda.synchronize()
ne = (out[0] != r1)
print("raw normal mismatch", ne.float().mean().item(), (out[0]-r1).abs().max().item())
print(r1[:4].tolist(), out[0][:4].tolist())
