"""Which Box-Muller rounding variant reproduces torch.randn on this device? (diagnostic)"""
import ctypes, os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
L = ctypes.CDLL(os.path.join(ROOT, "tests", "hip", "libprobe_rng.so"))
L.probe_rng.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int64, ctypes.c_void_p]
cuda = torch.device("cuda:0")
props = torch.cuda.get_device_properties(cuda)
T = props.multi_processor_count * (props.max_threads_per_multi_processor // 256) * 256
numel = 4 * T
torch.manual_seed(4321)
gen = torch.cuda.default_generators[0]
seed, off = gen.initial_seed(), gen.get_offset()
ref = torch.randn(numel, device=cuda)
out = torch.empty(16 * numel, device=cuda)
torch.cuda.synchronize()
assert L.probe_rng(seed, off, T, out.data_ptr()) == 0
out = out.view(16, numel)
for v in range(16):
    mm = (out[v] != ref).float().mean().item()
    print(f"variant {v:2d} (fma_uv={v&1} fast_log={(v>>1)&1} approx_sqrt={(v>>2)&1} accurate_sincos={(v>>3)&1}): mismatch {mm:.6f}")
print("T", T, "SMs", props.multi_processor_count, "threads/SM", props.max_threads_per_multi_processor)
