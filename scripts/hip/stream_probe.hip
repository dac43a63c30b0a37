// Timing probe (not product code): what HBM rate does a streaming pass with R reads and W writes of
// 16-byte lanes reach on this device? Same volume as the GNN step at configs[4]'s shard
// (51200 x 1024 floats per stream). Prints one line per (R, W, layout) with GB/s.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
typedef float f32x4 __attribute__((ext_vector_type(4)));
template <int R, int W>
__global__ __launch_bounds__(256) void probe(const f32x4* __restrict__ in, f32x4* __restrict__ out, size_t n4, int iters_per_thread) {
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * 256;
    for (int it = 0; it < iters_per_thread; ++it, i += stride) {
        if (i >= n4) return;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int r = 0; r < R; ++r) acc += in[(size_t)r * n4 + i];
#pragma unroll
        for (int w = 0; w < W; ++w) out[(size_t)w * n4 + i] = acc + (float)w;
    }
}
template <int R, int W>
void run(const f32x4* in, f32x4* out, size_t n4, int grid, int ipt) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL((probe<R, W>), dim3(grid), dim3(256), 0, 0, in, out, n4, ipt);
    hipEventRecord(a);
    const int reps = 10;
    for (int rep = 0; rep < reps; ++rep) hipLaunchKernelGGL((probe<R, W>), dim3(grid), dim3(256), 0, 0, in, out, n4, ipt);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0; hipEventElapsedTime(&ms, a, b);
    const double bytes = (double)(R + W) * n4 * 16;
    printf("R=%d W=%d grid=%d ipt=%d: %.1f us, %.0f GB/s\n", R, W, grid, ipt, ms * 1e3 / reps, bytes / (ms / reps * 1e-3) / 1e9);
}
int main() {
    const size_t n4 = (size_t)51200 * 1024 / 4;
    f32x4 *in, *out;
    if (hipMalloc(&in, 6 * n4 * 16) != hipSuccess || hipMalloc(&out, 3 * n4 * 16) != hipSuccess) return 1;
    hipMemset(in, 0, 6 * n4 * 16); hipMemset(out, 0, 3 * n4 * 16);
    for (int ipt : {1, 4}) {
        const int grid = (int)((n4 + 256 * (size_t)ipt - 1) / (256 * (size_t)ipt));
        run<1, 1>(in, out, n4, grid, ipt);
        run<2, 1>(in, out, n4, grid, ipt);
        run<5, 3>(in, out, n4, grid, ipt);
        run<6, 3>(in, out, n4, grid, ipt);
        run<4, 2>(in, out, n4, grid, ipt);
    }
    hipFree(in); hipFree(out);
    return 0;
}
