// mfma_feed_probe.hip — f32 32x32x2 MFMA fed by global loads, the wgrad2 pattern: per step every
// lane loads LW consecutive floats of an A row and of a B row (LW = 1, 2, 4), a ring of RING steps
// in flight, and the wave issues 4 * LW / ... MFMAs per step on 2 LW x 2 LW accumulators... see
// below. Operands stream from a buffer that fits in L2 per XCD (rows reused across waves) or from
// HBM (BIG). Printed: TFLOP/s, fraction of 157.3.
//   hipcc --offload-arch=gfx950 -O3 -o scripts/hip/mfma_feed_probe scripts/hip/mfma_feed_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// LW = 1: lane (i, kh) loads A[row][c0 + i], A[row][c0 + 32 + i] and the same of B (4 dword loads),
//         2 x 2 accumulators (the wgrad2 kernel's step).
// LW = 2: lane loads A[row][c0 + 2i .. 2i+1] and B likewise (2 dwordx2 loads), 2 x 2 accumulators.
template <int LW, int RING>
__global__ __launch_bounds__(256) void feed(const float* __restrict__ A, const float* __restrict__ B, int ld,
                                            int rows, int steps, float* out) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, i = lane & 31, kh = lane >> 5;
    const int wave = blockIdx.x * 4 + w;
    // "L2": every wave walks the same few thousand rows (shared); "HBM": each wave its own range
    const size_t start = rows >= (1 << 22) ? ((size_t)wave * steps * 2) % (size_t)rows : (size_t)(wave * 2) % rows;
    const float* pa = A + start * ld;
    const float* pb = B + start * ld;
    f32x16 acc[2][2];
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[x][y][e] = 0.0f;
    float ra[RING][2], rb[RING][2];
    int r = kh;
    auto load = [&](int u) {
        const size_t off = (size_t)r * ld;   // r: row offset from the wave's start
        if constexpr (LW == 1) {
            ra[u][0] = pa[off + i];
            ra[u][1] = pa[off + 32 + i];
            rb[u][0] = pb[off + i];
            rb[u][1] = pb[off + 32 + i];
        } else {
            const f32x2 va = *(const f32x2*)(pa + off + 2 * i), vb = *(const f32x2*)(pb + off + 2 * i);
            ra[u][0] = va.x;
            ra[u][1] = va.y;
            rb[u][0] = vb.x;
            rb[u][1] = vb.y;
        }
        r += 2;
        if (rows < (1 << 22) && r >= rows) r -= rows;
    };
#pragma unroll
    for (int u = 0; u < RING; ++u) {
        load(u);
        __builtin_amdgcn_sched_barrier(0);
    }
    for (int s = 0; s < steps; s += RING) {
#pragma unroll
        for (int u = 0; u < RING; ++u) {
#pragma unroll
            for (int x = 0; x < 2; ++x)
#pragma unroll
                for (int y = 0; y < 2; ++y)
                    acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x2f32(ra[u][x], rb[u][y], acc[x][y], 0, 0, 0);
            load(u);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    float t = 0.0f;
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) t += acc[x][y][0] + acc[x][y][15];
    out[blockIdx.x * 256 + threadIdx.x] = t;
}

template <int LW, int RING>
static void run(const float* A, const float* B, int ld, int rows, float* out, int wps, const char* what) {
    const int blocks = 256 * wps, steps = 2048;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL((feed<LW, RING>), dim3(blocks), dim3(256), 0, 0, A, B, ld, rows, steps, out);
    hipEventRecord(e0);
    hipLaunchKernelGGL((feed<LW, RING>), dim3(blocks), dim3(256), 0, 0, A, B, ld, rows, steps, out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0.0f;
    hipEventElapsedTime(&ms, e0, e1);
    const double flops = 2.0 * 32 * 32 * 2 * 4.0 * steps * blocks * 4;
    const double tf = flops / (ms * 1e-3) / 1e12;
    printf("{\"load_width\": %d, \"ring\": %d, \"waves_per_simd\": %d, \"rows\": \"%s\", \"ms\": %.3f, \"tflops\": %.1f, \"frac\": %.3f}\n",
           LW, RING, wps, what, ms, tf, tf / 157.3);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
}

int main() {
    const int ld = 64;                    // 256-byte rows
    float *A, *B, *out;
    const size_t big = (size_t)16 << 20;  // rows for the HBM case: 16M x 256 B = 4 GB per operand
    if (hipMalloc(&A, big * ld * 4) != hipSuccess || hipMalloc(&B, big * ld * 4) != hipSuccess ||
        hipMalloc(&out, 256 * 256 * 4 * 4) != hipSuccess)
        return 1;
    hipMemset(A, 0, big * ld * 4);
    hipMemset(B, 0, big * ld * 4);
    for (int wps : {1, 2, 3}) {
        run<1, 8>(A, B, ld, 4096, out, wps, "L2");
        run<2, 8>(A, B, ld, 4096, out, wps, "L2");
        run<1, 16>(A, B, ld, 4096, out, wps, "L2");
        run<2, 16>(A, B, ld, 4096, out, wps, "L2");
        run<1, 8>(A, B, ld, (int)big, out, wps, "HBM");
        run<2, 8>(A, B, ld, (int)big, out, wps, "HBM");
        run<1, 16>(A, B, ld, (int)big, out, wps, "HBM");
    }
    hipFree(A);
    hipFree(B);
    hipFree(out);
    return 0;
}
