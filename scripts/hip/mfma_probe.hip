// mfma_probe.hip — f32 MFMA accumulation-chain throughput on gfx950, operands in registers.
//
// Each wave runs ITERS steps of NACC independent accumulators (one MFMA per accumulator per step,
// the same A/B registers), so a step is NACC back-to-back MFMAs whose results the next step reads
// as SrcC. The grid puts WPS waves on every SIMD (256 CUs x 4 SIMDs). Printed: TFLOP/s and the
// fraction of the 157.3 TF dense fp32 peak. Question it answers: how many independent chains, at
// how many waves per SIMD, the f32 32x32x2 / 16x16x4 forms need to keep the pipe busy.
//   hipcc --offload-arch=gfx950 -O3 -o scripts/hip/mfma_probe scripts/hip/mfma_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int NACC, bool BIG>
__global__ __launch_bounds__(256) void chain(float* out, int iters, float a0) {
    const float a = a0 + threadIdx.x * 1e-7f, b = a0 - threadIdx.x * 1e-7f;
    if constexpr (BIG) {
        f32x16 acc[NACC];
#pragma unroll
        for (int i = 0; i < NACC; ++i)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][e] = 0.0f;
        for (int it = 0; it < iters; ++it) {
#pragma unroll
            for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[i], 0, 0, 0);
        }
        float s = 0.0f;
#pragma unroll
        for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][15];
        out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    } else {
        f32x4 acc[NACC];
#pragma unroll
        for (int i = 0; i < NACC; ++i) acc[i] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
        for (int it = 0; it < iters; ++it) {
#pragma unroll
            for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
        }
        float s = 0.0f;
#pragma unroll
        for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][3];
        out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    }
}

template <int NACC, bool BIG>
static void run(float* out, int wps) {
    // 256-thread blocks = 4 waves = one per SIMD; wps blocks per CU
    const int blocks = 256 * wps, iters = BIG ? 4096 / NACC * 4 : 8192 / NACC * 4;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL((chain<NACC, BIG>), dim3(blocks), dim3(256), 0, 0, out, iters, 1.0f);   // warm
    hipEventRecord(e0);
    hipLaunchKernelGGL((chain<NACC, BIG>), dim3(blocks), dim3(256), 0, 0, out, iters, 1.0f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0.0f;
    hipEventElapsedTime(&ms, e0, e1);
    const double flop_per_mfma = BIG ? 2.0 * 32 * 32 * 2 : 2.0 * 16 * 16 * 4;
    const double flops = flop_per_mfma * (double)iters * NACC * blocks * 4;   // 4 waves per block
    const double tf = flops / (ms * 1e-3) / 1e12;
    printf("{\"mfma\": \"%s\", \"chains\": %d, \"waves_per_simd\": %d, \"ms\": %.4f, \"tflops\": %.1f, \"frac\": %.3f}\n",
           BIG ? "32x32x2f32" : "16x16x4f32", NACC, wps, ms, tf, tf / 157.3);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
}

int main() {
    float* out;
    if (hipMalloc(&out, sizeof(float) * 256 * 256 * 8) != hipSuccess) return 1;
    for (int wps : {1, 2, 3, 4}) {
        run<1, true>(out, wps);
        run<2, true>(out, wps);
        run<4, true>(out, wps);
        run<1, false>(out, wps);
        run<2, false>(out, wps);
        run<4, false>(out, wps);
        run<8, false>(out, wps);
    }
    hipFree(out);
    return 0;
}
