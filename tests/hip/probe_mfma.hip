// probe_mfma.hip — test-only probe of v_mfma_f32_16x16x4_f32 numerics (tests/test_gpu_parity.py).
// One wave per trial computes D = A(16x4) B(4x16) + C(16x16) with the operand lane maps the
// fused kernel uses; the test compares D with a CPU fma chain over k = 0,1,2,3.
#include <hip/hip_runtime.h>
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void probe_kernel(const float* A, const float* Bm, const float* C, float* D) {
    const int t = blockIdx.x, l = threadIdx.x;
    const int i = l & 15, kk = l >> 4;
    const float a = A[t * 64 + i * 4 + kk];      // A[i][k]
    const float b = Bm[t * 64 + kk * 16 + i];    // B[k][j], j = l & 15
    f32x4 c;
    for (int r = 0; r < 4; ++r) c[r] = C[t * 256 + (4 * kk + r) * 16 + i];   // C[row][col]
    f32x4 d = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    for (int r = 0; r < 4; ++r) D[t * 256 + (4 * kk + r) * 16 + i] = d[r];
}

extern "C" int probe_mfma16x16x4(const float* A, const float* B, const float* C, float* D,
                                  int trials) {
    float *dA, *dB, *dC, *dD;
    if (hipMalloc(&dA, trials * 64 * 4) || hipMalloc(&dB, trials * 64 * 4) ||
        hipMalloc(&dC, trials * 256 * 4) || hipMalloc(&dD, trials * 256 * 4))
        return -1;
    hipMemcpy(dA, A, trials * 64 * 4, hipMemcpyHostToDevice);
    hipMemcpy(dB, B, trials * 64 * 4, hipMemcpyHostToDevice);
    hipMemcpy(dC, C, trials * 256 * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe_kernel, dim3(trials), dim3(64), 0, 0, dA, dB, dC, dD);
    hipError_t e = hipMemcpy(D, dD, trials * 256 * 4, hipMemcpyDeviceToHost);
    hipFree(dA); hipFree(dB); hipFree(dC); hipFree(dD);
    return e == hipSuccess ? 0 : -2;
}
