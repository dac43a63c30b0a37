// dadmm_prepare.hip — lay out the per-agent operator for the fused kernel.
//
// Replaces the reference's one-time Gram precompute (unfolded_DLASSO.py:16 via compute_Atx,
// :120-124): instead of AtA_p (n x n) the kernels consume A_p and A_p^T, zero-padded to
// [m_pad x n_pad] and [n_pad x m_pad] (m_pad = 64 * ceil(m / 64), m_pad_of()); the zero padding
// is inert in every fma chain.

#include "dadmm_internal.h"

namespace dadmm {

__global__ void prepare_kernel(const float* __restrict__ A, float* __restrict__ Apad,
                               float* __restrict__ Atpad, int P, int m, int m_pad, int n, int n_pad) {
    const size_t total = (size_t)P * m_pad * n_pad;
    for (size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
         idx += (size_t)gridDim.x * blockDim.x) {
        const int col = (int)(idx % n_pad);
        const int row = (int)((idx / n_pad) % m_pad);
        const int p = (int)(idx / ((size_t)n_pad * m_pad));
        const float v = (row < m && col < n) ? A[((size_t)p * m + row) * n + col] : 0.0f;
        Apad[idx] = v;
        Atpad[((size_t)p * n_pad + col) * m_pad + row] = v;
    }
}

hipError_t launch_prepare(const float* A, float* Apad, float* Atpad, int P, int m, int n,
                          int n_pad, hipStream_t stream) {
    const int m_pad = m_pad_of(m);
    const size_t total = (size_t)P * m_pad * n_pad;
    int grid = (int)((total + 255) / 256);
    if (grid > 4096) grid = 4096;
    hipLaunchKernelGGL(prepare_kernel, dim3(grid), dim3(256), 0, stream, A, Apad, Atpad, P, m, m_pad,
                       n, n_pad);
    return hipGetLastError();
}

}  // namespace dadmm
