// dadmm_loss.hip — the drivers' loss on the iterates and its gradient, fused.
//
// Reference: gnn_dlasso_utils.compute_loss (gnn_dlasso_utils.py:27-88):
//   losses[k] = (1/P) sum_p mean_{b,c} (Y[k,b,p,c] - label[b,c])^2
//   (loss_mean, loss_final) = (mean_k losses + 1e-8, losses[K-1] + 1e-8),
//   and (1, 1) if Y, the label or any loss is non-finite (:36-43, :69-71, :83-86).
// One pass over Y (per-workgroup partial sums, then a fixed-order finish: deterministic) instead
// of the reference's K*P mse_loss calls; the backward writes dL/dY in one pass:
//   dY[k] = (g_mean / K + [k == K-1] g_final) * 2 (Y[k] - label) / (B n P)   (0 on the fallback).
// Y rows may be padded (row stride n_store >= n); padding columns are ignored / get gradient 0.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dadmm_internal.h"

namespace dadmm {
namespace loss {

constexpr int THREADS = 256;
constexpr int CHUNK = 4096;   // granules (float4 or float) of one layer per workgroup

__device__ __forceinline__ bool finitef(float x) { return __builtin_isfinite(x); }

typedef float f32x4 __attribute__((ext_vector_type(4)));

// partial[k][c] = sum of (Y - label)^2 over chunk c of layer k; flags |= 1 on a non-finite Y/label.
// V = 4: float4 granules (n % 4 == 0 and n_store % 4 == 0), else V = 1. 32-bit index arithmetic
// within a layer (the launcher checks B*P*n_store < 2^31).
template <int V>
__global__ __launch_bounds__(THREADS) void partial_kernel(LossArgs a) {
    __shared__ float red[THREADS / 64];
    const uint32_t nv = (uint32_t)a.n / V, nsv = (uint32_t)a.n_store / V, P = (uint32_t)a.P;
    const uint32_t rows = (uint32_t)a.rows;
    const uint32_t total = rows * nv;                   // granules of the layer
    const uint32_t nch = (total + CHUNK - 1) / CHUNK;
    const uint32_t k = blockIdx.x / nch, c = blockIdx.x % nch;
    const float* Yk = a.Y + (size_t)k * rows * a.n_store;
    const uint32_t e0 = c * CHUNK, e1 = e0 + CHUNK < total ? e0 + CHUNK : total;
    float acc = 0.0f;
    bool bad = false;
    for (uint32_t e = e0 + threadIdx.x; e < e1; e += THREADS) {
        const uint32_t row = e / nv, col = e - row * nv;   // row = b * P + p
        if constexpr (V == 4) {
            const f32x4 y = *(const f32x4*)(Yk + ((size_t)row * nsv + col) * 4);
            const f32x4 x = *(const f32x4*)(a.label + ((size_t)(row / P) * nv + col) * 4);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                bad |= !(finitef(y[r]) && finitef(x[r]));
                const float d = y[r] - x[r];
                acc += d * d;
            }
        } else {
            const float y = Yk[(size_t)row * nsv + col];
            const float x = a.label[(size_t)(row / P) * nv + col];
            bad |= !(finitef(y) && finitef(x));
            const float d = y - x;
            acc += d * d;
        }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    if (__ballot(bad) != 0 && (threadIdx.x & 63) == 0) atomicOr((unsigned int*)a.flags, 1u);
    __syncthreads();
    if (threadIdx.x == 0) {
        float s = 0.0f;
        for (int w = 0; w < THREADS / 64; ++w) s += red[w];
        a.partial[(size_t)k * nch + c] = s;
    }
}

// losses[k]: one wave per layer sums its chunk partials (lane-strided, then a fixed shuffle tree:
// deterministic); then out = (loss_mean, loss_final) with the reference's fallback
__global__ __launch_bounds__(THREADS) void finish_kernel(LossArgs a, int nch) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const double denom = (double)a.rows * a.n;   // B * P * n
    for (int k = w; k < a.K; k += THREADS / 64) {
        double s = 0.0;
        for (int c = lane; c < nch; c += 64) s += (double)a.partial[(size_t)k * nch + c];
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o);
        if (lane == 0) a.losses[k] = (float)(s / denom);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        bool ok = (*(volatile int32_t*)a.flags & 1) == 0;
        double mean = 0.0;
        for (int k = 0; k < a.K; ++k) {
            const float v = a.losses[k];
            ok &= finitef(v);
            mean += v;
        }
        float lm = (float)(mean / a.K) + 1e-8f;
        float lf = a.losses[a.K - 1] + 1e-8f;
        if (!ok) { lm = 1.0f; lf = 1.0f; }
        if (!finitef(lm)) lm = 1.0f;
        if (!finitef(lf)) lf = 1.0f;
        a.out[0] = lm;
        a.out[1] = lf;
        a.flags[1] = ok ? 0 : 1;   // the fallback fired: the gradient is zero
    }
}

// dY = (g_mean / K + [k == K-1] g_final) * 2 (Y - label) / (B n P); 0 when the fallback fired and
// in padding columns. blockIdx = (layer k, chunk of its padded rows); V as partial_kernel.
template <int V>
__global__ __launch_bounds__(THREADS) void grad_kernel(LossArgs a, const float* gout, float* dY) {
    const uint32_t nv = (uint32_t)a.n / V, nsv = (uint32_t)a.n_store / V, P = (uint32_t)a.P;
    const uint32_t total = (uint32_t)a.rows * nsv;
    const uint32_t nch = (total + CHUNK - 1) / CHUNK;
    const uint32_t k = blockIdx.x / nch, c = blockIdx.x % nch;
    const bool fallback = a.flags[1] != 0;
    const float scale = 2.0f / (float)((double)a.rows * a.n);
    const float coef = (gout[0] / (float)a.K + (k == (uint32_t)a.K - 1 ? gout[1] : 0.0f)) * scale;
    const size_t base = (size_t)k * total * V;
    const uint32_t e0 = c * CHUNK, e1 = e0 + CHUNK < total ? e0 + CHUNK : total;
    for (uint32_t e = e0 + threadIdx.x; e < e1; e += THREADS) {
        const uint32_t row = e / nsv, col = e - row * nsv;
        if constexpr (V == 4) {
            f32x4 g = {0.0f, 0.0f, 0.0f, 0.0f};
            if (!fallback && col < nv) {
                const f32x4 y = *(const f32x4*)(a.Y + base + (size_t)e * 4);
                const f32x4 x = *(const f32x4*)(a.label + ((size_t)(row / P) * nv + col) * 4);
#pragma unroll
                for (int r = 0; r < 4; ++r) g[r] = coef * (y[r] - x[r]);
            }
            *(f32x4*)(dY + base + (size_t)e * 4) = g;
        } else {
            float g = 0.0f;
            if (!fallback && col < nv) g = coef * (a.Y[base + e] - a.label[(size_t)(row / P) * nv + col]);
            dY[base + e] = g;
        }
    }
}

}  // namespace loss

static bool vec4(const LossArgs& a) { return (a.n % 4) == 0 && (a.n_store % 4) == 0; }

size_t loss_scratch_floats(int K, int64_t rows, int n) {
    const int64_t nch = (rows * (int64_t)n + loss::CHUNK - 1) / loss::CHUNK;   // >= the V=4 count
    return (size_t)(K * nch) + 64;
}

hipError_t launch_loss(const LossArgs& a, hipStream_t st) {
    if ((int64_t)a.rows * a.n_store >= ((int64_t)1 << 31)) return hipErrorInvalidValue;
    hipError_t e = hipMemsetAsync(a.flags, 0, 2 * sizeof(int32_t), st);
    if (e != hipSuccess) return e;
    const int V = vec4(a) ? 4 : 1;
    const int64_t nch = (a.rows * (int64_t)(a.n / V) + loss::CHUNK - 1) / loss::CHUNK;
    if (V == 4)
        hipLaunchKernelGGL(loss::partial_kernel<4>, dim3((unsigned)(a.K * nch)), dim3(loss::THREADS), 0, st, a);
    else
        hipLaunchKernelGGL(loss::partial_kernel<1>, dim3((unsigned)(a.K * nch)), dim3(loss::THREADS), 0, st, a);
    hipLaunchKernelGGL(loss::finish_kernel, dim3(1), dim3(loss::THREADS), 0, st, a, (int)nch);
    return hipGetLastError();
}

hipError_t launch_loss_grad(const LossArgs& a, const float* gout, float* dY, hipStream_t st) {
    const int64_t total = (int64_t)a.rows * a.n_store;
    if (total >= ((int64_t)1 << 31)) return hipErrorInvalidValue;
    const int V = vec4(a) ? 4 : 1;
    const int64_t nch = (total / V + loss::CHUNK - 1) / loss::CHUNK;
    if (V == 4)
        hipLaunchKernelGGL(loss::grad_kernel<4>, dim3((unsigned)(a.K * nch)), dim3(loss::THREADS), 0, st,
                           a, gout, dY);
    else
        hipLaunchKernelGGL(loss::grad_kernel<1>, dim3((unsigned)(a.K * nch)), dim3(loss::THREADS), 0, st,
                           a, gout, dY);
    return hipGetLastError();
}

}  // namespace dadmm
