// dadmm_hyper_tail.hip — the decoder tail of the training-mode GNN hypernetwork in one launch each
// way (gnn_dlasso_models_progressive.py:93-123 decoder blocks 2 and 3, fc and the head, :165-196).
//
// At training batch sizes (B = 256) these stages are ten small launches per iteration, each a
// latency-bound GEMM or row pass of a few microseconds. Here one workgroup owns 16 samples (one MFMA
// row block) and runs them all, its operands in LDS between stages:
//   forward : block 2 (Linear -> Dropout -> LayerNorm -> LeakyReLU), block 3 (same), fc + head
//             (the logits saved): dadmm_hyper_linear_ln_train x 2 + dadmm_hyper_head_train;
//   backward: fc's input gradient, block 3's LayerNorm backward (its dZ and affine partial sums to
//             the deferred-gradient block), its input gradient, block 2's likewise, and block 1's
//             output gradient: dadmm_hyper_linear + (dadmm_hyper_rownorm_bwd + dadmm_hyper_linear) x 2.
// Every value is the separate kernels' bit for bit: the GEMMs run linear_kernel's MFMA chains (per
// 16-wide k-step t, the four v_mfma_f32_16x16x4_f32 with lane (j, h) feeding k = 16 t + 4 h + r, the
// last K mod 16 columns as one zero-padded step; unsplit: the caller checks that the separate path
// would not split K either), the row passes rownorm_kernel's and rownorm_bwd_kernel's lane mapping,
// sums and 8-row partial blocks.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "dadmm_internal.h"

namespace dadmm {
namespace tail {

typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int RT = 16;                     // samples per workgroup
constexpr int WAVES = 8;
constexpr int THREADS = 64 * WAVES;

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// out[16][N] (LDS, row stride ldo) = X[16][K] (LDS, row stride ldx) W^T, W [N][K] (row stride K):
// the column blocks of 16 dealt to the waves; W loaded whole per block (K <= 16 WALL) or through a
// 4-deep register ring
constexpr int WALL = 32;
__device__ void gemm16(const float* X, int ldx, const float* __restrict__ W, int K, int N, float* out, int ldo) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int j = lane & 15, h = lane >> 4;
    const int KF = K / 16;
    const f32x4 z4 = {0.0f, 0.0f, 0.0f, 0.0f};
    for (int cb = w; 16 * cb < N; cb += WAVES) {
        const int col = 16 * cb + j;
        const float* wrow = W + (size_t)(col < N ? col : N - 1) * K + 4 * h;
        const float* xrow = X + j * ldx + 4 * h;
        f32x4 acc = z4, wr[4];
        if (KF <= WALL) {
            // the column block's whole W row segment in flight at once (one memory wait per block:
            // with 16 rows per workgroup the chains are short, the round trips were the time)
            f32x4 wall[WALL];
#pragma unroll
            for (int t = 0; t < WALL; ++t)
                if (t < KF) wall[t] = *(const f32x4*)(wrow + 16 * t);
#pragma unroll
            for (int t = 0; t < WALL; ++t)
                if (t < KF) {
                    const f32x4 xa = *(const f32x4*)(xrow + 16 * t);
#pragma unroll
                    for (int r = 0; r < 4; ++r) acc = mfma4(xa[r], wall[t][r], acc);
                }
        } else {
#pragma unroll
        for (int u = 0; u < 4; ++u) wr[u] = u < KF ? *(const f32x4*)(wrow + 16 * u) : z4;
        for (int t0 = 0; t0 < KF; t0 += 4) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int t = t0 + u;
                if (t < KF) {
                    const f32x4 xa = *(const f32x4*)(xrow + 16 * t);
                    const f32x4 wv = wr[u];
                    if (t + 4 < KF) wr[u] = *(const f32x4*)(wrow + 16 * (t + 4));
#pragma unroll
                    for (int r = 0; r < 4; ++r) acc = mfma4(xa[r], wv[r], acc);
                }
            }
        }
        }
        if (K & 15) {   // the last K mod 16 columns: lanes past K feed zeros
            const bool kin = 16 * KF + 4 * h < K;
            const f32x4 xa = kin ? *(const f32x4*)(xrow + 16 * KF) : z4;
            const f32x4 wv = kin ? *(const f32x4*)(wrow + 16 * KF) : z4;
#pragma unroll
            for (int r = 0; r < 4; ++r) acc = mfma4(xa[r], wv[r], acc);
        }
        if (col < N) {   // (+ 0: linear_kernel's epilogue adds its absent bias as 0, -0 -> +0)
#pragma unroll
            for (int r = 0; r < 4; ++r) out[(4 * h + r) * ldo + col] = acc[r] + 0.0f;
        }
    }
}

// LayerNorm rows in place (rownorm_kernel's lane mapping and sums): v = x + bias, Dropout (site,
// global row), xd saved, LayerNorm, LeakyReLU; the result to LDS (the next stage's input) and y
// CHMAX: 256-column chunks per lane (C <= 256 CHMAX; the kernels are instantiated for 1, 2, 4, 8)
template <int CHMAX>
__device__ void ln_rows(float* T, int ldt, int C, int r0, int rows_t, const float* __restrict__ bias,
                        const float* __restrict__ wln, const float* __restrict__ bln, float eps, float slope,
                        float drop_p, uint64_t seed, int site, float* xd, float* y) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int C4 = C / 4, CH = (C4 + 63) / 64;
    const f32x4 z4 = {0.0f, 0.0f, 0.0f, 0.0f};
    const uint32_t thr = drop_threshold(drop_p);
    const float scale = drop_p > 0.0f ? 1.0f / (1.0f - drop_p) : 1.0f;
    for (int lr = w; lr < rows_t; lr += WAVES) {
        const int row = r0 + lr;
        float* x = T + lr * ldt;
        f32x4 v[CHMAX];
        float s = 0.0f;
#pragma unroll
        for (int u = 0; u < CHMAX; ++u) {
            if (u >= CH) break;
            const int c4 = lane + 64 * u;
            v[u] = c4 < C4 ? *(const f32x4*)(x + 4 * c4) : z4;
            if (c4 < C4) {
                v[u] += *(const f32x4*)(bias + 4 * c4);
                if (drop_p > 0.0f) {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        v[u][e] = drop_hash(seed, site, (uint32_t)row, (uint32_t)(4 * c4 + e)) >= thr ? v[u][e] * scale
                                                                                                   : 0.0f;
                }
                *(f32x4*)(xd + (size_t)row * C + 4 * c4) = v[u];
            }
            s += (v[u][0] + v[u][1]) + (v[u][2] + v[u][3]);
        }
        s = ln_row_sum(s);
        const float mean = s / (float)C;
        float q = 0.0f;
#pragma unroll
        for (int u = 0; u < CHMAX; ++u) {
            if (u >= CH) break;
            const int c4 = lane + 64 * u;
            if (c4 < C4) {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float d = v[u][e] - mean;
                    q += d * d;
                }
            }
        }
        q = ln_row_sum(q);
        const float rstd = 1.0f / sqrtf(q / (float)C + eps);
#pragma unroll
        for (int u = 0; u < CHMAX; ++u) {
            if (u >= CH) break;
            const int c4 = lane + 64 * u;
            if (c4 >= C4) continue;
            const f32x4 wv = *(const f32x4*)(wln + 4 * c4);
            const f32x4 bv = *(const f32x4*)(bln + 4 * c4);
            f32x4 o;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float t = (v[u][e] - mean) * rstd * wv[e] + bv[e];
                t = t > 0.0f ? t : t * slope;
                o[e] = t;
            }
            *(f32x4*)(x + 4 * c4) = o;
            *(f32x4*)(y + (size_t)row * C + 4 * c4) = o;
        }
    }
}

// LayerNorm (+ LeakyReLU) backward of the tile's rows in place (rownorm_bwd_kernel's mapping: 8-row
// partial blocks, 4 waves x 2 rows each, lane columns c4 = lane + 64 u; the two blocks of the tile
// on waves 0-3 and 4-7): G holds dy, gets dx (through the Dropout), also written to dv; the
// affine partial sums of each 8-row block to part [block][2][C] (the 4 waves added in wave order)
template <int CHMAX>
__device__ void ln_bwd_rows(float* G, int ldg, int C, int r0, int rows_t, int B, const float* __restrict__ xd,
                            const float* __restrict__ wln, const float* __restrict__ bln, float eps, float slope,
                            float drop_p, uint64_t seed, int site, float* dv, float* part, float* red) {
    constexpr int RPW = ROWNORM_BWD_ROWS / 4;
    static_assert(RPW == 2 && RT == 2 * ROWNORM_BWD_ROWS && WAVES == 8, "tile = two partial blocks");
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int blk = w >> 2, wq = w & 3;
    const int C4 = C / 4, CH = (C4 + 63) / 64;
    const f32x4 z4 = {0.0f, 0.0f, 0.0f, 0.0f};
    const uint32_t thr = drop_threshold(drop_p);
    const float scale = drop_p > 0.0f ? 1.0f / (1.0f - drop_p) : 1.0f;
    const float invC = 1.0f / (float)C;
    f32x4 pw[CHMAX], pb[CHMAX], wv[CHMAX], bv[CHMAX];
    bool cok[CHMAX];
#pragma unroll
    for (int u = 0; u < CHMAX; ++u) {
        if (u >= CH) break;
        const int c4 = lane + 64 * u;
        cok[u] = c4 < C4;
        const int cc = cok[u] ? c4 : C4 - 1;
        pw[u] = pb[u] = z4;
        wv[u] = *(const f32x4*)(wln + 4 * cc);
        bv[u] = *(const f32x4*)(bln + 4 * cc);
    }
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
        const int lr = blk * ROWNORM_BWD_ROWS + wq * RPW + i;
        if (lr >= rows_t) break;
        const int row = r0 + lr;
        f32x4 v[CHMAX], g[CHMAX], dr[CHMAX];
        float s = 0.0f;
#pragma unroll
        for (int u = 0; u < CHMAX; ++u) {
            if (u >= CH) break;
            const int cc = cok[u] ? lane + 64 * u : C4 - 1;
            const f32x4 xr = *(const f32x4*)(xd + (size_t)row * C + 4 * cc);
            dr[u] = *(const f32x4*)(G + lr * ldg + 4 * cc);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[u][e] = cok[u] ? xr[e] : 0.0f;
            s += (v[u][0] + v[u][1]) + (v[u][2] + v[u][3]);
        }
        s = ln_row_sum(s);
        const float mean = s * invC;
        float q = 0.0f;
#pragma unroll
        for (int u = 0; u < CHMAX; ++u) {
            if (u >= CH) break;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float d = v[u][e] - mean;
                const float dd = d * d;
                q = cok[u] ? q + dd : q;
            }
        }
        q = ln_row_sum(q);
        const float rstd = 1.0f / sqrtf(q * invC + eps);
        float s1 = 0.0f, s2 = 0.0f;
#pragma unroll
        for (int u = 0; u < CHMAX; ++u) {
            if (u >= CH) break;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float xh = (v[u][e] - mean) * rstd;
                float dt = dr[u][e];
                const float t = xh * wv[u][e] + bv[u][e];
                dt = t > 0.0f ? dt : dt * slope;
                const float dxh = dt * wv[u][e];
                if (cok[u]) {
                    pw[u][e] += dt * xh;
                    pb[u][e] += dt;
                    s1 += dxh;
                    s2 += dxh * xh;
                }
                v[u][e] = xh;
                g[u][e] = dxh;
            }
        }
        s1 = ln_row_sum(s1);
        s2 = ln_row_sum(s2);
        const float m1 = s1 * invC, m2 = s2 * invC;
#pragma unroll
        for (int u = 0; u < CHMAX; ++u) {
            if (u >= CH) break;
            const int c4 = lane + 64 * u;
            if (!cok[u]) continue;
            f32x4 o;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float d = rstd * (g[u][e] - m1 - v[u][e] * m2);
                if (drop_p > 0.0f)
                    d = drop_hash(seed, site, (uint32_t)row, (uint32_t)(4 * c4 + e)) >= thr ? d * scale : 0.0f;
                o[e] = d;
            }
            *(f32x4*)(G + lr * ldg + 4 * c4) = o;
            *(f32x4*)(dv + (size_t)row * C + 4 * c4) = o;
        }
    }
#pragma unroll
    for (int u = 0; u < CHMAX; ++u) {
        if (u >= CH) break;
        const int c4 = lane + 64 * u;
        if (c4 < C4) {
            *(f32x4*)(red + ((size_t)w * 2 + 0) * C + 4 * c4) = pw[u];
            *(f32x4*)(red + ((size_t)w * 2 + 1) * C + 4 * c4) = pb[u];
        }
    }
    __syncthreads();
    // per 8-row block: the 4 waves' column partials in wave order (blocks past B are not written)
    for (int b2 = 0; b2 < 2; ++b2) {
        if (r0 + b2 * ROWNORM_BWD_ROWS >= B) break;
        float* pt = part + (size_t)(r0 / ROWNORM_BWD_ROWS + b2) * 2 * C;
        const float* rb = red + (size_t)(4 * b2) * 2 * C;
        for (int i = threadIdx.x; i < 2 * C; i += THREADS) {
            const int k = i / C, c = i - k * C;
            pt[i] = ((rb[(0 * 2 + k) * C + c] + rb[(1 * 2 + k) * C + c]) + rb[(2 * 2 + k) * C + c]) +
                    rb[(3 * 2 + k) * C + c];
        }
    }
}

__device__ __forceinline__ int ldp(int c) { return c + 4; }   // LDS row stride of a [16][c] tile

template <int CHMAX>
__global__ __launch_bounds__(THREADS) void tail_fwd_kernel(TailArgs a) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int r0 = blockIdx.x * RT;
    const int rows_t = a.B - r0 < RT ? a.B - r0 : RT;
    const int D0 = a.D[0], D1 = a.D[1], D2 = a.D[2], H4 = 4 * a.H;
    float* X0 = lds;
    float* Y1 = X0 + RT * ldp(D0);
    float* Y2 = Y1 + RT * ldp(D1);
    float* Z = Y2 + RT * ldp(D2);
    for (int i = threadIdx.x; i < RT * (D0 / 4); i += THREADS) {
        const int r = i / (D0 / 4), c4 = i - r * (D0 / 4);
        *(f32x4*)(X0 + r * ldp(D0) + 4 * c4) =
            r < rows_t ? *(const f32x4*)(a.x0 + (size_t)(r0 + r) * D0 + 4 * c4) : (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
    }
    __syncthreads();
    gemm16(X0, ldp(D0), a.W[0], D0, D1, Y1, ldp(D1));
    __syncthreads();
    ln_rows<CHMAX>(Y1, ldp(D1), D1, r0, rows_t, a.bias[0], a.lnw[0], a.lnb[0], a.eps[0], a.slope[0], a.drop[0], a.seed,
            a.site0, a.xd[0], a.y[0]);
    if (rows_t < RT)   // rows past B: zeros for the next GEMM (their results are never stored)
        for (int i = threadIdx.x; i < (RT - rows_t) * ldp(D1); i += THREADS) Y1[rows_t * ldp(D1) + i] = 0.0f;
    __syncthreads();
    gemm16(Y1, ldp(D1), a.W[1], D1, D2, Y2, ldp(D2));
    __syncthreads();
    ln_rows<CHMAX>(Y2, ldp(D2), D2, r0, rows_t, a.bias[1], a.lnw[1], a.lnb[1], a.eps[1], a.slope[1], a.drop[1], a.seed,
            a.site0 + 1, a.xd[1], a.y[1]);
    if (rows_t < RT)
        for (int i = threadIdx.x; i < (RT - rows_t) * ldp(D2); i += THREADS) Y2[rows_t * ldp(D2) + i] = 0.0f;
    __syncthreads();
    gemm16(Y2, ldp(D2), a.W[2], D2, H4, Z, ldp(H4));
    __syncthreads();
    // fc bias, the logits saved, the head (linear_kernel's HYPER_EPI_HEAD)
    for (int i = threadIdx.x; i < rows_t * H4; i += THREADS) {
        const int r = i / H4, col = i - r * H4;
        float v = Z[r * ldp(H4) + col] + a.bias[2][col];
        const size_t o = (size_t)(r0 + r) * H4 + col;
        a.z[o] = v;
        const int ch = col / a.H;
        v = 1.0f / (1.0f + expf(-v));                  // torch.sigmoid  (:170)
        v = fminf(fmaxf(v, 1e-4f), 0.9999f);          // clamp          (:171)
        v = v * a.maxv[ch];                           // * *_max        (:180-189)
        if (ch > 0) v = fminf(v, 0.9999f);            // tau/rho/eta    (:194-196)
        a.hyp[o] = v;
    }
}

template <int CHMAX>
__global__ __launch_bounds__(THREADS) void tail_bwd_kernel(TailArgs a) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int r0 = blockIdx.x * RT;
    const int rows_t = a.B - r0 < RT ? a.B - r0 : RT;
    const int D0 = a.D[0], D1 = a.D[1], D2 = a.D[2], H4 = 4 * a.H;
    float* DZ = lds;
    float* G2 = DZ + RT * ldp(H4);
    float* G1 = G2 + RT * ldp(D2);
    float* G0 = G1 + RT * ldp(D1);
    float* red = G0 + RT * ldp(D0);   // [8 waves][2][max(D1, D2)]
    for (int i = threadIdx.x; i < RT * (H4 / 4); i += THREADS) {
        const int r = i / (H4 / 4), c4 = i - r * (H4 / 4);
        *(f32x4*)(DZ + r * ldp(H4) + 4 * c4) =
            r < rows_t ? *(const f32x4*)(a.dz + (size_t)(r0 + r) * H4 + 4 * c4) : (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
    }
    __syncthreads();
    gemm16(DZ, ldp(H4), a.Wt[2], H4, D2, G2, ldp(D2));                 // d dec_y[2] = dz fc
    __syncthreads();
    ln_bwd_rows<CHMAX>(G2, ldp(D2), D2, r0, rows_t, a.B, a.xd[1], a.lnw[1], a.lnb[1], a.eps[1], a.slope[1], a.drop[1],
                a.seed, a.site0 + 1, a.dv[1], a.part[1], red);
    if (rows_t < RT)
        for (int i = threadIdx.x; i < (RT - rows_t) * ldp(D2); i += THREADS) G2[rows_t * ldp(D2) + i] = 0.0f;
    __syncthreads();
    gemm16(G2, ldp(D2), a.Wt[1], D2, D1, G1, ldp(D1));                 // d dec_y[1]
    __syncthreads();
    ln_bwd_rows<CHMAX>(G1, ldp(D1), D1, r0, rows_t, a.B, a.xd[0], a.lnw[0], a.lnb[0], a.eps[0], a.slope[0], a.drop[0],
                a.seed, a.site0, a.dv[0], a.part[0], red);
    if (rows_t < RT)
        for (int i = threadIdx.x; i < (RT - rows_t) * ldp(D1); i += THREADS) G1[rows_t * ldp(D1) + i] = 0.0f;
    __syncthreads();
    gemm16(G1, ldp(D1), a.Wt[0], D1, D0, G0, ldp(D0));                 // d dec_y[0]
    __syncthreads();
    for (int i = threadIdx.x; i < rows_t * (D0 / 4); i += THREADS) {
        const int r = i / (D0 / 4), c4 = i - r * (D0 / 4);
        *(f32x4*)(a.dx0 + (size_t)(r0 + r) * D0 + 4 * c4) = *(const f32x4*)(G0 + r * ldp(D0) + 4 * c4);
    }
}

}  // namespace tail

size_t tail_lds_bytes(const TailArgs& a, bool bwd) {
    const int D0 = a.D[0], D1 = a.D[1], D2 = a.D[2], H4 = 4 * a.H;
    size_t f = (size_t)tail::RT * ((D0 + 4) + (D1 + 4) + (D2 + 4) + (H4 + 4));
    if (bwd) f += (size_t)tail::WAVES * 2 * (D1 > D2 ? D1 : D2);
    return 4 * f;
}

hipError_t launch_tail(const TailArgs& a, bool bwd, hipStream_t st) {
    if (a.B <= 0) return hipSuccess;
    const size_t lds = tail_lds_bytes(a, bwd);
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    const int cmax = (a.D[1] > a.D[2] ? a.D[1] : a.D[2]) / 4;   // LayerNorm widths, in quads
    const int ch = cmax <= 64 ? 1 : cmax <= 128 ? 2 : cmax <= 256 ? 4 : 8;
    const dim3 g((a.B + tail::RT - 1) / tail::RT), b(tail::THREADS);
    auto go = [&](auto chc) -> hipError_t {
        constexpr int CH = decltype(chc)::value;
        const void* f = bwd ? (const void*)tail::tail_bwd_kernel<CH> : (const void*)tail::tail_fwd_kernel<CH>;
        if (lds > 64 * 1024) {
            hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (e != hipSuccess) return e;
        }
        if (bwd)
            hipLaunchKernelGGL(tail::tail_bwd_kernel<CH>, g, b, lds, st, a);
        else
            hipLaunchKernelGGL(tail::tail_fwd_kernel<CH>, g, b, lds, st, a);
        return hipGetLastError();
    };
    switch (ch) {
        case 1: return go(std::integral_constant<int, 1>{});
        case 2: return go(std::integral_constant<int, 2>{});
        case 4: return go(std::integral_constant<int, 4>{});
        default: return go(std::integral_constant<int, 8>{});
    }
}

}  // namespace dadmm
