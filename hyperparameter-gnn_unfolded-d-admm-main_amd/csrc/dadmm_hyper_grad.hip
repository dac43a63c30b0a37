// dadmm_hyper_grad.hip — the parameter-gradient GEMMs and reductions of the training-mode GNN
// hypernetwork (gnn_dlasso_models_progressive.py:9-72, :93-123; backward through them as the
// reference's loss_final.backward(), gnn_dlasso_progressive.py:207-214), accumulated in place:
//
//   wgrad2_kernel : G[N][K] += dZ^T X  (the weight gradient of one nn.Linear / GCNConv.lin over R
//                   rows: dZ [R][N] is the gradient of the linear's output, X [R][K] its input,
//                   optionally read as two column segments, cat(AtAy, Atb) in place), and
//                   g_bias[N] += sum_r dZ[r][n] (the bias gradient) from the same dZ reads, on
//                   v_mfma_f32_32x32x2_f32 with the R rows as the reduction dimension (below).
//                   Splits > 1 write partial tiles that reduce_kernel adds into G in split order.
//   colsum_kernel : out[g][c] += sum_r part[g][r][c] — the per-block partial sums of the BatchNorm /
//                   bias (dadmm_hyper_gcn_train_bwd) and LayerNorm (dadmm_hyper_rownorm_bwd) parameter
//                   gradients: 16 columns x 16 row slices per workgroup, slices added in order.
// Every sum runs in a fixed order: the gradients are deterministic run to run. They match torch's
// autograd (hipBLASLt) to f32 rounding of a different summation order.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "dadmm_internal.h"

namespace dadmm {
namespace hgrad {

typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int THREADS = 256;

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// XCD-aware order: consecutive tiles (the k-tiles of one n-tile, which read the same dZ columns)
// on blocks of one XCD (the dispatcher deals blocks round-robin over the 8 XCDs)
__device__ __forceinline__ int xcd_tile(int bid, int G) {
    constexpr int NX = 8;
    const int xcd = bid % NX, i = bid / NX, q = G / NX, r = G % NX;
    return xcd < r ? xcd * (q + 1) + i : r * (q + 1) + (xcd - r) * q + i;
}

// ---- wgrad on 32x32x2 MFMA with coalesced row operands (round 4, the default) -------------------
// The round-3 wgrad_kernel (16x16x4 MFMA, lanes loading one float of 16-column segments, 32 x 32
// tiles; removed, in git history) could not split the rows of the deferred batched gradients, so a 400 x 400 weight over B P K rows
// ran on 169 workgroups: the gradients took ~40 % of the B = 4096 training step. Here: 64 x 64
// output tiles, 4 waves each owning the whole tile (four 32x32 accumulators: 4096 flop per MFMA,
// 16 flop per operand byte) over interleaved row-pair steps; lane (i, kh) of a step reads row
// 2 s + kh of dZ and X at columns c0 + i and c0 + 32 + i, so each half-wave load is one contiguous
// 128-byte row segment. The rows split over S workgroups per tile (partial tiles in scratch, added
// in split order by reduce_kernel: deterministic); the four waves' partials add through LDS in a
// fixed tree. The bias column sums come from the same dZ reads (k-tile 0).
constexpr int W2_T = 64, W2_WAVES = 4, W2_RING = 8;
typedef float f32x16 __attribute__((ext_vector_type(16)));
__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

__global__ __launch_bounds__(64 * W2_WAVES) void wgrad2_kernel(WgradArgs a) {
    __shared__ float red[2][4 * 16 + 1][64];          // two waves' partial tiles (+ bias) per tree level
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int i = lane & 31, kh = lane >> 5;
    const int gn = (a.N + W2_T - 1) / W2_T, gk = (a.K + W2_T - 1) / W2_T;
    const int tl = xcd_tile(blockIdx.x, gridDim.x);
    const int kt = tl % gk, nt = (tl / gk) % gn, split = tl / (gk * gn);
    const int n0 = nt * W2_T, k0 = kt * W2_T;
    // rows in full pairs; an odd R leaves each block's last row to the tail below
    const int spb = a.R / 2;                          // row-pair steps per batch block
    const int steps = spb * a.nb;
    const int per = (steps + a.splits - 1) / a.splits;
    const int s_begin = split * per;
    const int s_end = s_begin + per < steps ? s_begin + per : steps;
    const int wv = __builtin_amdgcn_readfirstlane(w);

    // this lane's operand columns (clamped: columns past N / K compute garbage, never stored)
    int nc[2];
    const float* xs[2];
    int ldx[2];
    size_t sx[2];
#pragma unroll
    for (int b = 0; b < 2; ++b) {
        const int n = n0 + 32 * b + i;
        nc[b] = n < a.N ? n : a.N - 1;
        int k = k0 + 32 * b + i;
        k = k < a.K ? k : a.K - 1;
        if (k < a.K1) {
            xs[b] = a.x1 + k;
            ldx[b] = a.ld1;
            sx[b] = a.s1;
        } else {
            xs[b] = a.x2 + (k - a.K1);
            ldx[b] = a.ld2;
            sx[b] = a.s2;
        }
    }
    const bool do_bias = a.gbias != nullptr && kt == 0;
    f32x16 acc[2][2];
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[x][y][e] = 0.0f;
    float bsum[2] = {0.0f, 0.0f};
    auto consume = [&](const float (&za)[2], const float (&xb)[2]) {
#pragma unroll
        for (int x = 0; x < 2; ++x)
#pragma unroll
            for (int y = 0; y < 2; ++y) acc[x][y] = mfma32(za[x], xb[y], acc[x][y]);
        if (do_bias) {
            bsum[0] += za[0];
            bsum[1] += za[1];
        }
    };
    // The load cursor: the lane's four operand pointers at row 2 loc + kh of batch block bb, the
    // wave's next load step. Every load of the ring is unconditional from a valid row (the cursor
    // stays on the last step of the range once it gets there; those slots are never consumed), so
    // the compiler keeps one wait per slot instead of a full drain per step; the cursor moves by a
    // pointer add per operand, a block change (uniform branch) re-seeks.
    const float* pz[2];
    const float* px[2];
    int lbb = 0, lloc = 0, lst = 0;
    auto seek = [&](int st) {
        lst = st;
        lbb = st / spb;
        lloc = st - lbb * spb;
        const size_t r = (size_t)(2 * lloc + kh);
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            pz[b] = a.dz + (size_t)lbb * a.zs + r * a.ldz + nc[b];
            px[b] = xs[b] + (size_t)lbb * sx[b] + r * ldx[b];
        }
    };
    auto advance = [&]() {
        if (lst + W2_WAVES >= s_end) return;          // stay on the last step of the range
        lst += W2_WAVES;
        lloc += W2_WAVES;
        if (lloc >= spb) {
            seek(lst);
        } else {
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                pz[b] += (size_t)(2 * W2_WAVES) * a.ldz;
                px[b] += (size_t)(2 * W2_WAVES) * ldx[b];
            }
        }
    };
    const int first = s_begin + wv;
    if (first < s_end && spb >= W2_WAVES) {
        // Branch-free rings: the load cursor's four pointers move by a per-step delta chosen with
        // wave-uniform conditions (the next step inside the block: 8 rows; into the next block:
        // that block's first rows; past the wave's range: 0, the slot is never consumed), and every
        // full ring's eight steps are consumed unconditionally; only the last, partial ring tests
        // each step. (The per-step range / block / guard branches of the form below cost a sixth
        // of the kernel: 3.24 -> 2.7 ms at 512000 x 400 x 400.)
        float ra[W2_RING][2], rb[W2_RING][2];
        seek(first);
        // per-step pointer deltas: 8 rows on; into the next block adds (block stride - 2 spb rows)
        const long long dz_step = (long long)(2 * W2_WAVES) * a.ldz;
        const long long dz_wrapx = (long long)a.zs - 2ll * spb * a.ldz;
        long long dx_step[2], dx_wrapx[2];
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            dx_step[b] = (long long)(2 * W2_WAVES) * ldx[b];
            dx_wrapx[b] = (long long)sx[b] - 2ll * spb * ldx[b];
        }
        // CHECK: the step may be past the wave's range (the cursor then stays: delta 0). Masks
        // instead of selects, so that the compiler emits no branch.
        auto load_next = [&](int u, auto check) {
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                ra[u][b] = *pz[b];
                rb[u][b] = *px[b];
            }
            const bool wr = lloc + W2_WAVES >= spb;
            const long long mw = -(long long)wr;
            long long mv = -1ll;
            if constexpr (decltype(check)::value) mv = -(long long)(lst + W2_WAVES < s_end);
            const long long dz = (dz_step + (dz_wrapx & mw)) & mv;
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                pz[b] += dz;
                px[b] += (dx_step[b] + (dx_wrapx[b] & mw)) & mv;
            }
            const int adv = W2_WAVES & (int)mv;
            lst += adv;
            lloc += adv - (spb & (int)(mw & mv));
        };
        auto mma = [&](int u) {
#pragma unroll
            for (int x = 0; x < 2; ++x)
#pragma unroll
                for (int y = 0; y < 2; ++y) acc[x][y] = mfma32(ra[u][x], rb[u][y], acc[x][y]);
            bsum[0] += ra[u][0];   // (only read when do_bias)
            bsum[1] += ra[u][1];
        };
        const int nsteps = (s_end - first + W2_WAVES - 1) / W2_WAVES;   // this wave's steps
        const int nfull = nsteps / W2_RING;
        // load j of the wave is its step j and moves the cursor to step j + 1; ring g loads steps
        // 8 (g + 1) .. 8 (g + 1) + 7, so its loads AND moves stay inside the range (the last move
        // reaching step 8 g + 16 <= nsteps - 1) for g < (nsteps - 9) / 8: those rings run
        // unchecked, the rest (and the prologue) with the range test
        // (tests/test_wgrad_bounds.py::test_wgrad2_fast_cursor_sequence restates this)
        const int nunc = min(nsteps >= 9 ? (nsteps - 9) / W2_RING : 0, nfull);
#pragma unroll
        for (int u = 0; u < W2_RING; ++u) {
            load_next(u, std::true_type{});
            __builtin_amdgcn_sched_barrier(0);
        }
        for (int g = 0; g < nunc; ++g) {
#pragma unroll
            for (int u = 0; u < W2_RING; ++u) {
                mma(u);
                load_next(u, std::false_type{});
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        for (int g = nunc; g < nfull; ++g) {
#pragma unroll
            for (int u = 0; u < W2_RING; ++u) {
                mma(u);
                load_next(u, std::true_type{});
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        const int rem = nsteps - nfull * W2_RING;
#pragma unroll
        for (int u = 0; u < W2_RING; ++u)
            if (u < rem) mma(u);
        if (!do_bias) bsum[0] = bsum[1] = 0.0f;
    } else if (first < s_end) {
        float ra[W2_RING][2], rb[W2_RING][2];
        seek(first);
#pragma unroll
        for (int u = 0; u < W2_RING; ++u) {
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                ra[u][b] = *pz[b];
                rb[u][b] = *px[b];
            }
            advance();
            __builtin_amdgcn_sched_barrier(0);
        }
        for (int st = first; st < s_end; st += W2_WAVES * W2_RING) {
#pragma unroll
            for (int u = 0; u < W2_RING; ++u) {
                if (st + W2_WAVES * u < s_end) consume(ra[u], rb[u]);
#pragma unroll
                for (int b = 0; b < 2; ++b) {
                    ra[u][b] = *pz[b];
                    rb[u][b] = *px[b];
                }
                advance();
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    }
    // odd R: each block's last row (split 0, the waves taking blocks in turn; the kh = 1 half of
    // the step is that row again with dZ zeroed)
    if ((a.R & 1) && split == 0) {
        for (int bb = wv; bb < a.nb; bb += W2_WAVES) {
            const size_t r = (size_t)(a.R - 1);
            float za[2], xb[2];
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                za[b] = a.dz[(size_t)bb * a.zs + r * a.ldz + nc[b]];
                xb[b] = xs[b][(size_t)bb * sx[b] + r * ldx[b]];
                za[b] = kh ? 0.0f : za[b];
            }
            consume(za, xb);
        }
    }
    // bias: the wave's two row halves (lanes i and i + 32), in order
#pragma unroll
    for (int b = 0; b < 2; ++b) bsum[b] = bsum[b] + __shfl_down(bsum[b], 32);
    // lane (i, kh) carries column n0 + 32 kh + i (lanes 0..31 hold both halves' sums)
    const float b1 = __shfl(bsum[1], i);
    float bcol = kh ? b1 : bsum[0];
    // fixed pairwise tree over the waves (wave w adds wave w + half's partials)
#pragma unroll
    for (int half = W2_WAVES / 2; half >= 1; half /= 2) {
        if (w >= half && w < 2 * half) {
#pragma unroll
            for (int x = 0; x < 2; ++x)
#pragma unroll
                for (int y = 0; y < 2; ++y)
#pragma unroll
                    for (int e = 0; e < 16; ++e) red[w - half][(2 * x + y) * 16 + e][lane] = acc[x][y][e];
            red[w - half][64][lane] = bcol;
        }
        __syncthreads();
        if (w < half) {
#pragma unroll
            for (int x = 0; x < 2; ++x)
#pragma unroll
                for (int y = 0; y < 2; ++y)
#pragma unroll
                    for (int e = 0; e < 16; ++e) acc[x][y][e] += red[w][(2 * x + y) * 16 + e][lane];
            bcol += red[w][64][lane];
        }
        __syncthreads();
    }
    if (w > 0) return;
    // acc[x][y] register e: G row n0 + 32 x + (e & 3) + 8 (e >> 2) + 4 kh, column k0 + 32 y + i
    float* out = a.splits > 1 ? a.scratch + (size_t)split * a.N * a.K : a.g;
    const bool accum = a.splits == 1 && a.beta != 0;
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) {
            const int k = k0 + 32 * y + i;
            if (k >= a.K) continue;
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int n = n0 + 32 * x + (e & 3) + 8 * (e >> 2) + 4 * kh;
                if (n >= a.N) continue;
                float* o = out + (size_t)n * a.K + k;
                *o = accum ? *o + acc[x][y][e] : acc[x][y][e];
            }
        }
    if (do_bias) {
        const int n = n0 + 32 * kh + i;
        if (n < a.N) {
            if (a.splits > 1) a.scratch_bias[(size_t)split * a.N + n] = bcol;
            else a.gbias[n] = a.beta != 0 ? a.gbias[n] + bcol : bcol;
        }
    }
}

// dst[i] (+)= sum_s src[s][i], s in order
__global__ __launch_bounds__(THREADS) void reduce_kernel(const float* __restrict__ src, int splits, size_t count,
                                                         float* __restrict__ dst, int beta) {
    const size_t idx = (size_t)blockIdx.x * THREADS + threadIdx.x;
    if (idx >= count) return;
    float v = beta ? dst[idx] : 0.0f;
    float s = 0.0f;
    // eight partials' loads in flight at a time, added in split order (the sum is unchanged)
    int k = 0;
    for (; k + 8 <= splits; k += 8) {
        float p[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) p[u] = src[(size_t)(k + u) * count + idx];
#pragma unroll
        for (int u = 0; u < 8; ++u) s += p[u];
    }
    for (; k < splits; ++k) s += src[(size_t)k * count + idx];
    dst[idx] = v + s;
}

// out[g][c] (+)= sum_r part[g][r][c]. The partial rows are few columns wide and short (a few
// hundred rows), so the sum is latency-bound: each workgroup takes CS_C = 16 columns of one g and
// splits the rows over CS_S = 16 slices (slice s: rows s, s + 16, ..., 8 loads in flight), then
// adds the 16 slice sums in slice order through LDS — a fixed order, deterministic run to run.
constexpr int CS_C = 16, CS_S = THREADS / CS_C;
// bout (round 4, two-stage form for many batch blocks): workgroup (x, y) sums batch block y alone
// and writes it to bout [G][nb][C]; a second colsum over bout (R = nb) adds the blocks in order.
// The one-stage form left G x C / 16 workgroups (21 for a 100-wide BatchNorm) walking nb x R rows.
__global__ __launch_bounds__(THREADS) void colsum_kernel(const float* __restrict__ part, int G, int R, int C,
                                                         float* __restrict__ out, int beta, int nb,
                                                         size_t pstride, float* __restrict__ bout) {
    __shared__ float red[CS_S][CS_C + 1];
    const int cb = (C + CS_C - 1) / CS_C;
    const int g = blockIdx.x / cb, c0 = (blockIdx.x % cb) * CS_C;
    const int cl = threadIdx.x % CS_C, sl = threadIdx.x / CS_C;
    const int c = c0 + cl < C ? c0 + cl : C - 1;
    float s = 0.0f;
    const int b0 = bout ? (int)blockIdx.y : 0, b1 = bout ? b0 + 1 : nb;
    for (int bb = b0; bb < b1; ++bb) {   // batch blocks (deferred training gradients), in order
        const float* p = part + (size_t)bb * pstride + (size_t)g * R * C + c;
        int r = sl;
        for (; r + 7 * CS_S < R; r += 8 * CS_S) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = p[(size_t)(r + u * CS_S) * C];
#pragma unroll
            for (int u = 0; u < 8; ++u) s += v[u];
        }
        for (; r < R; r += CS_S) s += p[(size_t)r * C];
    }
    red[sl][cl] = s;
    __syncthreads();
    if (sl == 0 && c0 + cl < C) {
        float t = 0.0f;
#pragma unroll
        for (int k = 0; k < CS_S; ++k) t += red[k][cl];
        if (bout) {
            bout[((size_t)g * nb + b0) * C + c0 + cl] = t;
            return;
        }
        float* o = out + (size_t)g * C + c0 + cl;
        *o = beta ? *o + t : t;
    }
}

// out [cols][rows] = in [rows][cols], 32 x 32 tiles through LDS (the weight transposes the input
// gradient GEMM dX = dZ W reads as the K-contiguous operand of dadmm_hyper_linear)
__global__ __launch_bounds__(THREADS) void transpose_kernel(const float* __restrict__ in, int rows, int cols,
                                                            float* __restrict__ out) {
    __shared__ float t[32][33];
    const int gc = (cols + 31) / 32;
    const int r0 = (blockIdx.x / gc) * 32, c0 = (blockIdx.x % gc) * 32;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;   // 8 rows of 32 per pass
    for (int y = ty; y < 32; y += 8) {
        const int r = r0 + y, c = c0 + tx;
        if (r < rows && c < cols) t[y][tx] = in[(size_t)r * cols + c];
    }
    __syncthreads();
    for (int y = ty; y < 32; y += 8) {
        const int c = c0 + y, r = r0 + tx;
        if (r < rows && c < cols) out[(size_t)c * rows + r] = t[tx][y];
    }
}

}  // namespace hgrad

hipError_t launch_transpose(const float* in, int rows, int cols, float* out, hipStream_t st) {
    const int g = ((rows + 31) / 32) * ((cols + 31) / 32);
    hipLaunchKernelGGL(hgrad::transpose_kernel, dim3(g), dim3(hgrad::THREADS), 0, st, in, rows, cols, out);
    return hipGetLastError();
}

namespace {
// wgrad2 workgroups resident at once: 3 per CU (80 VGPRs + 64 AGPRs hold 3 waves per SIMD) x the
// current device's CU count, queried per call (256 CUs on MI355X: 768)
long w2_slots() {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
        cus = 256;
    return 3L * cus;
}
}

int wgrad_splits(int R, int N, int K) {
    // 64 x 64 tiles; rows split until ~4 workgroups per CU or each wave walks < 64 row pairs
    const long tiles = (long)((N + hgrad::W2_T - 1) / hgrad::W2_T) * ((K + hgrad::W2_T - 1) / hgrad::W2_T);
    const long steps = ((long)R + 1) / 2;
    int s = 1;
    bool short_walk = false;   // the doubling stopped on the walk length, not the grid size
    while (tiles * s * 2 <= 1024 && s < 64) {
        if (steps / (hgrad::W2_WAVES * s * 2) < 64) {
            short_walk = true;
            break;
        }
        s *= 2;
    }
    // Short walks on a small grid (the output head's and the last decoder layer's gradients
    // over B K rows: 16 and 64 workgroups whose waves walked ~100 row pairs at ~0.25 us each,
    // the ring's memory round trips exposed): split further, to >= 16 row pairs per wave
    // (28.8 -> 15.7 and 25.6 -> 15.6 us at B = 256). Grids of 224-512 workgroups measured no
    // faster or slower split.
    const long slots = w2_slots();
    if (short_walk && tiles * s <= 128) {
        long f = slots / tiles;
        const long fmax = steps / (hgrad::W2_WAVES * 16);
        f = f < fmax ? f : fmax;
        if (f > s) return (int)f;
    }
    // A grid past one round of resident workgroups (w2_slots(): 3 per CU, 80 VGPRs + 64 AGPRs hold 3
    // waves per SIMD) ran its last 16-128 workgroups as a second round (784 for a 400 x 400
    // weight, 896 for 400 x 200): such grids split to fill one round exactly instead, each
    // wave walking >= 32 row pairs. (Filling the smaller grids too, 512 -> 768 workgroups for
    // the 100 x 512 layer, measured slower: 87 vs 78 us.)
    if (tiles * s > slots) {
        long f = slots / tiles;
        const long fmax = steps / (hgrad::W2_WAVES * 32);
        f = f < fmax ? f : fmax;
        return f > 1 ? (int)f : 1;
    }
    return s;
}

hipError_t launch_wgrad(const WgradArgs& a, hipStream_t st) {
    const int tiles = ((a.N + hgrad::W2_T - 1) / hgrad::W2_T) * ((a.K + hgrad::W2_T - 1) / hgrad::W2_T);
    hipLaunchKernelGGL(hgrad::wgrad2_kernel, dim3(tiles * a.splits), dim3(64 * hgrad::W2_WAVES), 0, st, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || a.splits == 1) return e;
    const size_t cnt = (size_t)a.N * a.K;
    hipLaunchKernelGGL(hgrad::reduce_kernel, dim3((unsigned)((cnt + hgrad::THREADS - 1) / hgrad::THREADS)),
                       dim3(hgrad::THREADS), 0, st, a.scratch, a.splits, cnt, a.g, a.beta);
    e = hipGetLastError();
    if (e != hipSuccess || a.gbias == nullptr) return e;
    hipLaunchKernelGGL(hgrad::reduce_kernel, dim3((unsigned)((a.N + hgrad::THREADS - 1) / hgrad::THREADS)),
                       dim3(hgrad::THREADS), 0, st, a.scratch_bias, a.splits, (size_t)a.N, a.gbias, a.beta);
    return hipGetLastError();
}

hipError_t launch_colsum(const float* part, int G, int R, int C, float* out, int beta, hipStream_t st, int nb,
                         size_t pstride, float* bscratch) {
    const int blocks = G * ((C + hgrad::CS_C - 1) / hgrad::CS_C);
    if (bscratch && nb > 1) {
        hipLaunchKernelGGL(hgrad::colsum_kernel, dim3(blocks, nb), dim3(hgrad::THREADS), 0, st, part, G, R, C,
                           out, beta, nb, pstride, bscratch);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(hgrad::colsum_kernel, dim3(blocks), dim3(hgrad::THREADS), 0, st, (const float*)bscratch,
                           G, nb, C, out, beta, 1, (size_t)0, (float*)nullptr);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(hgrad::colsum_kernel, dim3(blocks), dim3(hgrad::THREADS), 0, st, part, G, R, C, out, beta,
                       nb, pstride, (float*)nullptr);
    return hipGetLastError();
}

}  // namespace dadmm
