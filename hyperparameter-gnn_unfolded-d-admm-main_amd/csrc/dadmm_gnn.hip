// dadmm_gnn.hip — per-iteration D-ADMM kernels for the GNN-hypernetwork model
// (DLASSO_GNNHyp3_Progressive.forward, gnn_dlasso_models_progressive.py:131-243).
//
// There the hyper-parameters of iteration k come from a GNN evaluated on [A^T A y_k, A^T b], so
// the K-step loop cannot be fused: each iteration is
//   gram     AtAy_k = A^T (A y_k)            (:158-162; MFMA GEMM pair, f32 fma chains)
//   [host]   hyp_k = GNN(cat(AtAy_k, Atb))   (the HIP hypernetwork, dadmm_hyper*.hip; :165-196)
//   step     g_k = clamp(AtAy - Atb + sign(y) tau + U deg + delta rho, +-gclip)   (:205-213)
//            y_{k+1} = clamp(y - alpha g); delta_{k+1} = clamp(2 L y_{k+1}); U_{k+1} = clamp(U +
//            delta eta)                                                           (:221-232)
//            as ONE pass over the state (update_kernel<true>: g is formed in registers, never
//            stored); the reference zeroes the WHOLE batch's gradient when any g is NaN
//            (:216-218), which no workgroup can know while it updates, so the pass is optimistic
//            and a resolve launch (resolve_kernel) either commits its y_next / U guard flags
//            (no NaN: the common case, one workgroup's work) or redoes the update with g = 0.
// with the reference's batch-global NaN/Inf guards (:150-156, :216-218, :235-237) decided through
// device flag words between launches (no host synchronisation), exactly as dadmm_stepwise.hip
// does for the unfolded model. Y[k] stores y_{k+1}; a y_next guard that fired is resolved by
// every later reader (y_source), Y[k] itself is rewritten by the next iteration's grad launch,
// and Y[K-1] by dadmm_gnn_finish.
//
// Operation order (restated bit-for-bit by oracle_forward_f32 with gram_mode = 1): AtAy is one
// fma chain per row through R = A y (from +0) and A^T R (from +0), each in the fused kernel's
// 16-block order; Atb = A^T b likewise; the gradient is ((((AtAy - Atb) + sign*tau) + U*deg) +
// delta*rho), every operation rounded on its own (-ffp-contract=off).
//
// The adjoint of one iteration (dadmm_gnn_step_backward) recomputes the iteration from its
// inputs and returns the gradients w.r.t. y_k, U_k, delta_k, AtAy_k and hyp_k; the gradient
// w.r.t. y_k through AtAy_k is the caller's gram of the AtAy gradient (A^T A is symmetric).

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "dadmm_internal.h"

namespace dadmm {
namespace gnn {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int THREADS = 256;   // 4 waves
constexpr int WAVES = 4;
// Decisions (variants measured and dropped; git history holds them, DESIGN.md §4 the numbers):
// gram_kernel's GEMM1 with x staged through LDS (slower: the chunk barriers serialise the waves,
// profiles/r04/variants_r04c.txt) and a one-wave-per-item gram with R in registers (no faster,
// variants_r04d.txt) are gone. Kept: gram_kernel mode 2 prefetches the out rows one GEMM2 unit
// ahead; GEMM1's ring is 8 deep where the column steps divide and a wave's whole GEMM2 (<= 4
// units) is loaded at once (round 5); the step adjoint's per-sample hyper-parameter sums run on
// DPP moves and readlanes (wave_sum_dpp); update_item loads the guard flags and y_k's table entry
// together; gram_kernel<true> serves grids of <= 2 items per CU at m_pad = 64, n_pad = 256.

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
// torch.clamp: NaN propagates, +-inf saturate
__device__ __forceinline__ float clamp_t(float x, float lo, float hi) {
    return x != x ? x : fminf(fmaxf(x, lo), hi);
}
__device__ __forceinline__ bool inside(float x, float lo, float hi) { return x >= lo && x <= hi; }
__device__ __forceinline__ bool finitef(float x) { return __builtin_isfinite(x); }
__device__ __forceinline__ int flag_ld(const int32_t* f) {
    return __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void flag_or(int32_t* f, bool v) {
    if (__ballot(v) != 0 && (threadIdx.x & 63) == 0)
        __hip_atomic_fetch_or(f, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void clips(const GnnArgs& a, int k, float& gclip, float& vclip) {
    if (a.variant == 0) {
        gclip = fmaxf(1.0f, 30.0f - (float)k);          // unfolded_DLASSO.py:80
        vclip = fmaxf(10.0f, 200.0f - (float)(k * 3));  // unfolded_DLASSO.py:92
    } else {
        gclip = 10.0f;                                   // gnn_dlasso_models_progressive.py:212
        vclip = 100.0f;                                  // :224, :232
    }
}

// y_k as the reference holds it at the top of iteration k: y_{j+1} (yptr[j+1]) for the last
// j < k whose y_next passed its guard, else y0 — read as zeros when the k = 0 guard fired
__device__ __forceinline__ const float* y_source(const GnnArgs& a, int k, bool& zero) {
    for (int j = k - 1; j >= 0; --j)
        if (!flag_ld(a.flags + GNN_F_YNB(j))) {
            zero = false;
            return a.yptr[j + 1];
        }
    zero = flag_ld(a.flags + GNN_F_Y0) != 0;
    return a.yptr[0];
}

// hyp_k of sample s, agent p, component c (alpha, tau, rho, eta): [B][4][H] (view(B, 4, P|1))
__device__ __forceinline__ float hyp_at(const GnnArgs& a, int s, int c, int p) {
    return a.hyp[((size_t)s * 4 + c) * a.hyp_rows + (a.hyp_rows == 1 ? 0 : p)];
}

// ---- zero: the guard flag words (a kernel, not hipMemsetAsync: the inference forward is captured
// into a HIP graph, whose memset nodes were measured to replay with a corrupted fill pattern from
// the second launch on — every guard flag set, profiles/r03/gnn_graph_memset_r03.txt) ------------
__global__ __launch_bounds__(THREADS) void zero_kernel(int32_t* p, int words) {
    for (int i = blockIdx.x * THREADS + threadIdx.x; i < words; i += gridDim.x * THREADS) p[i] = 0;
}

// ---- check0: the k = 0 guards on y0 / U0 (:150-156) --------------------------------------------
__global__ __launch_bounds__(THREADS) void check0_kernel(GnnArgs a, const float* y0) {
    const size_t S4 = (size_t)a.B * a.P * a.n / 4;
    bool by = false, bu = false;
    for (size_t i = (size_t)blockIdx.x * THREADS + threadIdx.x; i < S4; i += (size_t)gridDim.x * THREADS) {
        const f32x4 y = ((const f32x4*)y0)[i];
        const f32x4 u = ((const f32x4*)a.U)[i];
        by |= !(finitef(y[0]) && finitef(y[1]) && finitef(y[2]) && finitef(y[3]));
        bu |= !(finitef(u[0]) && finitef(u[1]) && finitef(u[2]) && finitef(u[3]));
    }
    flag_or(a.flags + GNN_F_Y0, by);
    flag_or(a.flags + GNN_F_UBAD(0), bu);
}

// ---- gram: out = A^T (A x) per agent (mode 0), out = A^T b (mode 1), out += A^T (A x) (mode 2) --
// item = (16-sample tile, agent p); x is y_k resolved through the guard flags (x_raw == nullptr)
// or the raw operand x_raw (the adjoints' gradient operands).
// SMALL (gram_small: a grid of at most two items per CU, m_pad = 64, n_pad = 256, mode != 1): the
// same chains as the general form, with every operand load issued up front — the A rows, A^T rows
// and (mode 2) out rows before the guard-flag walk that names x, then all 16 column steps of x —
// so each wave waits on memory once before GEMM1 instead of once per ring refill and again for the
// A^T rows after the barrier. Bit-identical (the chains and their order are unchanged).
template <bool SMALL>
__global__ __launch_bounds__(THREADS) void gram_kernel(GnnArgs a, int k, const float* x_raw,
                                                       float* out, int mode) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int P = a.P, n = a.n, m = a.m, B = a.B, NP = a.n_pad, MP = a.m_pad;
    const int tile = blockIdx.x / P, p = blockIdx.x % P;
    const int RS = MP + 4;
    float* Rlds = lds;               // [16][RS]
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int j = lane & 15, h = lane >> 4;
    const int s = tile * BT + j;
    const bool sv = s < B;

    if constexpr (SMALL) {
        // (host: m = 64 exactly, so every wave owns one live m-block and no load sits under a branch)
        constexpr int T = 16, MB = 4;   // column steps of x (n_pad = 256), m-blocks (m_pad = 64)
        // x's source first: the guard flag of iteration k - 1 and the table entry it names, issued
        // before the operator loads so that their wait does not include them
        const bool walk_x = x_raw == nullptr;
        const bool prev = walk_x && k >= 1;
        // the flag word through a descriptor whose range is empty when there is no k - 1 (reads 0,
        // touches nothing); flags written by earlier launches are visible at this launch's start
        const __amdgpu_buffer_rsrc_t rf = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<int32_t*>(a.flags), 0, prev ? 4 * (GNN_F_YNB(k - 1) + 1) : 0, 0x00020000);
        const int f_raw = __builtin_amdgcn_raw_buffer_load_b32(rf, prev ? 4 * GNN_F_YNB(k - 1) : 0, 0, 0);
        const float* y_prev = nullptr;
        if (prev) y_prev = a.yptr[k];
        __builtin_amdgcn_sched_barrier(0);
        f32x4 ar[T], at_all[MB][4], oall[MB];
        const float* arow = a.A + ((size_t)p * 64 + 16 * w + j) * 256 + 4 * h;
#pragma unroll
        for (int u = 0; u < T; ++u) ar[u] = *(const f32x4*)(arow + 16 * u);
        // GEMM2's units: n-tiles w, w + 4, w + 8, w + 12 (one m-group)
        const float* atb = a.At + ((size_t)p * 256 + j) * 64 + 4 * h;
        const __amdgpu_buffer_rsrc_t ro =
            __builtin_amdgcn_make_buffer_rsrc(out, 0, mode == 2 ? (int)((size_t)B * P * n * 4) : 0, 0x00020000);
#pragma unroll
        for (int u = 0; u < MB; ++u) {
#pragma unroll
            for (int t = 0; t < 4; ++t) at_all[u][t] = *(const f32x4*)(atb + (size_t)16 * (w + WAVES * u) * 64 + 16 * t);
            const int n0 = 16 * (w + WAVES * u) + 4 * h;
            const uint32_t off = (sv && n0 < n) ? (uint32_t)((((size_t)s * P + p) * n + n0) * 4) : 0x80000000u;
            oall[u] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(ro, off, 0, 0));
        }
        __builtin_amdgcn_sched_barrier(0);
        bool zero = false;
        const float* xs = !walk_x ? x_raw
                        : (prev && __builtin_amdgcn_readfirstlane(f_raw) == 0) ? y_prev : y_source(a, k, zero);
        {   // wave-uniform (scalar) pointer and guard: the descriptor below must live in SGPRs
            const uint64_t xa = (uint64_t)xs;
            const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)xa);
            const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(xa >> 32));
            xs = (const float*)(((uint64_t)hi << 32) | lo);
            zero = __builtin_amdgcn_readfirstlane((int)zero) != 0;
        }
        const uint32_t xbytes = zero ? 0u : (uint32_t)((size_t)B * P * n * 4);
        const __amdgpu_buffer_rsrc_t rx =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(xs), 0, (int)xbytes, 0x00020000);
        const uint32_t xoff = sv ? (uint32_t)((((size_t)s * P + p) * n + 4 * h) * 4) : 0x80000000u;
        f32x4 xr[T];
#pragma unroll
        for (int u = 0; u < T; ++u)
            xr[u] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                rx, 16 * u + 4 * h < n && sv ? xoff + 64u * u : 0x80000000u, 0, 0));
        __builtin_amdgcn_sched_barrier(0);
        f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int u = 0; u < T; ++u)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc = mfma4(ar[u][r], xr[u][r], acc);
        *(f32x4*)(Rlds + j * RS + 16 * w + 4 * h) = acc;
        __syncthreads();
        f32x4 rv0[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) rv0[t] = *(const f32x4*)(Rlds + j * RS + 16 * t + 4 * h);
#pragma unroll
        for (int u = 0; u < MB; ++u) {
            f32x4 g = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int r = 0; r < 4; ++r) g = mfma4(at_all[u][t][r], rv0[t][r], g);
            const int n0 = 16 * (w + WAVES * u) + 4 * h;
            if (sv && n0 < n) {
                f32x4 v = mode == 2 ? oall[u] + g : g;
                if (mode == 2 && a.acc_add != nullptr) v = v + *(const f32x4*)(a.acc_add + ((size_t)s * P + p) * n + n0);
                *(f32x4*)(out + ((size_t)s * P + p) * n + n0) = v;
            }
        }
        return;
    }

    if (mode != 1) {
        bool zero = false;
        const float* xs = x_raw != nullptr ? x_raw : y_source(a, k, zero);
        // GEMM1: R = A_p x (chain from +0); wave w = m-blocks w, w + 4, .... Both operands stream
        // through a ring of GD steps (the loads of step t + GD issue after step t's MFMAs): A rows
        // from L2, the x columns (16 samples) from L2/HBM through a buffer descriptor whose range
        // check returns 0 for columns past n, samples past B and a guard-zeroed x. NP / 16 is a
        // multiple of GD.
        for (int mq = w; mq < MP / 16; mq += WAVES) {
            f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
            if (16 * mq < m) {
                const float* arow = a.A + ((size_t)p * MP + 16 * mq + j) * NP + 4 * h;
                const uint32_t xbytes = zero ? 0u : (uint32_t)((size_t)B * P * n * 4);
                const __amdgpu_buffer_rsrc_t rx =
                    __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(xs), 0, (int)xbytes, 0x00020000);
                const uint32_t xoff = sv ? (uint32_t)((((size_t)s * P + p) * n + 4 * h) * 4) : 0x80000000u;
                auto ldx = [&](int t) -> f32x4 {
                    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                        rx, 16 * t + 4 * h < n && sv ? xoff + 64u * t : 0x80000000u, 0, 0));
                };
                const int T = NP / 16;
                // ring depth 8 where the steps divide (round 5: half the exposed round trips of the
                // latency-bound small-batch grams), else 4; the chain is the same either way
                auto gemm1 = [&](auto gd) {
                    constexpr int GD = decltype(gd)::value;
                    f32x4 ar[GD], xr[GD];
#pragma unroll
                    for (int u = 0; u < GD; ++u) {
                        ar[u] = *(const f32x4*)(arow + 16 * u);
                        xr[u] = ldx(u);
                    }
                    for (int t0 = 0; t0 < T; t0 += GD) {
#pragma unroll
                        for (int u = 0; u < GD; ++u) {
#pragma unroll
                            for (int r = 0; r < 4; ++r) acc = mfma4(ar[u][r], xr[u][r], acc);
                            if (t0 + GD + u < T) {
                                ar[u] = *(const f32x4*)(arow + 16 * (t0 + GD + u));
                                xr[u] = ldx(t0 + GD + u);
                            }
                        }
                    }
                };
                if (T % 8 == 0)
                    gemm1(std::integral_constant<int, 8>{});
                else
                    gemm1(std::integral_constant<int, 4>{});
            }
            *(f32x4*)(Rlds + j * RS + 16 * mq + 4 * h) = acc;
        }
    } else {
        // R = b_p (rows past m are zero)
        for (int mq = w; mq < MP / 16; mq += WAVES) {
            f32x4 v;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int mi = 16 * mq + 4 * h + r;
                v[r] = (sv && mi < m) ? a.b[((size_t)s * P + p) * m + mi] : 0.0f;
            }
            *(f32x4*)(Rlds + j * RS + 16 * mq + 4 * h) = v;
        }
    }
    __syncthreads();
    // GEMM2: out = A_p^T R, one chain from +0 over the m-blocks in ascending order; wave w takes
    // n-tiles w, w + 4, ...; the m-blocks past m (zero rows of R and of the padded operator) are
    // skipped. Work unit u = (n-tile, m-group of 4 blocks); the A^T rows of unit u + 1 load under
    // unit u's MFMAs. R of m-group 0 is held in registers, later groups are read from LDS.
    const int mbk = (m + 15) / 16;                 // m-blocks holding rows
    const int MG = (mbk + 3) / 4;                  // m-groups holding rows
    f32x4 rv0[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) rv0[t] = *(const f32x4*)(Rlds + j * RS + 16 * t + 4 * h);
    const float* atb = a.At + ((size_t)p * NP + j) * MP + 4 * h;
    f32x4 at_cur[4], at_nxt[4];
    auto load_at = [&](f32x4 (&dst)[4], int u) {
        const int nb = w + WAVES * (u / MG), mg = u % MG;
#pragma unroll
        for (int t = 0; t < 4; ++t)
            if (4 * mg + t < mbk) dst[t] = *(const f32x4*)(atb + (size_t)16 * nb * MP + 64 * mg + 16 * t);
    };
    const int units = (NP / 16 - w + WAVES - 1) / WAVES * MG;
    if (MG == 1 && units <= 4) {
        // (round 5) every unit's A^T rows (and mode 2's out rows) loaded at once: one memory wait
        // for the wave's whole GEMM2 instead of one per unit; the chains are the loop's below
        f32x4 at_all[4][4], oall[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (u < units) {
                load_at(at_all[u], u);
                const int n0 = 16 * (w + WAVES * u) + 4 * h;
                const bool st = sv && n0 < n;
                oall[u] = (mode == 2 && st) ? *(const f32x4*)(out + ((size_t)s * P + p) * n + n0)
                                            : (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
            }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (u >= units) break;
            f32x4 g = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                if (t < mbk) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) g = mfma4(at_all[u][t][r], rv0[t][r], g);
                }
            }
            const int n0 = 16 * (w + WAVES * u) + 4 * h;
            if (sv && n0 < n) {
                f32x4 v = mode == 2 ? oall[u] + g : g;
                if (mode == 2 && a.acc_add != nullptr) v = v + *(const f32x4*)(a.acc_add + ((size_t)s * P + p) * n + n0);
                *(f32x4*)(out + ((size_t)s * P + p) * n + n0) = v;
            }
        }
        return;
    }
    if (units > 0) load_at(at_cur, 0);
    f32x4 gc = {0.0f, 0.0f, 0.0f, 0.0f};
    // mode 2 (out += ...): the out rows of the unit that completes a tile are loaded one unit
    // ahead (a load issued just before its add left the HBM latency exposed once per tile)
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
        out, 0, (mode == 2) ? (int)((size_t)B * P * n * 4) : 0, 0x00020000);
    auto ldo = [&](int u) -> f32x4 {
        const int nb = w + WAVES * (u / MG), mg = u % MG, n0 = 16 * nb + 4 * h;
        const uint32_t off = (mg == MG - 1 && sv && n0 < n) ? (uint32_t)((((size_t)s * P + p) * n + n0) * 4)
                                                           : 0x80000000u;
        return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(ro, off, 0, 0));
    };
    f32x4 ocur = {0.0f, 0.0f, 0.0f, 0.0f}, onxt = ocur;
    if (mode == 2 && units > 0) ocur = ldo(0);
    for (int u = 0; u < units; ++u) {
        const int nb = w + WAVES * (u / MG), mg = u % MG;
        if (u + 1 < units) load_at(at_nxt, u + 1);
        if (mode == 2 && u + 1 < units) onxt = ldo(u + 1);
        if (mg == 0) {
            gc = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                if (t < mbk) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) gc = mfma4(at_cur[t][r], rv0[t][r], gc);
                }
            }
        } else {
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                if (4 * mg + t < mbk) {
                    const f32x4 rt = *(const f32x4*)(Rlds + j * RS + 64 * mg + 16 * t + 4 * h);
#pragma unroll
                    for (int r = 0; r < 4; ++r) gc = mfma4(at_cur[t][r], rt[r], gc);
                }
            }
        }
        const int n0 = 16 * nb + 4 * h;
        if (mg == MG - 1 && sv && n0 < n) {
            f32x4* o = (f32x4*)(out + ((size_t)s * P + p) * n + n0);
            f32x4 v = mode == 2 ? ocur + gc : gc;
            if (mode == 2 && a.acc_add != nullptr) v = v + *(const f32x4*)(a.acc_add + ((size_t)s * P + p) * n + n0);
            *o = v;
        }
        ocur = onxt;
#pragma unroll
        for (int t = 0; t < 4; ++t) at_cur[t] = at_nxt[t];
    }
}

// ---- gram with the agent's operator resident in LDS (round 4, the default where it fits) ---------
// gram_kernel re-reads A_p and A_p^T from L2 for every (16-sample tile, agent) item and runs one
// dependent MFMA chain per wave (PMC at configs[2]: MFMA busy 0.25, waves half the time stalled on
// issue). Here a workgroup owns ONE agent and a run of tiles: A_p's rows (16 MQ x n_pad) are copied
// into LDS once (row stride n_pad + 4 floats: the GEMM2 fragment gathers, rows 4 h + r apart, land
// in 64 distinct banks) and every wave runs whole items — GEMM1 with the MQ
// m-block chains interleaved and R kept in registers (the accumulator layout is GEMM2's B operand),
// GEMM2 with two n-tiles' chains interleaved — reading both operand fragments from LDS; only the x
// and out streams touch HBM (x through a GX-deep register ring, mode 2's out rows two n-tile pairs
// ahead). 16 waves (four per SIMD) hide the stream latency. Chains and their order are
// gram_kernel's: GEMM1 from +0 over the columns in 16-blocks (0,4,8,12,1,... inside), GEMM2 from +0
// over the m-blocks ascending — bit-identical output.
constexpr int GL_WAVES = 16;
__host__ __device__ constexpr size_t gram_lds_bytes(int mq, int n_pad) { return 4 * (size_t)16 * mq * (n_pad + 4); }

template <int MQ>
__global__ __launch_bounds__(64 * GL_WAVES) void gram_lds_kernel(GnnArgs a, int k, const float* x_raw, float* out,
                                                                 int mode, int tpw) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    constexpr int GX = 4;                          // x k-steps in flight
    const int P = a.P, n = a.n, B = a.B, NP = a.n_pad, MP = a.m_pad;
    const int LS = NP + 4;
    const int p = blockIdx.x % P, grp = blockIdx.x / P;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int j = lane & 15, h = lane >> 4;
    constexpr int mbk = MQ;                        // m-blocks holding rows (the host picks MQ = ceil(m / 16))
    const int T = NP / 16;                         // 16-column steps
    const int tiles = (B + BT - 1) / BT;

    // A_p rows [0, 16 mbk) -> LDS (rows past m are the operator's zero padding)
    {
        const int q4 = NP / 4, total = 16 * mbk * q4;
        const float* src = a.A + (size_t)p * MP * NP;
        for (int i = threadIdx.x; i < total; i += 64 * GL_WAVES) {
            const int r = i / q4, c = i - r * q4;
            *(f32x4*)(lds + r * LS + 4 * c) = *(const f32x4*)(src + (size_t)r * NP + 4 * c);
        }
    }
    bool zero = false;
    const float* xs = x_raw != nullptr ? x_raw : y_source(a, k, zero);
    const uint32_t sbytes = (uint32_t)((size_t)B * P * n * 4);
    const __amdgpu_buffer_rsrc_t rx =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(xs), 0, zero ? 0 : (int)sbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(out, 0, (int)sbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t roi = __builtin_amdgcn_make_buffer_rsrc(out, 0, mode == 2 ? (int)sbytes : 0, 0x00020000);
    const bool has_add = mode == 2 && a.acc_add != nullptr;
    const __amdgpu_buffer_rsrc_t rad =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.acc_add), 0, has_add ? (int)sbytes : 0, 0x00020000);
    __syncthreads();

    const int t_end = min(tiles, (grp + 1) * tpw);
    for (int tile = grp * tpw + w; tile < t_end; tile += GL_WAVES) {
        const int s = tile * BT + j;
        const bool sv = s < B;
        const uint32_t rowoff = sv ? (uint32_t)(((size_t)s * P + p) * n * 4) : 0x80000000u;
        // GEMM1: R[g] = A_p[16 g + j, :] x, MQ chains interleaved
        f32x4 R[MQ];
#pragma unroll
        for (int g = 0; g < MQ; ++g) R[g] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
        auto ldx = [&](int t) -> f32x4 {
            const uint32_t off = (t < T && 16 * t + 4 * h < n && sv) ? rowoff + (uint32_t)(64 * t + 16 * h) : 0x80000000u;
            return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, off, 0, 0));
        };
        auto lda = [&](f32x4 (&dst)[MQ], int t) {
#pragma unroll
            for (int g = 0; g < MQ; ++g)
                dst[g] = *(const f32x4*)(lds + (16 * g + j) * LS + 16 * t + 4 * h);
        };
        f32x4 xr[GX], af[2][MQ];
#pragma unroll
        for (int u = 0; u < GX; ++u) xr[u] = ldx(u);
        lda(af[0], 0);
        for (int t0 = 0; t0 < T; t0 += GX) {
#pragma unroll
            for (int u = 0; u < GX; ++u) {
                const int t = t0 + u;
                if (t < T) {
                    if (t + 1 < T) lda(af[(u + 1) & 1], t + 1);
#pragma unroll
                    for (int r = 0; r < 4; ++r)
#pragma unroll
                        for (int g = 0; g < MQ; ++g) R[g] = mfma4(af[u & 1][g][r], xr[u][r], R[g]);
                }
                xr[u] = ldx(t + GX);
            }
        }
        // GEMM2: out rows of n-tiles nb, nb + 1 = A_p^T R, one chain per n-tile over the m-blocks
        const int NT = T;
        auto ldt = [&](f32x4 (&dst)[MQ], int nb) {
#pragma unroll
            for (int g = 0; g < MQ; ++g)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    dst[g][r] = lds[(16 * g + 4 * h + r) * LS + 16 * nb + j];
        };
        auto ldo = [&](int nb) -> f32x4 {
            const uint32_t off = (nb < NT && 16 * nb + 4 * h < n && sv) ? rowoff + (uint32_t)(64 * nb + 16 * h) : 0x80000000u;
            return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(roi, off, 0, 0));
        };
        auto ldd = [&](int nb) -> f32x4 {   // mode 2's addend rows (zeros when there is none)
            const uint32_t off = (nb < NT && 16 * nb + 4 * h < n && sv) ? rowoff + (uint32_t)(64 * nb + 16 * h) : 0x80000000u;
            return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rad, off, 0, 0));
        };
        // mode 2's out rows (and addend rows) two pairs ahead (oc: this pair, on: the next)
        f32x4 oc0 = ldo(0), oc1 = ldo(1), on0 = ldo(2), on1 = ldo(3);
        f32x4 dc0 = ldd(0), dc1 = ldd(1), dn0 = ldd(2), dn1 = ldd(3);
        for (int n0 = 0; n0 < NT; n0 += 2) {
            f32x4 at0[MQ], at1[MQ];
            ldt(at0, n0);
            ldt(at1, n0 + 1 < NT ? n0 + 1 : n0);
            f32x4 g0 = {0.0f, 0.0f, 0.0f, 0.0f}, g1 = g0;
#pragma unroll
            for (int g = 0; g < MQ; ++g)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    g0 = mfma4(at0[g][r], R[g][r], g0);
                    g1 = mfma4(at1[g][r], R[g][r], g1);
                }
            f32x4 o0 = mode == 2 ? oc0 + g0 : g0;
            f32x4 o1 = mode == 2 ? oc1 + g1 : g1;
            if (has_add) {
                o0 = o0 + dc0;
                o1 = o1 + dc1;
            }
            const uint32_t s0 = (16 * n0 + 4 * h < n && sv) ? rowoff + (uint32_t)(64 * n0 + 16 * h) : 0x80000000u;
            const uint32_t s1 = (n0 + 1 < NT && 16 * (n0 + 1) + 4 * h < n && sv)
                                    ? rowoff + (uint32_t)(64 * (n0 + 1) + 16 * h) : 0x80000000u;
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, o0), ro, s0, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, o1), ro, s1, 0, 0);
            oc0 = on0;
            oc1 = on1;
            on0 = ldo(n0 + 4);
            on1 = ldo(n0 + 5);
            dc0 = dn0;
            dc1 = dn1;
            dn0 = ldd(n0 + 4);
            dn1 = ldd(n0 + 5);
        }
    }
}

// ---- step: gradient, primal update, consensus and dual update of (sample, 128 columns) ----------
// One workgroup per (sample, UCB = 128 columns). A lane owns 4 columns of one agent row; a wave
// instruction covers two agent rows (lanes 0-31 and 32-63), so every global access is a 16-byte
// vector and a wave keeps UP_CH row pairs of loads in flight. y_{k+1} of all P agents is staged in
// LDS ([P][UCB], 25.6 KB at P = 50) next to the sample's visit lists, and the consensus reads its
// neighbours from there in the reference's visit order (one fp32 add chain per column from 0).
// update_item<FUSED> on item (sample, column block). FUSED: the gradient g = clamp(((AtAy - Atb) + sign(y) tau) + U deg + delta rho) (:205-213) is
//   formed from AtAy, Atb, y, U, delta in the same pass (its NaN sets GBAD(k)); the y_next / U
//   guard flags go to the optimistic slots. Also rewrites Y[k-1] when the previous y_next guard
//   fired (:235-237: the reference keeps y_k = y_{k-1} and appends it).
// !FUSED (resolve, launched after the fused pass): no NaN gradient -> block 0 commits the
//   optimistic flags, every block exits; else the update again with g = 0 (:216-218), writing the
//   guard flags themselves.
constexpr int UP_CH = 4;
// columns per item: 128 (a wave instruction covers 2 agent rows) or 64 (4 rows; half the LDS per
// workgroup, so more workgroups fit per CU at large P)
constexpr int UCB = 128;
constexpr int RPI = 256 / UCB;    // agent rows per wave instruction (UCB / 4 lanes per row)
static_assert(UCB == 64 || UCB == 128, "UCB");
// Keeping phase 1's U rows in registers for phase 2 (one fewer HBM stream) was measured and
// dropped: 97 instead of 82 VGPRs, four instead of five waves per SIMD, 86.1-86.4 vs 84.7-85.0 ms
// at the configs[4] shard forward (profiles/r04/variants_r04o_step_keepu.txt)
// LDS bytes for one sample's visit lists: at most 2 P entries per agent (each incident edge is
// visited from both of its ends; a self-loop twice), one byte each
__host__ __device__ constexpr int update_visit_words(int P) { return (2 * P * P + 3) / 4; }
__host__ __device__ constexpr size_t update_lds_bytes(int P) {
    return 4 * ((size_t)P * UCB + (size_t)(P + 1) + update_visit_words(P));
}
template <bool FUSED>
__device__ __forceinline__ void update_item(const GnnArgs& a, int k, int item, float* lds) {
    // row pairs in flight per wave: the fused pass streams 5 state tensors, so fewer pairs keep
    // its registers at 4+ waves per SIMD
    constexpr int UP_CH = FUSED ? 2 : gnn::UP_CH;
    const int P = a.P, n = a.n;
    const int ncb = (n + UCB - 1) / UCB;
    const int s = item / ncb;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int half = lane / (UCB / 4);               // the lane's row within the instruction's RPI
    const int c = (item % ncb) * UCB + 4 * (lane % (UCB / 4));
    const int cl = 4 * (lane % (UCB / 4));                  // column within the block
    const bool cv = c < n;
    const size_t base = (size_t)s * P * n + (cv ? c : 0);
    bool yzero = false;
    // the guard words and the table entry y_k comes from in the common case, issued together
    // (y_source's walk only when the k - 1 guard fired): one round trip before
    // the visit lists instead of the walk's flag -> table -> flag chain
    const int f_prev = k > 0 ? __builtin_amdgcn_readfirstlane(flag_ld(a.flags + GNN_F_YNB(k - 1))) : 0;
    const int f_u = __builtin_amdgcn_readfirstlane(flag_ld(a.flags + GNN_F_UBAD(k)));
    float* const y_prev = a.yptr[k];
    const float* __restrict__ ys = (k > 0 && f_prev == 0) ? y_prev : y_source(a, k, yzero);
    const bool uzero = f_u != 0;
    float* const fix = (FUSED && k > 0 && f_prev != 0) ? y_prev : nullptr;
    float gclip, vclip;
    clips(a, k, gclip, vclip);
    float* yl = lds;                                  // [P][UCB] y_{k+1}
    int32_t* vpl = (int32_t*)(yl + P * UCB);          // [P + 1] list starts (sample-local)
    uint8_t* vl = (uint8_t*)(vpl + P + 1);            // the sample's visit lists
    const int g0 = a.graph_shared ? 0 : s * P;
    const int vb = a.vptr[g0], vlen = a.vptr[g0 + P] - vb;
    for (int i = threadIdx.x; i <= P; i += THREADS) vpl[i] = a.vptr[g0 + i] - vb;
    for (int i = threadIdx.x; i < vlen; i += THREADS) vl[i] = a.vq[vb + i];
    const float* __restrict__ U = a.U;
    float* __restrict__ Yk = a.yptr[k + 1];
    const f32x4 z4 = {0.0f, 0.0f, 0.0f, 0.0f};
    // row groups (RPI rows): wave w handles groups w, w + 4, ...; `half` selects the lane's row
    bool bad_y = false, bad_g = false;
    auto phase1 = [&](int q0) {
        f32x4 gv[UP_CH], yv[UP_CH];
        float alv[UP_CH];
        if constexpr (FUSED) {
            // every load unconditional (rows past P read agent P - 1, columns past n column 0 —
            // both valid addresses), the results selected afterwards: no load sits under a branch,
            // so the pass's loads stay in flight together instead of draining at each merge
            f32x4 tv[UP_CH], bv[UP_CH], uv[UP_CH], dv[UP_CH];
            float tav[UP_CH], rhv[UP_CH], dgv[UP_CH];
            bool okv[UP_CH];
#pragma unroll
            for (int u = 0; u < UP_CH; ++u) {
                const int p = RPI * (q0 + WAVES * u) + half;
                const int pc = p < P ? p : P - 1;
                okv[u] = p < P && cv;
                const size_t off = base + (size_t)pc * n;
                tv[u] = *(const f32x4*)(a.AtAy + off);
                bv[u] = *(const f32x4*)(a.Atb + off);
                yv[u] = *(const f32x4*)(ys + off);
                uv[u] = *(const f32x4*)(U + off);
                dv[u] = *(const f32x4*)(a.D + off);
                tav[u] = hyp_at(a, s, 1, pc);
                rhv[u] = hyp_at(a, s, 2, pc);
                alv[u] = hyp_at(a, s, 0, pc);
                dgv[u] = a.deg[(a.graph_shared ? 0 : (size_t)s * P) + pc];
            }
#pragma unroll
            for (int u = 0; u < UP_CH; ++u) {
                const bool ok = okv[u];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    tv[u][r] = ok ? tv[u][r] : 0.0f;
                    bv[u][r] = ok ? bv[u][r] : 0.0f;
                    yv[u][r] = (ok && !yzero) ? yv[u][r] : 0.0f;
                    uv[u][r] = (ok && !uzero) ? uv[u][r] : 0.0f;
                    dv[u][r] = ok ? dv[u][r] : 0.0f;
                }
                const int p = RPI * (q0 + WAVES * u) + half;
                if (ok && fix != nullptr) *(f32x4*)(fix + base + (size_t)p * n) = yv[u];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float g = tv[u][r] - bv[u][r];
                    g = g + sign_times(yv[u][r], tav[u]);   // sign(y) * tau
                    g = g + uv[u][r] * dgv[u];
                    g = g + dv[u][r] * rhv[u];
                    g = clamp_t(g, -gclip, gclip);
                    bad_g |= ok && g != g;                  // after the clamp only NaN (:216)
                    gv[u][r] = ok ? g : 0.0f;
                }
            }
        } else {   // resolve: the batch's gradient is zero (:216-218)
#pragma unroll
            for (int u = 0; u < UP_CH; ++u) {
                const int p = RPI * (q0 + WAVES * u) + half;
                gv[u] = yv[u] = z4;
                if (p < P && cv && !yzero) yv[u] = *(const f32x4*)(ys + base + (size_t)p * n);
            }
        }
#pragma unroll
        for (int u = 0; u < UP_CH; ++u) {
            const int p = RPI * (q0 + WAVES * u) + half;
            if (p < P) {
                f32x4 v = z4;
                if (cv) {
                    const float al = FUSED ? alv[u] : hyp_at(a, s, 0, p);
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        v[r] = clamp_t(yv[u][r] - al * gv[u][r], -vclip, vclip);   // :221-225
                        bad_y |= !finitef(v[r]);
                    }
                    *(f32x4*)(Yk + base + (size_t)p * n) = v;
                }
                *(f32x4*)(yl + p * UCB + cl) = v;
            }
        }
    };
    for (int q0 = w; RPI * q0 < P; q0 += WAVES * UP_CH) phase1(q0);
    __syncthreads();
    bool bad_u = false;
    auto phase2 = [&](int q0) {
        f32x4 uv[UP_CH];
        float etv[UP_CH];
#pragma unroll
        for (int u = 0; u < UP_CH; ++u) {
            const int p = RPI * (q0 + WAVES * u) + half;
            if constexpr (FUSED) {
                // unconditional (agent clamped), selected after, as in phase 1
                const int pc = p < P ? p : P - 1;
                const f32x4 t = *(const f32x4*)(U + base + (size_t)pc * n);
                etv[u] = hyp_at(a, s, 3, pc);
                const bool ok = p < P && cv && !uzero;
#pragma unroll
                for (int r = 0; r < 4; ++r) uv[u][r] = ok ? t[r] : 0.0f;
            } else {
                uv[u] = (p < P && cv && !uzero) ? *(const f32x4*)(U + base + (size_t)p * n) : z4;
            }
        }
#pragma unroll
        for (int u = 0; u < UP_CH; ++u) {
            const int p = RPI * (q0 + WAVES * u) + half;
            if (p >= P || !cv) continue;
            const f32x4 yp = *(const f32x4*)(yl + p * UCB + cl);
            f32x4 acc = z4;
            const int v0 = vpl[p], v1 = vpl[p + 1];
            // whole-vector ops: two v_pk_add_f32 / v_pk_add_f32(neg) per visit instead of eight
            // scalar instructions, each lane of the pair rounded exactly as the scalar op
            for (int t = v0; t < v1; ++t) {
                const f32x4 yq = *(const f32x4*)(yl + (int)vl[t] * UCB + cl);
                acc = acc + (yp - yq);
            }
            const float et = FUSED ? etv[u] : hyp_at(a, s, 3, p);
            f32x4 un;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                if (a.variant != 0) acc[r] = clamp_t(acc[r], -20.0f, 20.0f);          // :229
                un[r] = clamp_t(uv[u][r] + acc[r] * et, -vclip, vclip);              // :231-232
                bad_u |= !finitef(un[r]);
            }
            const size_t off = base + (size_t)p * n;
            *(f32x4*)(a.U_next + off) = un;
            *(f32x4*)(a.D_next + off) = acc;
        }
    };
    for (int q0 = w; RPI * q0 < P; q0 += WAVES * UP_CH) phase2(q0);
    if (FUSED) {
        flag_or(a.flags + GNN_F_GBAD(k), bad_g);
        flag_or(a.flags + GNN_F_YNB_OPT(k), bad_y);
        flag_or(a.flags + GNN_F_UNB_OPT(k), bad_u);
    } else {
        flag_or(a.flags + GNN_F_YNB(k), bad_y);
        flag_or(a.flags + GNN_F_UBAD(k + 1), bad_u);
    }
}

// the fused pass: one workgroup per item
__global__ __launch_bounds__(THREADS) void step_kernel(GnnArgs a, int k) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    update_item<true>(a, k, blockIdx.x, lds);
}

// the resolve: a short grid (every workgroup reads one flag word); the g = 0 update, if needed,
// strides over the items
__global__ __launch_bounds__(THREADS) void resolve_kernel(GnnArgs a, int k, int items) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    if (!flag_ld(a.flags + GNN_F_GBAD(k))) {
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            a.flags[GNN_F_YNB(k)] = flag_ld(a.flags + GNN_F_YNB_OPT(k));
            a.flags[GNN_F_UBAD(k + 1)] = flag_ld(a.flags + GNN_F_UNB_OPT(k));
        }
        return;
    }
    for (int item = blockIdx.x; item < items; item += gridDim.x) {
        update_item<false>(a, k, item, lds);
        __syncthreads();   // the LDS tile is reused by the next item
    }
}

// ---- finish: Y[K-1] = y_{K-1} when the last y_next failed its guard; status bits ----------------
__global__ __launch_bounds__(THREADS) void finish_kernel(GnnArgs a) {
    const int K = a.K;
    if (flag_ld(a.flags + GNN_F_YNB(K - 1))) {
        bool zero = false;
        const float* ys = y_source(a, K, zero);   // skips yptr[K]
        const size_t S4 = (size_t)a.B * a.P * a.n / 4;
        f32x4* dst = (f32x4*)a.yptr[K];
        for (size_t i = (size_t)blockIdx.x * THREADS + threadIdx.x; i < S4; i += (size_t)gridDim.x * THREADS)
            dst[i] = zero ? (f32x4){0.0f, 0.0f, 0.0f, 0.0f} : ((const f32x4*)ys)[i];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0 && a.status != nullptr) {
        int st = flag_ld(a.flags + GNN_F_Y0) ? 1 : 0;
        for (int k = 0; k < K; ++k) {
            st |= flag_ld(a.flags + GNN_F_UBAD(k)) ? 2 : 0;
            st |= flag_ld(a.flags + GNN_F_GBAD(k)) ? 4 : 0;
            st |= flag_ld(a.flags + GNN_F_YNB(k)) ? 8 : 0;
        }
        *a.status = st;
    }
}

// ---- adjoint of one iteration (no guard fired) ---------------------------------------------------
// One workgroup per sample, its 4 waves on the sample's 64-column chunks w, w + 4, ... (lanes =
// columns, all P agents per lane: the consensus and its adjoint are lane-local); the per-sample
// hyper-parameter gradients reduce over the columns: wave shuffles per chunk, accumulated per wave
// in LDS in chunk order, then the 4 waves' sums in wave order (deterministic). (One wave per sample
// left most CUs idle at training batch sizes: B = 256 samples filled 64 workgroups.)
// PR > 0 (P <= PR agents): every agent's operands of the lane's column are loaded at once into
// registers (rows past P re-read agent P - 1, never used) and kept through the four phases, so a
// wave waits for memory once per chunk instead of once per agent and phase (the per-agent loads of
// the loop form serialised ~10 HBM round trips: 22 us per iteration at B = 256). The same
// operations in the same order as the loop form: bit-identical.
template <int PR>
__global__ __launch_bounds__(THREADS) void step_backward_kernel(GnnArgs a, int k, GnnGrads gg) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int P = a.P, n = a.n, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int H = a.hyp_rows;
    const int VW = (P + 1) + (2 * P * P + 3) / 4;   // visit-list words per wave
    float* sl = lds + wv * (3 * P * 64 + 4 * P + VW);
    float* y1l = sl;                           // [P][64] y_{k+1}
    float* dbl = sl + P * 64;                  // [P][64] d_bar_raw
    float* ybl = sl + 2 * P * 64;              // [P][64] 2 L d_bar_raw
    float* red = sl + 3 * P * 64;              // [4][H] per-sample hyp gradient
    int32_t* vpl = (int32_t*)(red + 4 * P);    // the sample's visit lists: starts [P + 1], entries
    uint8_t* vql = (uint8_t*)(vpl + P + 1);
    const int s = blockIdx.x;
    float gclip, vclip;
    clips(a, k, gclip, vclip);
    const float* ys = a.yk;
    const int g0 = a.graph_shared ? 0 : s * P;
    for (int i = lane; i < 4 * H; i += 64) red[i] = 0.0f;
    {
        const int v0 = a.vptr[g0], ve = a.vptr[g0 + P];
        for (int i = lane; i <= P; i += 64) vpl[i] = a.vptr[g0 + i] - v0;
        for (int i = lane; i < ve - v0; i += 64) vql[i] = a.vq[v0 + i];
    }
    __builtin_amdgcn_wave_barrier();
    auto accum = [&](int c, int p, float v) {   // wave-sum v into red[c][p or 0]
        v = wave_sum_dpp(v);
    
        if (lane == 0) red[c * H + (H == 1 ? 0 : p)] += v;
    };
    // (round 4) no-alias views of the streams, so that the unrolled agent loops below can put
    // several agents' loads in flight together; the loads read column min(c, n - 1) (always a
    // valid address) and the lanes past n select zeros, as before
    const float* __restrict__ AtAy_r = a.AtAy;
    const float* __restrict__ Atb_r = a.Atb;
    const float* __restrict__ U_r = a.U;
    const float* __restrict__ D_r = a.D;
    const float* __restrict__ ys_r = ys;
    if constexpr (PR > 0) {
        for (int c0 = 64 * wv; c0 < n; c0 += 64 * WAVES) {
            const int c = c0 + lane;
            const bool cv = c < n;
            const size_t base = (size_t)s * P * n + (cv ? c : n - 1);
            float ry[PR], rA[PR], rB[PR], rU[PR], rD[PR], rgy1[PR], rgU1[PR], rgd1[PR], rwb[PR];
#pragma unroll
            for (int p = 0; p < PR; ++p) {
                const size_t off = base + (size_t)(p < P ? p : P - 1) * n;
                ry[p] = ys_r[off];
                rA[p] = AtAy_r[off];
                rB[p] = Atb_r[off];
                rU[p] = U_r[off];
                rD[p] = D_r[off];
                rgy1[p] = gg.gy1 != nullptr ? gg.gy1[off] : 0.0f;
                rgU1[p] = gg.gU1 != nullptr ? gg.gU1[off] : 0.0f;
                rgd1[p] = gg.gd1 != nullptr ? gg.gd1[off] : 0.0f;
            }
            // recompute y_{k+1} for every agent of this column
#pragma unroll
            for (int p = 0; p < PR; ++p) {
                if (p >= P) break;
                const float y = ry[p];
                const float ta = hyp_at(a, s, 1, p);
                const float st = sign_times(y, ta);
                float gr = rA[p] - rB[p];
                gr = gr + st;
                gr = gr + rU[p] * a.deg[g0 + p];
                gr = gr + rD[p] * hyp_at(a, s, 2, p);
                const float g = clamp_t(gr, -gclip, gclip);
                const float y1 = clamp_t(y - hyp_at(a, s, 0, p) * g, -vclip, vclip);
                y1l[p * 64 + lane] = cv ? y1 : 0.0f;
            }
            // dual update adjoint; d_bar_raw (w.r.t. 2 L y_{k+1} before the GNN clamp)
#pragma unroll
            for (int p = 0; p < PR; ++p) {
                if (p >= P) break;
                const float yp = y1l[p * 64 + lane];
                float acc = 0.0f;
                const int t1 = vpl[p + 1];
                for (int t = vpl[p]; t < t1; ++t) acc = acc + (yp - y1l[(int)vql[t] * 64 + lane]);
                float dbr = 0.0f, pe = 0.0f;
                rwb[p] = 0.0f;
                if (cv) {
                    const float d1 = a.variant != 0 ? clamp_t(acc, -20.0f, 20.0f) : acc;
                    const float et = hyp_at(a, s, 3, p);
                    const float wvv = rU[p] + d1 * et;
                    const float wb = (gg.gU1 != nullptr && inside(wvv, -vclip, vclip)) ? rgU1[p] : 0.0f;
                    pe = wb * d1;
                    const float db = (gg.gd1 != nullptr ? rgd1[p] : 0.0f) + wb * et;
                    dbr = (a.variant == 0 || inside(acc, -20.0f, 20.0f)) ? db : 0.0f;
                    rwb[p] = wb;
                }
                accum(3, p, pe);
                dbl[p * 64 + lane] = dbr;
            }
#pragma unroll
            for (int p = 0; p < PR; ++p) {   // 2 L d_bar_raw, same visit lists (the map is symmetric)
                if (p >= P) break;
                const float xp = dbl[p * 64 + lane];
                float acc = 0.0f;
                const int t1 = vpl[p + 1];
                for (int t = vpl[p]; t < t1; ++t) acc = acc + (xp - dbl[(int)vql[t] * 64 + lane]);
                ybl[p * 64 + lane] = acc;
            }
            // primal update + gradient clamp adjoint
#pragma unroll
            for (int p = 0; p < PR; ++p) {
                if (p >= P) break;
                float pa = 0.0f, pt = 0.0f, pr = 0.0f;
                if (cv) {
                    const size_t off = base + (size_t)p * n;
                    const float al = hyp_at(a, s, 0, p), ta = hyp_at(a, s, 1, p), rh = hyp_at(a, s, 2, p);
                    const float y = ry[p];
                    const float sg = sign_times(y, 1.0f);
                    const float st = sign_times(y, ta);
                    float gr = rA[p] - rB[p];
                    gr = gr + st;
                    gr = gr + rU[p] * a.deg[g0 + p];
                    gr = gr + rD[p] * rh;
                    const float g = clamp_t(gr, -gclip, gclip);
                    const float z = y - al * g;
                    const float yb = (gg.gy1 != nullptr ? rgy1[p] : 0.0f) + ybl[p * 64 + lane];
                    const float zb = inside(z, -vclip, vclip) ? yb : 0.0f;
                    pa = -zb * g;
                    const float grb = inside(gr, -gclip, gclip) ? -al * zb : 0.0f;
                    pt = grb * sg;
                    pr = grb * rD[p];
                    gg.gy[off] = zb;
                    gg.gU[off] = rwb[p] + grb * a.deg[g0 + p];
                    gg.gd[off] = grb * rh;
                    gg.gAtAy[off] = grb;
                }
                accum(0, p, pa);
                accum(1, p, pt);
                accum(2, p, pr);
            }
        }
    } else {
        for (int c0 = 64 * wv; c0 < n; c0 += 64 * WAVES) {
            const int c = c0 + lane;
            const bool cv = c < n;
            const size_t base = (size_t)s * P * n + (cv ? c : n - 1);
            // recompute y_{k+1} for every agent of this column
    #pragma unroll 4
            for (int p = 0; p < P; ++p) {
                const size_t off = base + (size_t)p * n;
                const float y = ys_r[off];
                const float ta = hyp_at(a, s, 1, p);
                const float st = sign_times(y, ta);
                float gr = AtAy_r[off] - Atb_r[off];
                gr = gr + st;
                gr = gr + U_r[off] * a.deg[g0 + p];
                gr = gr + D_r[off] * hyp_at(a, s, 2, p);
                const float g = clamp_t(gr, -gclip, gclip);
                const float y1 = clamp_t(y - hyp_at(a, s, 0, p) * g, -vclip, vclip);
                y1l[p * 64 + lane] = cv ? y1 : 0.0f;
            }
            // dual update adjoint; d_bar_raw (w.r.t. 2 L y_{k+1} before the GNN clamp)
            for (int p = 0; p < P; ++p) {
                const float yp = y1l[p * 64 + lane];
                float acc = 0.0f;
                const int t1 = vpl[p + 1];
                for (int t = vpl[p]; t < t1; ++t) acc = acc + (yp - y1l[(int)vql[t] * 64 + lane]);
                float dbr = 0.0f, pe = 0.0f;
                if (cv) {
                    const size_t off = base + (size_t)p * n;
                    const float d1 = a.variant != 0 ? clamp_t(acc, -20.0f, 20.0f) : acc;
                    const float et = hyp_at(a, s, 3, p);
                    const float wvv = a.U[off] + d1 * et;
                    const float wb = (gg.gU1 != nullptr && inside(wvv, -vclip, vclip)) ? gg.gU1[off] : 0.0f;
                    pe = wb * d1;
                    const float db = (gg.gd1 != nullptr ? gg.gd1[off] : 0.0f) + wb * et;
                    dbr = (a.variant == 0 || inside(acc, -20.0f, 20.0f)) ? db : 0.0f;
                    gg.gU[off] = wb;
                }
                accum(3, p, pe);
                dbl[p * 64 + lane] = dbr;
            }
            for (int p = 0; p < P; ++p) {   // 2 L d_bar_raw, same visit lists (the map is symmetric)
                const float xp = dbl[p * 64 + lane];
                float acc = 0.0f;
                const int t1 = vpl[p + 1];
                for (int t = vpl[p]; t < t1; ++t) acc = acc + (xp - dbl[(int)vql[t] * 64 + lane]);
                ybl[p * 64 + lane] = acc;
            }
            // primal update + gradient clamp adjoint
            for (int p = 0; p < P; ++p) {
                float pa = 0.0f, pt = 0.0f, pr = 0.0f;
                if (cv) {
                    const size_t off = base + (size_t)p * n;
                    const float al = hyp_at(a, s, 0, p), ta = hyp_at(a, s, 1, p), rh = hyp_at(a, s, 2, p);
                    const float y = ys[off];
                    const float sg = sign_times(y, 1.0f);
                    const float st = sign_times(y, ta);
                    float gr = a.AtAy[off] - a.Atb[off];
                    gr = gr + st;
                    gr = gr + a.U[off] * a.deg[g0 + p];
                    gr = gr + a.D[off] * rh;
                    const float g = clamp_t(gr, -gclip, gclip);
                    const float z = y - al * g;
                    const float yb = (gg.gy1 != nullptr ? gg.gy1[off] : 0.0f) + ybl[p * 64 + lane];
                    const float zb = inside(z, -vclip, vclip) ? yb : 0.0f;
                    pa = -zb * g;
                    const float grb = inside(gr, -gclip, gclip) ? -al * zb : 0.0f;
                    pt = grb * sg;
                    pr = grb * a.D[off];
                    gg.gy[off] = zb;
                    gg.gU[off] = gg.gU[off] + grb * a.deg[g0 + p];
                    gg.gd[off] = grb * rh;
                    gg.gAtAy[off] = grb;
                }
                accum(0, p, pa);
                accum(1, p, pt);
                accum(2, p, pr);
            }
        }
    }
    __syncthreads();
    const int SW = 3 * P * 64 + 4 * P + VW;     // floats per wave slice
    for (int i = threadIdx.x; i < 4 * H; i += THREADS) {
        const float* r0 = lds + 3 * P * 64 + i;
        const size_t idx = (size_t)s * 4 * H + i;
        float g = ((r0[0] + r0[SW]) + r0[2 * SW]) + r0[3 * SW];
        if (gg.ghyp_add != nullptr) g = g + gg.ghyp_add[idx];
        gg.ghyp[idx] = g;
        if (gg.hdz != nullptr) {
            // the hyper-parameter head's backward (dadmm_hyper_train.hip head_act_kernel, mode 1)
            const int c = i / H;
            const float mx = gg.hmax[c];
            const float sg = 1.0f / (1.0f + expf(-gg.hz[idx]));
            const float v = fminf(fmaxf(sg, 1e-4f), 0.9999f) * mx;
            if (c > 0 && !(v <= 0.9999f)) g = 0.0f;           // clamp(max=0.9999)
            g = g * mx;
            if (!(sg >= 1e-4f && sg <= 0.9999f)) g = 0.0f;    // clamp(1e-4, 0.9999)
            gg.hdz[idx] = g * ((1.0f - sg) * sg);              // sigmoid
        }
    }
}

}  // namespace gnn

// ---- launchers -----------------------------------------------------------------------------------
static int grid_for(size_t work, int per_block, int cap) {
    size_t g = (work + per_block - 1) / per_block;
    if (g < 1) g = 1;
    return (int)(g < (size_t)cap ? g : cap);
}

hipError_t gnn_launch_zero(int32_t* p, int words, hipStream_t st) {
    hipLaunchKernelGGL(gnn::zero_kernel, dim3(grid_for((size_t)words, gnn::THREADS, 64)), dim3(gnn::THREADS), 0, st,
                       p, words);
    return hipGetLastError();
}

hipError_t gnn_launch_check0(const GnnArgs& a, const float* y0, hipStream_t st) {
    const int g = grid_for((size_t)a.B * a.P * a.n / 4, gnn::THREADS, 2048);
    hipLaunchKernelGGL(gnn::check0_kernel, dim3(g), dim3(gnn::THREADS), 0, st, a, y0);
    return hipGetLastError();
}

size_t gnn_gram_lds(int m_pad) { return 4 * (size_t)(BT * (m_pad + 4) + 0); }

hipError_t gnn_launch_gram(const GnnArgs& a, int k, const float* x_raw, float* out, int mode,
                           hipStream_t st) {
    const int mbk = (a.m + 15) / 16;
    const int mq = mbk;
    if (mode != 1 && mbk >= 1 && mbk <= 4 && gnn::gram_lds_bytes(mq, a.n_pad) <= 160 * 1024) {
        // workgroups = P x S splits of the tiles; S minimises (rounds of workgroups over the CUs) x
        // (tiles each wave runs), preferring fewer workgroups on a tie
        // the current device's CU count, queried per call (the runtime caches the attribute; a
        // function-static cache would size the splits for the first device a process used)
        int dev = 0, cus = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
            cus = 256;
        const int tiles = (a.B + BT - 1) / BT;
        // a workgroup per (agent, run of tiles) at >= one tile per wave: too few workgroups to
        // spread over the CUs at small P x B (P = 5, B = 1024: 20) -> gram_kernel's items instead
        if ((long)a.P * ((tiles + gnn::GL_WAVES - 1) / gnn::GL_WAVES) * 2 < cus) goto item_kernel;
        int best_s = 1;
        long best = -1;
        for (int S = 1; S <= (tiles + gnn::GL_WAVES - 1) / gnn::GL_WAVES; ++S) {
            const int tpw = (tiles + S - 1) / S;
            const long cost = (long)((a.P * S + cus - 1) / cus) * ((tpw + gnn::GL_WAVES - 1) / gnn::GL_WAVES);
            if (best < 0 || cost < best) {
                best = cost;
                best_s = S;
            }
        }
        const int tpw = (tiles + best_s - 1) / best_s;
        const size_t lds = gnn::gram_lds_bytes(mq, a.n_pad);
        const void* kern = mq == 1 ? (const void*)gnn::gram_lds_kernel<1>
                         : mq == 2 ? (const void*)gnn::gram_lds_kernel<2>
                         : mq == 3 ? (const void*)gnn::gram_lds_kernel<3> : (const void*)gnn::gram_lds_kernel<4>;
        hipError_t e = hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        const dim3 grid(a.P * best_s), block(64 * gnn::GL_WAVES);
        if (mq == 1)
            hipLaunchKernelGGL(gnn::gram_lds_kernel<1>, grid, block, lds, st, a, k, x_raw, out, mode, tpw);
        else if (mq == 2)
            hipLaunchKernelGGL(gnn::gram_lds_kernel<2>, grid, block, lds, st, a, k, x_raw, out, mode, tpw);
        else if (mq == 3)
            hipLaunchKernelGGL(gnn::gram_lds_kernel<3>, grid, block, lds, st, a, k, x_raw, out, mode, tpw);
        else
            hipLaunchKernelGGL(gnn::gram_lds_kernel<4>, grid, block, lds, st, a, k, x_raw, out, mode, tpw);
        return hipGetLastError();
    }
item_kernel:
    const size_t lds = gnn_gram_lds(a.m_pad);
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute((const void*)gnn::gram_kernel<false>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    const int items = ((a.B + BT - 1) / BT) * a.P;
    if (mode != 1 && a.m == 64 && a.m_pad == 64 && a.n_pad == 256 && items <= 512) {
        hipLaunchKernelGGL(gnn::gram_kernel<true>, dim3(items), dim3(gnn::THREADS), lds, st, a, k, x_raw, out,
                           mode);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(gnn::gram_kernel<false>, dim3(items), dim3(gnn::THREADS), lds, st, a, k, x_raw, out,
                       mode);
    return hipGetLastError();
}

hipError_t gnn_launch_step(const GnnArgs& a, int k, hipStream_t st) {
    const int items = a.B * ((a.n + gnn::UCB - 1) / gnn::UCB);
    const size_t lds = gnn::update_lds_bytes(a.P);
    if (lds > 64 * 1024) {
        for (const void* f : {(const void*)gnn::step_kernel, (const void*)gnn::resolve_kernel}) {
            hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (e != hipSuccess) return e;
        }
    }
    hipLaunchKernelGGL(gnn::step_kernel, dim3(items), dim3(gnn::THREADS), lds, st, a, k);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const int rg = items < 256 ? items : 256;
    hipLaunchKernelGGL(gnn::resolve_kernel, dim3(rg), dim3(gnn::THREADS), lds, st, a, k, items);
    return hipGetLastError();
}

hipError_t gnn_launch_finish(const GnnArgs& a, hipStream_t st) {
    const int g = grid_for((size_t)a.B * a.P * a.n / 4, gnn::THREADS, 2048);
    hipLaunchKernelGGL(gnn::finish_kernel, dim3(g), dim3(gnn::THREADS), 0, st, a);
    return hipGetLastError();
}

hipError_t gnn_launch_step_backward(const GnnArgs& a, int k, const GnnGrads& gg, hipStream_t st) {
    const size_t lds = 4 * (size_t)gnn::WAVES * (3 * a.P * 64 + 4 * a.P + (a.P + 1) + (2 * a.P * a.P + 3) / 4);
    if (lds > 160 * 1024) return hipErrorInvalidConfiguration;
    if (lds > 64 * 1024) {
        for (const void* f : {(const void*)gnn::step_backward_kernel<8>, (const void*)gnn::step_backward_kernel<0>}) {
            hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (e != hipSuccess) return e;
        }
    }
    if (a.P <= 8)
        hipLaunchKernelGGL(gnn::step_backward_kernel<8>, dim3(a.B), dim3(gnn::THREADS), lds, st, a, k, gg);
    else
        hipLaunchKernelGGL(gnn::step_backward_kernel<0>, dim3(a.B), dim3(gnn::THREADS), lds, st, a, k, gg);
    return hipGetLastError();
}

}  // namespace dadmm
