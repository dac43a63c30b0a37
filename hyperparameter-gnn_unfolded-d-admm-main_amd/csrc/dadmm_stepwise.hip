// dadmm_stepwise.hip — iteration-at-a-time unfolded D-ADMM forward with the reference's
// batch-global NaN/Inf guards, for every shape (P <= 64, any m up to M_MAX, n % 4 == 0).
//
// Reference semantics: unfolded_DLASSO.py:53-107 (DLASSO_unfolded.forward), :127-140
// (compute_delta); the GNN variant's fixed clamps gnn_dlasso_models_progressive.py:205-232.
//
// Why a second path: the guards (:55-61 y/U reset, :84-86 zero gradient, :102-104 keep y_k) are
// BATCH-GLOBAL — one non-finite value anywhere resets the whole batch — so an exact restatement
// needs a grid-wide decision between the gradient and the primal update and again after the
// primal update. The fused kernel keeps state on-chip for all K iterations and cannot take those
// decisions; it flags the cases instead (status bits) and this path recomputes the batch:
//   * gate = 1 (after dadmm_forward on the same stream): ONE persistent launch whose workgroups
//     all exit at once unless the fused kernel set a status bit; otherwise they run the phases
//     below separated by an in-launch grid barrier (one workgroup per CU, bounded spins);
//   * gate = 0: the same phases as separate launches (shapes the fused kernel does not cover).
//
// Per iteration k:
//   phase G  (item = 16 samples x one agent): y_k tile -> LDS; R = A_p y_k - b_p (GEMM1) and
//            g = A_p^T R (GEMM2) as f32 MFMA fma chains in exactly the fused kernel's (and the
//            oracle's) reduction order; grad assembly + clamp; flag a NaN gradient.
//   phase U  (item = one sample x 64 columns, one wave): y_next = clamp(y_k - alpha g) (g = 0
//            when any gradient was NaN), Y[k] = y_next; delta_{k+1} = 2 L y_next accumulated in
//            the reference's visit order; U_{k+1} = clamp(U_k + delta eta); flag non-finite
//            y_next / U_{k+1}.
// y_k itself is never copied: it is Y[j] for the last j < k whose y_next passed the guard (or y0,
// read as zeros when the k = 0 guard fired); when the guard fired at k - 1, phase G of k rewrites
// Y[k - 1] with y_k, and a final pass does the same for Y[K - 1].

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dadmm_internal.h"

namespace dadmm {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int SW_THREADS = 256;   // 4 waves
constexpr int SW_WAVES = 4;
// per-wave LDS bytes for a sample's visit lists: the worst case 2 P^2 (a complete graph) up to
// 4 KB; longer lists are read from global memory (P > 45 with dense graphs)
__host__ __device__ constexpr int sw_vcap(int P) {
    return ((2 * P * P < 4096 ? 2 * P * P : 4096) + 3) & ~3;
}

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
// torch.clamp: NaN propagates, +-inf saturate
__device__ __forceinline__ float clamp_t(float x, float lo, float hi) {
    return x != x ? x : fminf(fmaxf(x, lo), hi);
}
__device__ __forceinline__ bool finitef(float x) { return __builtin_isfinite(x); }

__device__ __forceinline__ int flag_ld(const int32_t* f) {
    return __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// one atomic per wave (called with every lane of the wave active)
__device__ __forceinline__ void flag_or(int32_t* f, bool v) {
    if (__ballot(v) != 0 && (threadIdx.x & 63) == 0)
        __hip_atomic_fetch_or(f, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// iteration k's y_k: Y[j] for the last j < k whose y_next passed the guard, else y0 (zeros when
// the k = 0 guard fired)
__device__ __forceinline__ const float* y_source(const StepArgs& a, int k, bool& zero) {
    const size_t S = (size_t)a.B * a.P * a.n;
    for (int j = k - 1; j >= 0; --j)
        if (!flag_ld(a.flags + SW_F_YNB(j))) {
            zero = false;
            return a.Y + (size_t)j * S;
        }
    zero = flag_ld(a.flags + SW_F_Y0) != 0;
    return a.y0;
}

__device__ __forceinline__ void hyp_row(const StepArgs& a, int k, int p, float& al, float& ta,
                                        float& rh, float& et) {
    const float* h = a.hyp + ((size_t)k * a.hyp_rows + (a.hyp_rows == 1 ? 0 : p)) * 4;
    al = h[0]; ta = h[1]; rh = h[2]; et = h[3];
}

__device__ __forceinline__ void clips(const StepArgs& a, int k, float& gclip, float& vclip) {
    if (a.variant == 0) {
        gclip = fmaxf(1.0f, 30.0f - (float)k);          // unfolded_DLASSO.py:80
        vclip = fmaxf(10.0f, 200.0f - (float)(k * 3));  // unfolded_DLASSO.py:92
    } else {
        gclip = 10.0f;                                   // gnn_dlasso_models_progressive.py:212
        vclip = 100.0f;                                  // :224, :232
    }
}

// ---- phase 0: the k = 0 guards on y0 / U0 (:55-61), grid-stride over float4s -------------------
__device__ void phase_check0(const StepArgs& a, int wid, int nw) {
    const size_t S4 = (size_t)a.B * a.P * a.n / 4;
    bool by = false, bu = false;
    for (size_t i = (size_t)wid * SW_THREADS + threadIdx.x; i < S4; i += (size_t)nw * SW_THREADS) {
        const f32x4 y = ((const f32x4*)a.y0)[i];
        const f32x4 u = ((const f32x4*)a.U0)[i];
        by |= !(finitef(y[0]) && finitef(y[1]) && finitef(y[2]) && finitef(y[3]));
        bu |= !(finitef(u[0]) && finitef(u[1]) && finitef(u[2]) && finitef(u[3]));
    }
    flag_or(a.flags + SW_F_Y0, by);
    flag_or(a.flags + SW_F_UBAD(0), bu);
}

// ---- phase G: gradient of (16-sample tile, agent p) -------------------------------------------
__device__ void phase_grad(const StepArgs& a, int k, int item, float* lds) {
    const int P = a.P, n = a.n, m = a.m, B = a.B, NP = a.n_pad, MP = a.m_pad;
    const int tile = item / P, p = item % P;
    const int YS = NP + 4, RS = MP + 4;
    float* Ylds = lds;                   // [16][YS]
    float* Rlds = lds + 16 * YS;         // [16][RS]
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int j = lane & 15, h = lane >> 4;
    const int s = tile * BT + j;
    const bool sv = s < B;
    const size_t S = (size_t)B * P * n;

    bool yzero;
    const float* ysrc = y_source(a, k, yzero);
    const bool fix_prev = k > 0 && flag_ld(a.flags + SW_F_YNB(k - 1)) != 0;
    const bool uzero = flag_ld(a.flags + SW_F_UBAD(k)) != 0;
    const float* usrc = k == 0 ? a.U0 : a.U;
    const float* dsrc = k == 0 ? a.d0 : a.D;

    // y_k tile -> LDS (columns past n read as 0: the padded operator columns are 0 too)
    const int nc4 = NP / 4;
    for (int idx = threadIdx.x; idx < BT * nc4; idx += SW_THREADS) {
        const int jj = idx / nc4, c = 4 * (idx % nc4);
        const int s2 = tile * BT + jj;
        f32x4 v = {0.0f, 0.0f, 0.0f, 0.0f};
        if (s2 < B && c < n) {
            const size_t off = ((size_t)s2 * P + p) * n + c;
            if (!yzero) v = *(const f32x4*)(ysrc + off);
            if (fix_prev) *(f32x4*)(a.Y + (size_t)(k - 1) * S + off) = v;   // guard :102-104
        }
        *(f32x4*)(Ylds + jj * YS + c) = v;
    }
    __syncthreads();

    // GEMM1: wave w computes m-blocks w, w + 4, ...: R = A_p y - b_p, one fma chain per row from
    // -b (rows past m stay 0: the padded A^T rows they meet in GEMM2 are 0 too)
    for (int mq = w; mq < MP / 16; mq += SW_WAVES) {
        f32x4 acc;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int mi = 16 * mq + 4 * h + r;
            acc[r] = (sv && mi < m) ? -a.b[((size_t)s * P + p) * m + mi] : 0.0f;
        }
        if (16 * mq < m) {
            const float* arow = a.A + ((size_t)p * MP + 16 * mq + j) * NP + 4 * h;
            const float* brow = Ylds + j * YS + 4 * h;
            for (int t = 0; t < NP / 16; ++t) {
                const f32x4 av = *(const f32x4*)(arow + 16 * t);
                const f32x4 bv = *(const f32x4*)(brow + 16 * t);
#pragma unroll
                for (int r = 0; r < 4; ++r) acc = mfma4(av[r], bv[r], acc);
            }
        }
        *(f32x4*)(Rlds + j * RS + 16 * mq + 4 * h) = acc;
    }
    __syncthreads();

    // GEMM2 + gradient assembly (:73-81): wave w takes n-tiles w, w + 4, ...
    float al, ta, rh, et, gclip, vclip;
    hyp_row(a, k, p, al, ta, rh, et);
    clips(a, k, gclip, vclip);
    const float dg = sv ? a.deg[(a.graph_shared ? 0 : (size_t)s * P) + p] : 0.0f;
    bool bad = false;
    for (int nb = w; nb < NP / 16; nb += SW_WAVES) {
        // one fma chain over every m-block in ascending order (m-blocks past m add exact zeros)
        const float* atrow = a.At + ((size_t)p * NP + 16 * nb + j) * MP + 4 * h;
        f32x4 gc = {0.0f, 0.0f, 0.0f, 0.0f};
        for (int t = 0; t < MP / 16; ++t) {
            const f32x4 av = *(const f32x4*)(atrow + 16 * t);
            const f32x4 rv = *(const f32x4*)(Rlds + j * RS + 16 * t + 4 * h);
#pragma unroll
            for (int r = 0; r < 4; ++r) gc = mfma4(av[r], rv[r], gc);
        }
        const int n0 = 16 * nb + 4 * h;
        if (sv && n0 < n) {
            const size_t off = ((size_t)s * P + p) * n + n0;
            const f32x4 yv = *(const f32x4*)(Ylds + j * YS + n0);
            f32x4 uv = {0.0f, 0.0f, 0.0f, 0.0f};
            if (!uzero) uv = *(const f32x4*)(usrc + off);
            const f32x4 dv = *(const f32x4*)(dsrc + off);
            f32x4 gv, gpre;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float y = yv[r];
                const float st = sign_times(y, ta);   // sign(y) * tau
                float g = gc[r] + st;
                g = g + uv[r] * dg;
                g = g + dv[r] * rh;
                gpre[r] = g;
                g = clamp_t(g, -gclip, gclip);
                bad |= g != g;                     // after the clamp only NaN remains (:84)
                gv[r] = g;
            }
            *(f32x4*)(a.G + off) = gv;
            if (a.Grec != nullptr) {   // the adjoint's trajectory (training)
                *(f32x4*)(a.Grec + (size_t)k * S + off) = gpre;
                *(f32x4*)(a.Urec + (size_t)k * S + off) = uv;
            }
        }
    }
    flag_or(a.flags + SW_F_GBAD(k), bad);
}

// ---- phase U: primal update, consensus and dual update of (sample, 64 columns) -----------------
__device__ void phase_update(const StepArgs& a, int k, int item, float* ylds) {
    const int P = a.P, n = a.n, B = a.B;
    const int nch = (n + 63) / 64;
    const int s = item / nch, c = (item % nch) * 64 + (threadIdx.x & 63);
    const bool cv = c < n;
    const size_t S = (size_t)B * P * n;
    const size_t base = (size_t)s * P * n + c;
    bool yzero;
    const float* ysrc = y_source(a, k, yzero);
    const bool gzero = flag_ld(a.flags + SW_F_GBAD(k)) != 0;
    const bool uzero = flag_ld(a.flags + SW_F_UBAD(k)) != 0;
    const float* usrc = k == 0 ? a.U0 : a.U;
    float gclip, vclip;
    clips(a, k, gclip, vclip);
    float* yl = ylds + (threadIdx.x >> 6) * (P * 64);   // this wave's [P][64] y_next
    const int lane = threadIdx.x & 63;
    // this wave's copy of the sample's visit lists: starts [P + 1] (relative), entries (bytes)
    int32_t* vpl = (int32_t*)(ylds + SW_WAVES * P * 64) + (threadIdx.x >> 6) * (P + 1 + sw_vcap(P) / 4);
    uint8_t* vql = (uint8_t*)(vpl + P + 1);
    const int g0 = a.graph_shared ? 0 : s * P;
    const int v0 = a.vptr[g0], ve = a.vptr[g0 + P];
    // the sample's lists in LDS when they fit the per-wave budget (always for P <= 45; sparse
    // graphs far beyond), else read from global memory (many agents, dense graphs)
    const bool vl = ve - v0 <= sw_vcap(P);
    for (int i = lane; i <= P; i += 64) vpl[i] = a.vptr[g0 + i] - v0;
    if (vl)
        for (int i = lane; i < ve - v0; i += 64) vql[i] = a.vq[v0 + i];

    bool bad_y = false;
    for (int p = 0; p < P; ++p) {
        float al, ta, rh, et;
        hyp_row(a, k, p, al, ta, rh, et);
        float v = 0.0f;
        if (cv) {
            const float g = gzero ? 0.0f : a.G[base + (size_t)p * n];     // :84-86
            const float y = yzero ? 0.0f : ysrc[base + (size_t)p * n];
            v = clamp_t(y - al * g, -vclip, vclip);                         // :89-93
            a.Y[(size_t)k * S + base + (size_t)p * n] = v;
            bad_y |= !finitef(v);
        }
        yl[p * 64 + lane] = v;
    }
    // delta_{k+1}[p] = sum over p's visit list of (y_p - y_q), in the reference's order (:127-140),
    // the list read from LDS (no chain of dependent global loads per agent)
    __builtin_amdgcn_wave_barrier();
    bool bad_u = false;
    for (int p = 0; p < P; ++p) {
        float al, ta, rh, et;
        hyp_row(a, k, p, al, ta, rh, et);
        const float yp = yl[p * 64 + lane];
        float acc = 0.0f;
        const int t1 = vpl[p + 1];
        if (vl) {
            for (int t = vpl[p]; t < t1; ++t) acc = acc + (yp - yl[(int)vql[t] * 64 + lane]);
        } else {
            const uint8_t* __restrict__ vg = a.vq + v0;
            for (int t = vpl[p]; t < t1; ++t) acc = acc + (yp - yl[(int)vg[t] * 64 + lane]);
        }
        if (a.variant != 0) acc = clamp_t(acc, -20.0f, 20.0f);             // GNN :229
        if (cv) {
            const size_t off = base + (size_t)p * n;
            const float u = uzero ? 0.0f : usrc[off];
            const float un = clamp_t(u + acc * et, -vclip, vclip);          // :98-99
            a.U[off] = un;
            a.D[off] = acc;
            bad_u |= !finitef(un);
        }
    }
    flag_or(a.flags + SW_F_YNB(k), bad_y);
    flag_or(a.flags + SW_F_UBAD(k + 1), bad_u);
}

// ---- final pass: Y[K-1] = y_{K-1} when the last y_next failed the guard; status bits ----------
__device__ void phase_final(const StepArgs& a, int wid, int nw) {
    const int K = a.K;
    if (flag_ld(a.flags + SW_F_TIMEOUT)) {
        // the persistent run gave up: poison every iterate so no caller reads a half result
        const size_t T4 = (size_t)K * a.B * a.P * a.n / 4;
        const float qnan = __builtin_nanf("");
        for (size_t i = (size_t)wid * SW_THREADS + threadIdx.x; i < T4; i += (size_t)nw * SW_THREADS)
            ((f32x4*)a.Y)[i] = (f32x4){qnan, qnan, qnan, qnan};
    } else if (flag_ld(a.flags + SW_F_YNB(K - 1))) {
        bool yzero;
        const float* ysrc = y_source(a, K, yzero);   // skips Y[K-1]
        const size_t S4 = (size_t)a.B * a.P * a.n / 4;
        f32x4* dst = (f32x4*)(a.Y + (size_t)(K - 1) * a.B * a.P * a.n);
        for (size_t i = (size_t)wid * SW_THREADS + threadIdx.x; i < S4; i += (size_t)nw * SW_THREADS)
            dst[i] = yzero ? (f32x4){0.0f, 0.0f, 0.0f, 0.0f} : ((const f32x4*)ysrc)[i];
    }
    if (wid == 0 && threadIdx.x == 0 && a.status != nullptr) {
        int st = flag_ld(a.flags + SW_F_Y0) ? 1 : 0;
        for (int k = 0; k < K; ++k) {
            st |= flag_ld(a.flags + SW_F_UBAD(k)) ? 2 : 0;
            st |= flag_ld(a.flags + SW_F_GBAD(k)) ? 4 : 0;
            st |= flag_ld(a.flags + SW_F_YNB(k)) ? 8 : 0;
        }
        st |= flag_ld(a.flags + SW_F_TIMEOUT) ? 0x100 : 0;
        __hip_atomic_store(a.status, st, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// ---- multi-launch form (gate = 0) ---------------------------------------------------------------
__global__ __launch_bounds__(SW_THREADS) void sw_check0_kernel(StepArgs a) {
    phase_check0(a, blockIdx.x, gridDim.x);
}
__global__ __launch_bounds__(SW_THREADS) void sw_grad_kernel(StepArgs a, int k) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    phase_grad(a, k, blockIdx.x, lds);
}
__global__ __launch_bounds__(SW_THREADS) void sw_update_kernel(StepArgs a, int k, int items) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int item = blockIdx.x * SW_WAVES + (threadIdx.x >> 6);
    if (item < items) phase_update(a, k, item, lds);
}
__global__ __launch_bounds__(SW_THREADS) void sw_final_kernel(StepArgs a) {
    phase_final(a, blockIdx.x, gridDim.x);
}

// ---- persistent form (gate = 1): grid barrier between phases ------------------------------------
// Barrier: one monotonic counter (zeroed by the launcher's memset); every wave drains its stores,
// lane 0 releases (agent scope) and arrives, polls relaxed with s_sleep, then acquires (agent
// scope: this CU's L1 drops stale lines) before the workgroup continues (MI355X_MICROARCH.md
// § inter-workgroup visibility). Spins are bounded by the 100 MHz real-time clock: a grid that
// is not co-resident ends with status bit 0x100 instead of hanging.
__device__ bool grid_barrier(const StepArgs& a, uint32_t target) {
    __shared__ int timed_out;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        uint32_t* ctr = (uint32_t*)(a.flags + SW_F_BARRIER);
        __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        int to = 0;
        while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            __builtin_amdgcn_s_sleep(2);
            if (flag_ld(a.flags + SW_F_TIMEOUT) ||
                __builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {   // 2 s
                __hip_atomic_store(a.flags + SW_F_TIMEOUT, 1, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
                to = 1;
                break;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        // a workgroup that gave up earlier has already poisoned (or is poisoning) Y: a late
        // arrival that saw the counter reach the target must not go on writing over it
        if (flag_ld(a.flags + SW_F_TIMEOUT)) to = 1;
        timed_out = to;
    }
    __syncthreads();
    return timed_out == 0;
}

__global__ __launch_bounds__(SW_THREADS) void sw_persistent_kernel(StepArgs a) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    if (__hip_atomic_load(a.status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) return;
    const int G = gridDim.x;
    uint32_t nbar = 0;
    phase_check0(a, blockIdx.x, G);
    if (!grid_barrier(a, (++nbar) * G)) goto out;
    {
        const int items_g = ((a.B + BT - 1) / BT) * a.P;
        const int items_u = a.B * ((a.n + 63) / 64);
        for (int k = 0; k < a.K; ++k) {
            for (int it = blockIdx.x; it < items_g; it += G) {
                phase_grad(a, k, it, lds);
                __syncthreads();
            }
            if (!grid_barrier(a, (++nbar) * G)) goto out;
            for (int it = blockIdx.x * SW_WAVES + (threadIdx.x >> 6); it < items_u;
                 it += G * SW_WAVES)
                phase_update(a, k, it, lds);
            if (!grid_barrier(a, (++nbar) * G)) goto out;
        }
    }
out:
    // The final pass (the Y[K-1] fix-up, or the NaN poison after a timeout) runs in the LAST
    // workgroup to leave: every other workgroup is then past its last write to Y, so no late
    // phase_update of a workgroup that missed the timeout can land over the poison.
    {
        __shared__ int last;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            const uint32_t prev = __hip_atomic_fetch_add((uint32_t*)(a.flags + SW_F_EXIT), 1u,
                                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            last = prev == (uint32_t)(G - 1);
        }
        __syncthreads();
        if (last) phase_final(a, 0, 1);
    }
}

size_t grad_lds_bytes(int n_pad, int m_pad) { return 4 * (size_t)(BT * (n_pad + 4) + BT * (m_pad + 4)); }
size_t update_lds_bytes(int P) {
    return 4 * ((size_t)SW_WAVES * P * 64 + (size_t)SW_WAVES * (P + 1 + sw_vcap(P) / 4));
}

}  // namespace

size_t stepwise_flag_bytes(int K) { return (size_t)SW_FLAG_WORDS(K) * 4; }

hipError_t launch_stepwise(const StepArgs& a, int gate, bool flags_zeroed, hipStream_t stream) {
    hipError_t e = hipSuccess;
    if (!flags_zeroed && (e = hipMemsetAsync(a.flags, 0, stepwise_flag_bytes(a.K), stream)) != hipSuccess)
        return e;
    const size_t lds_g = grad_lds_bytes(a.n_pad, a.m_pad), lds_u = update_lds_bytes(a.P);
    const size_t lds = lds_g > lds_u ? lds_g : lds_u;
    if (lds > 160 * 1024) return hipErrorInvalidConfiguration;
    const void* fns[3] = {(const void*)sw_persistent_kernel, (const void*)sw_grad_kernel,
                          (const void*)sw_update_kernel};
    const size_t need[3] = {lds, lds_g, lds_u};
    for (int i = 0; i < 3; ++i)
        if (need[i] > 64 * 1024 &&
            (e = hipFuncSetAttribute(fns[i], hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)need[i])) != hipSuccess)
            return e;
    if (gate) {
        int dev = 0, cus = 0, per_cu = 0;
        if ((e = hipGetDevice(&dev)) != hipSuccess) return e;
        if ((e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev)) != hipSuccess)
            return e;
        if ((e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, sw_persistent_kernel,
                                                              SW_THREADS, lds)) != hipSuccess)
            return e;
        if (per_cu < 1) return hipErrorInvalidConfiguration;
        // one workgroup per CU: co-resident whenever nothing else occupies the device
        hipLaunchKernelGGL(sw_persistent_kernel, dim3(cus), dim3(SW_THREADS), lds, stream, a);
        return hipGetLastError();
    }
    const int S4 = (int)(((size_t)a.B * a.P * a.n / 4 + SW_THREADS - 1) / SW_THREADS);
    const int gridc = S4 < 2048 ? (S4 > 0 ? S4 : 1) : 2048;
    hipLaunchKernelGGL(sw_check0_kernel, dim3(gridc), dim3(SW_THREADS), 0, stream, a);
    const int items_g = ((a.B + BT - 1) / BT) * a.P;
    const int items_u = a.B * ((a.n + 63) / 64);
    for (int k = 0; k < a.K; ++k) {
        hipLaunchKernelGGL(sw_grad_kernel, dim3(items_g), dim3(SW_THREADS), lds_g, stream, a, k);
        hipLaunchKernelGGL(sw_update_kernel, dim3((items_u + SW_WAVES - 1) / SW_WAVES),
                           dim3(SW_THREADS), lds_u, stream, a, k, items_u);
    }
    hipLaunchKernelGGL(sw_final_kernel, dim3(gridc), dim3(SW_THREADS), 0, stream, a);
    return hipGetLastError();
}

}  // namespace dadmm
