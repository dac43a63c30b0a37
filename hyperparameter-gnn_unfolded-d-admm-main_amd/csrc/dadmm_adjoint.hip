// dadmm_adjoint.hip — the adjoint of the unfolded D-ADMM forward for EVERY shape (P <= 64, any m,
// n % 4 == 0): the shapes the fused adjoint (dadmm_backward.hip: P <= 6, n <= 256, m <= 64) does
// not hold on chip, e.g. the reference's defaults m = 100, n = 500 (configurations.py:6-9) and
// BASELINE configs[2] (P = 16, n = 512).
//
// Same mathematics as dadmm_backward.hip (see its header): dL/dhyp [K][H][4] for
// L = sum_k <gY[k], Y[k]>, differentiating the reference's eager ops the way torch autograd does
// (unfolded_train_new.py:74-80 through unfolded_DLASSO.py:53-107): sign() has zero derivative,
// clamp passes the gradient where lo <= x <= hi, delta_{k+1} = compute_delta(y_{k+1}) = 2 L y_{k+1}
// (self-adjoint), delta_0 is a leaf. Masks are re-evaluated with the forward's own float ops.
//
// State in HBM (scratch): y_bar, U_bar and gr_bar_{k+1} ([B][P][n] each). Per reverse iteration k:
//   adj_update_kernel  one wave per (sample, 64 columns), all P agents: delta_{k+1} from Y[k] and
//                      delta_k from y_k in the reference's visit order (rows staged in LDS), the
//                      dual-update adjoint, 2 L d_bar, the primal-update / gradient-clamp adjoint;
//                      dhyp partial sums (wave shuffles, then the workgroup's 4 waves in order);
//   gram (mode 2)      y_bar += A_p^T (A_p gr_bar), the forward's MFMA GEMM pair
//                      (dadmm_gnn.hip gram_kernel).
// A fixed-order reduce (dadmm_backward.hip's) sums the workgroup partials: deterministic.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dadmm_internal.h"

namespace dadmm {
namespace adj {

constexpr int THREADS = 256;   // 4 waves, one (sample, 64-column) item each
constexpr int WAVES = 4;

__device__ __forceinline__ float tclamp(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }
__device__ __forceinline__ bool inside(float x, float lo, float hi) { return x >= lo && x <= hi; }

__device__ __forceinline__ void clips(int variant, int k, float& gclip, float& vclip) {
    if (variant == 0) {
        gclip = fmaxf(1.0f, 30.0f - (float)k);          // unfolded_DLASSO.py:80
        vclip = fmaxf(10.0f, 200.0f - (float)(k * 3));  // unfolded_DLASSO.py:92
    } else {
        gclip = 10.0f;                                   // gnn_dlasso_models_progressive.py:212
        vclip = 100.0f;                                  // :224, :232
    }
}

// sum over p's visit list of (x_p - x_q): compute_delta's accumulation order (:127-140). The
// sample's list starts vp [P + 1] (relative) and entries vq sit in this wave's LDS slice: the
// list walk is LDS reads, not a chain of dependent global loads per agent.
__device__ __forceinline__ float visit_sum(const float* __restrict__ x, const int32_t* __restrict__ vp,
                                           const uint8_t* __restrict__ vq, int p, int lane) {
    const float xp = x[p * 64 + lane];
    float acc = 0.0f;
    const int t1 = vp[p + 1];
    for (int t = vp[p]; t < t1; ++t) acc = acc + (xp - x[(int)vq[t] * 64 + lane]);
    return acc;
}

// wave-sum of v into red[p][c] (lane 0 accumulates; one wave owns its red slice)
__device__ __forceinline__ void wave_accum(float* red, int p, int c, float v, int lane) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
    if (lane == 0) red[p * 4 + c] += v;
}

__global__ __launch_bounds__(THREADS) void adj_update_kernel(AdjArgs a, int k, int items) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int P = a.P, n = a.n, K = a.K, H = a.hyp_rows;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    float* xs = lds + w * (2 * P * 64);        // [P][64] rows of y_{k+1}, then of y_k
    float* ds = xs + P * 64;                   // [P][64] d_bar (w.r.t. delta_{k+1})
    float* red = lds + WAVES * 2 * P * 64;     // [WAVES][P][4] partial sums
    float* rw = red + w * P * 4;
    // per wave: the sample's visit-list starts [P + 1] and entries [<= 2 P^2 bytes]
    int32_t* vpl = (int32_t*)(red + WAVES * P * 4) + w * (P + 1 + (2 * P * P + 3) / 4);
    uint8_t* vql = (uint8_t*)(vpl + P + 1);
    for (int i = lane; i < P * 4; i += 64) rw[i] = 0.0f;
    const int item = blockIdx.x * WAVES + w;
    const size_t S = (size_t)a.B * P * n;
    if (item < items) {
        const int nch = (n + 63) / 64;
        const int s = item / nch, c = (item % nch) * 64 + lane;
        const bool cv = c < n;
        const size_t base = (size_t)s * P * n + (cv ? c : 0);
        const int g0 = a.graph_shared ? 0 : s * P;
        {
            const int v0 = a.vptr[g0], ve = a.vptr[g0 + P];
            for (int i = lane; i <= P; i += 64) vpl[i] = a.vptr[g0 + i] - v0;
            for (int i = lane; i < ve - v0; i += 64) vql[i] = a.vq[v0 + i];
        }
        float gclip, vclip;
        clips(a.variant, k, gclip, vclip);
        auto hyp = [&](int kk, int p, int comp) {
            return a.hyp[((size_t)kk * H + (H == 1 ? 0 : p)) * 4 + comp];
        };
        const float* __restrict__ y1 = a.Y + (size_t)k * S;                    // y_{k+1}
        const float* __restrict__ yk = k > 0 ? a.Y + (size_t)(k - 1) * S : a.y0;
        // restrict-qualified views: the scratch state (yb, Ub, Gb) never aliases the recorded
        // trajectory, so the compiler may batch the loads of several agents ahead of the stores
        const float* __restrict__ gYk = a.gY + (size_t)k * S;
        const float* __restrict__ Urk = a.Urec + (size_t)k * S;
        const float* __restrict__ Grk = a.Grec + (size_t)k * S;
        float* __restrict__ ybs = a.yb;
        float* __restrict__ Ubs = a.Ub;
        float* __restrict__ Gbs = a.Gb;
#pragma unroll 4
        for (int p = 0; p < P; ++p) xs[p * 64 + lane] = cv ? y1[base + (size_t)p * n] : 0.0f;
        __builtin_amdgcn_wave_barrier();
        // dual-update adjoint of iteration k (:95-99): w = U_k + delta_{k+1} eta_k. Agents go in
        // groups of GP: the group's visit sums (LDS) first, then all its loads in flight at once,
        // then the arithmetic and the stores (a per-agent load -> use chain was latency-bound)
        constexpr int GP = 4;
        for (int p0 = 0; p0 < P; p0 += GP) {
            float d1[GP], gy[GP], ur[GP], ub[GP], gb[GP], yb[GP];
#pragma unroll
            for (int i = 0; i < GP; ++i) d1[i] = p0 + i < P ? visit_sum(xs, vpl, vql, p0 + i, lane) : 0.0f;
#pragma unroll
            for (int i = 0; i < GP; ++i) {
                const int p = p0 + i;
                gy[i] = ur[i] = ub[i] = gb[i] = yb[i] = 0.0f;
                if (cv && p < P) {
                    const size_t off = base + (size_t)p * n;
                    gy[i] = gYk[off];
                    ur[i] = Urk[off];
                    ub[i] = Ubs[off];
                    gb[i] = Gbs[off];
                    yb[i] = ybs[off];
                }
            }
#pragma unroll
            for (int i = 0; i < GP; ++i) {
                const int p = p0 + i;
                if (p >= P) break;
                const bool md = a.variant == 0 || inside(d1[i], -20.0f, 20.0f);   // GNN clamp :229
                const float dcl = a.variant == 0 ? d1[i] : tclamp(d1[i], -20.0f, 20.0f);
                float pe = 0.0f, db = 0.0f;
                if (cv) {
                    const size_t off = base + (size_t)p * n;
                    const float et = hyp(k, p, 3);
                    const float rh1 = k + 1 < K ? hyp(k + 1, p, 2) : 0.0f;
                    ybs[off] = yb[i] + gy[i];                                     // + gY[k]
                    const float wv = ur[i] + dcl * et;
                    const float wb = inside(wv, -vclip, vclip) ? ub[i] : 0.0f;
                    pe = wb * dcl;
                    db = md ? gb[i] * rh1 + wb * et : 0.0f;
                    Ubs[off] = wb;
                }
                ds[p * 64 + lane] = db;
                wave_accum(rw, p, 3, pe, lane);
            }
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll 4
        for (int p = 0; p < P; ++p) xs[p * 64 + lane] = cv ? yk[base + (size_t)p * n] : 0.0f;
        __builtin_amdgcn_wave_barrier();
        // y_bar += 2 L d_bar; primal-update and gradient-clamp adjoint (:73-93), grouped as above
        for (int p0 = 0; p0 < P; p0 += GP) {
            float tv[GP], dk[GP], gr[GP], yb[GP], ub[GP];
#pragma unroll
            for (int i = 0; i < GP; ++i) {
                const int p = p0 + i;
                tv[i] = dk[i] = 0.0f;
                if (p < P) {
                    tv[i] = visit_sum(ds, vpl, vql, p, lane);
                    if (k > 0) {
                        dk[i] = visit_sum(xs, vpl, vql, p, lane);
                        if (a.variant != 0) dk[i] = tclamp(dk[i], -20.0f, 20.0f);
                    }
                }
            }
#pragma unroll
            for (int i = 0; i < GP; ++i) {
                const int p = p0 + i;
                gr[i] = yb[i] = ub[i] = 0.0f;
                if (cv && p < P) {
                    const size_t off = base + (size_t)p * n;
                    if (k == 0) dk[i] = a.d0[off];
                    gr[i] = Grk[off];
                    yb[i] = ybs[off];
                    ub[i] = Ubs[off];
                }
            }
#pragma unroll
            for (int i = 0; i < GP; ++i) {
                const int p = p0 + i;
                if (p >= P) break;
                float pa = 0.0f, pt = 0.0f, pr = 0.0f;
                if (cv) {
                    const size_t off = base + (size_t)p * n;
                    const float al = hyp(k, p, 0);
                    const float y = xs[p * 64 + lane];
                    const float g = tclamp(gr[i], -gclip, gclip);
                    const float z = y - al * g;
                    const float ybv = yb[i] + tv[i];
                    const float zb = inside(z, -vclip, vclip) ? ybv : 0.0f;
                    pa = -zb * g;
                    const float grb = inside(gr[i], -gclip, gclip) ? -al * zb : 0.0f;
                    pt = grb * sign_times(y, 1.0f);
                    pr = grb * dk[i];
                    const float dg = a.deg[g0 + p];
                    Ubs[off] = ub[i] + grb * dg;
                    ybs[off] = zb;
                    Gbs[off] = grb;
                }
                wave_accum(rw, p, 0, pa, lane);
                wave_accum(rw, p, 1, pt, lane);
                wave_accum(rw, p, 2, pr, lane);
            }
        }
    }
    __syncthreads();
    // workgroup partial: the 4 waves in order -> partial[wg][k][p][c]
    for (int i = threadIdx.x; i < P * 4; i += THREADS) {
        float v = 0.0f;
#pragma unroll
        for (int ww = 0; ww < WAVES; ++ww) v += red[ww * P * 4 + i];
        a.partial[((size_t)blockIdx.x * K + k) * P * 4 + i] = v;
    }
}

// The same iteration with y_bar and U_bar held in registers between the two phases (P <= PM):
// the first phase's y_bar + gY[k] and U_bar' never go to HBM, so each element of y_bar / U_bar is
// read once and written once per iteration (1.47 instead of 2.0 GB per iteration at configs[2]).
// Every value and operation order is the generic kernel's.
template <int PM>
__global__ __launch_bounds__(THREADS) void adj_update_reg(AdjArgs a, int k, int items) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int P = a.P, n = a.n, K = a.K, H = a.hyp_rows;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    float* xs = lds + w * (2 * P * 64);
    float* ds = xs + P * 64;
    float* red = lds + WAVES * 2 * P * 64;
    float* rw = red + w * P * 4;
    int32_t* vpl = (int32_t*)(red + WAVES * P * 4) + w * (P + 1 + (2 * P * P + 3) / 4);
    uint8_t* vql = (uint8_t*)(vpl + P + 1);
    for (int i = lane; i < P * 4; i += 64) rw[i] = 0.0f;
    const int item = blockIdx.x * WAVES + w;
    const size_t S = (size_t)a.B * P * n;
    if (item < items) {
        const int nch = (n + 63) / 64;
        const int s = item / nch, c = (item % nch) * 64 + lane;
        const bool cv = c < n;
        const size_t base = (size_t)s * P * n + (cv ? c : 0);
        const int g0 = a.graph_shared ? 0 : s * P;
        {
            const int v0 = a.vptr[g0], ve = a.vptr[g0 + P];
            for (int i = lane; i <= P; i += 64) vpl[i] = a.vptr[g0 + i] - v0;
            for (int i = lane; i < ve - v0; i += 64) vql[i] = a.vq[v0 + i];
        }
        float gclip, vclip;
        clips(a.variant, k, gclip, vclip);
        auto hyp = [&](int kk, int p, int comp) {
            return a.hyp[((size_t)kk * H + (H == 1 ? 0 : p)) * 4 + comp];
        };
        const float* __restrict__ y1 = a.Y + (size_t)k * S;
        const float* __restrict__ yk = k > 0 ? a.Y + (size_t)(k - 1) * S : a.y0;
        const float* __restrict__ gYk = a.gY + (size_t)k * S;
        const float* __restrict__ Urk = a.Urec + (size_t)k * S;
        const float* __restrict__ Grk = a.Grec + (size_t)k * S;
        float* __restrict__ ybs = a.yb;
        float* __restrict__ Ubs = a.Ub;
        float* __restrict__ Gbs = a.Gb;
        for (int p = 0; p < P; ++p) xs[p * 64 + lane] = cv ? y1[base + (size_t)p * n] : 0.0f;
        __builtin_amdgcn_wave_barrier();
        float ybr[PM], ubr[PM];
        constexpr int GP = 4;
#pragma unroll
        for (int p0 = 0; p0 < PM; p0 += GP) {
            if (p0 >= P) break;
            float d1[GP], gy[GP], ur[GP], gb[GP];
#pragma unroll
            for (int i = 0; i < GP; ++i) d1[i] = p0 + i < P ? visit_sum(xs, vpl, vql, p0 + i, lane) : 0.0f;
#pragma unroll
            for (int i = 0; i < GP; ++i) {
                const int p = p0 + i;
                gy[i] = ur[i] = gb[i] = ybr[p] = ubr[p] = 0.0f;
                if (cv && p < P) {
                    const size_t off = base + (size_t)p * n;
                    gy[i] = gYk[off];
                    ur[i] = Urk[off];
                    ubr[p] = Ubs[off];
                    gb[i] = Gbs[off];
                    ybr[p] = ybs[off];
                }
            }
#pragma unroll
            for (int i = 0; i < GP; ++i) {
                const int p = p0 + i;
                if (p >= P) break;
                const bool md = a.variant == 0 || inside(d1[i], -20.0f, 20.0f);   // GNN clamp :229
                const float dcl = a.variant == 0 ? d1[i] : tclamp(d1[i], -20.0f, 20.0f);
                float pe = 0.0f, db = 0.0f;
                if (cv) {
                    const float et = hyp(k, p, 3);
                    const float rh1 = k + 1 < K ? hyp(k + 1, p, 2) : 0.0f;
                    ybr[p] = ybr[p] + gy[i];                                      // + gY[k]
                    const float wv = ur[i] + dcl * et;
                    const float wb = inside(wv, -vclip, vclip) ? ubr[p] : 0.0f;
                    pe = wb * dcl;
                    db = md ? gb[i] * rh1 + wb * et : 0.0f;
                    ubr[p] = wb;
                }
                ds[p * 64 + lane] = db;
                wave_accum(rw, p, 3, pe, lane);
            }
        }
        __builtin_amdgcn_wave_barrier();
        for (int p = 0; p < P; ++p) xs[p * 64 + lane] = cv ? yk[base + (size_t)p * n] : 0.0f;
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int p0 = 0; p0 < PM; p0 += GP) {
            if (p0 >= P) break;
            float tv[GP], dk[GP], gr[GP];
#pragma unroll
            for (int i = 0; i < GP; ++i) {
                const int p = p0 + i;
                tv[i] = dk[i] = 0.0f;
                if (p < P) {
                    tv[i] = visit_sum(ds, vpl, vql, p, lane);
                    if (k > 0) {
                        dk[i] = visit_sum(xs, vpl, vql, p, lane);
                        if (a.variant != 0) dk[i] = tclamp(dk[i], -20.0f, 20.0f);
                    }
                }
            }
#pragma unroll
            for (int i = 0; i < GP; ++i) {
                const int p = p0 + i;
                gr[i] = 0.0f;
                if (cv && p < P) {
                    const size_t off = base + (size_t)p * n;
                    if (k == 0) dk[i] = a.d0[off];
                    gr[i] = Grk[off];
                }
            }
#pragma unroll
            for (int i = 0; i < GP; ++i) {
                const int p = p0 + i;
                if (p >= P) break;
                float pa = 0.0f, pt = 0.0f, pr = 0.0f;
                if (cv) {
                    const size_t off = base + (size_t)p * n;
                    const float al = hyp(k, p, 0);
                    const float y = xs[p * 64 + lane];
                    const float g = tclamp(gr[i], -gclip, gclip);
                    const float z = y - al * g;
                    const float ybv = ybr[p] + tv[i];
                    const float zb = inside(z, -vclip, vclip) ? ybv : 0.0f;
                    pa = -zb * g;
                    const float grb = inside(gr[i], -gclip, gclip) ? -al * zb : 0.0f;
                    pt = grb * sign_times(y, 1.0f);
                    pr = grb * dk[i];
                    const float dg = a.deg[g0 + p];
                    Ubs[off] = ubr[p] + grb * dg;
                    ybs[off] = zb;
                    Gbs[off] = grb;
                }
                wave_accum(rw, p, 0, pa, lane);
                wave_accum(rw, p, 1, pt, lane);
                wave_accum(rw, p, 2, pr, lane);
            }
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < P * 4; i += THREADS) {
        float v = 0.0f;
#pragma unroll
        for (int ww = 0; ww < WAVES; ++ww) v += red[ww * P * 4 + i];
        a.partial[((size_t)blockIdx.x * K + k) * P * 4 + i] = v;
    }
}

}  // namespace adj

size_t adjoint_lds_bytes(int P) {
    return 4 * ((size_t)adj::WAVES * 2 * P * 64 + (size_t)adj::WAVES * P * 4 +
                (size_t)adj::WAVES * (P + 1 + (2 * P * P + 3) / 4));
}
int adjoint_workgroups(int B, int n) {
    const long items = (long)B * ((n + 63) / 64);
    return (int)((items + adj::WAVES - 1) / adj::WAVES);
}

hipError_t launch_adjoint(const AdjArgs& a, float* dhyp, hipStream_t st) {
    const size_t S = (size_t)a.B * a.P * a.n;
    hipError_t e;
    // y_bar = U_bar = gr_bar_K = 0
    if ((e = hipMemsetAsync(a.yb, 0, 4 * S, st)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(a.Ub, 0, 4 * S, st)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(a.Gb, 0, 4 * S, st)) != hipSuccess) return e;
    const size_t lds = adjoint_lds_bytes(a.P);
    if (lds > 160 * 1024) return hipErrorInvalidConfiguration;
    // y_bar / U_bar register-resident between the phases for P <= 16, the generic kernel above
    auto kern = a.P <= 8 ? adj::adj_update_reg<8> : a.P <= 16 ? adj::adj_update_reg<16> : adj::adj_update_kernel;
    if (lds > 64 * 1024 &&
        (e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)) !=
            hipSuccess)
        return e;
    const int items = a.B * ((a.n + 63) / 64);
    const int nwg = adjoint_workgroups(a.B, a.n);
    GnnArgs g{};
    g.A = a.A;
    g.At = a.At;
    g.B = a.B;
    g.P = a.P;
    g.m = a.m;
    g.m_pad = a.m_pad;
    g.n = a.n;
    g.n_pad = a.n_pad;
    g.K = a.K;
    for (int k = a.K - 1; k >= 0; --k) {
        hipLaunchKernelGGL(kern, dim3(nwg), dim3(adj::THREADS), lds, st, a, k, items);
        if ((e = gnn_launch_gram(g, k, a.Gb, a.yb, 2, st)) != hipSuccess) return e;
    }
    if ((e = hipGetLastError()) != hipSuccess) return e;
    return launch_backward_reduce(a.partial, dhyp, nwg, a.K, a.P, a.hyp_rows, st);
}

}  // namespace dadmm
