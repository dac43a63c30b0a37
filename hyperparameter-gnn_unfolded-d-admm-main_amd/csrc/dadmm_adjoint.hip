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
typedef float f32x4v __attribute__((ext_vector_type(4)));
// the register-resident update runs in the 16-byte-lane form (adj_update_v4)

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

// wave-sum of v into red[p][c] (lane 0 accumulates; one wave owns its red slice) on DPP moves
// (wave_sum_dpp)
__device__ __forceinline__ void wave_accum(float* red, int p, int c, float v, int lane) {
    v = wave_sum_dpp(v);
    if (lane == 0) red[p * 4 + c] += v;
}

// W waves per workgroup (4; 2 or 1 for the agent counts whose per-wave LDS rows and visit lists
// would not fit four times, P > 64)
template <int W>
__global__ __launch_bounds__(64 * W) void adj_update_kernel(AdjArgs a, int k, int items) {
    constexpr int WAVES = W, THREADS = 64 * W;
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

// The register-resident iteration with 16-byte lanes (P <= PM): y_bar and U_bar stay in
// registers between the two phases (each element read and written once per iteration); lane l owns agent
// p0 + l / 16 of the current group of four and columns 4 (l % 16) .. + 3 of the item's 64, so one
// wave instruction moves four agents' 256-byte rows (1 KB) instead of one agent's 256 bytes, and
// the LDS rows are read as b128 (a 16-lane group spans 16 distinct 16-byte bank slots). Every
// element's value and operation order is the generic kernel's; only the dhyp partial sums are
// associated differently (each lane's 4 columns, then a 16-lane shuffle tree per agent).
__device__ __forceinline__ f32x4v visit_sum4(const float* __restrict__ x, const int32_t* __restrict__ vp,
                                             const uint8_t* __restrict__ vq, int p, int cq) {
    const f32x4v xp = *(const f32x4v*)(x + p * 64 + 4 * cq);
    f32x4v acc = {0.0f, 0.0f, 0.0f, 0.0f};
    const int t1 = vp[p + 1];
    for (int t = vp[p]; t < t1; ++t) {
        const f32x4v xq = *(const f32x4v*)(x + (int)vq[t] * 64 + 4 * cq);
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[r] = acc[r] + (xp[r] - xq[r]);
    }
    return acc;
}

// sum of v over this lane's 4 columns and its 16-lane group -> red[p][c] (lane 16 a adds)
__device__ __forceinline__ void group_accum(float* red, int p, int c, f32x4v v, bool live, int lane) {
    float s = (v[0] + v[1]) + (v[2] + v[3]);
    s = row16_sum_dpp(s);
    if ((lane & 15) == 0 && live) red[p * 4 + c] += s;
}

template <int PM>
__global__ __launch_bounds__(THREADS) void adj_update_v4(AdjArgs a, int k, int items) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int P = a.P, n = a.n, K = a.K, H = a.hyp_rows;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int ag = lane >> 4, cq = lane & 15;          // agent within the group, column quad
    float* xs = lds + w * (2 * P * 64);
    float* ds = xs + P * 64;
    float* red = lds + WAVES * 2 * P * 64;
    float* rw = red + w * P * 4;
    int32_t* vpl = (int32_t*)(red + WAVES * P * 4) + w * (P + 1 + (2 * P * P + 3) / 4);
    uint8_t* vql = (uint8_t*)(vpl + P + 1);
    for (int i = lane; i < P * 4; i += 64) rw[i] = 0.0f;
    const int item = blockIdx.x * WAVES + w;
    const size_t S = (size_t)a.B * P * n;
    constexpr int NG = (PM + 3) / 4;                   // agent groups
    if (item < items) {
        const int nch = (n + 63) / 64;
        const int s = item / nch, c = (item % nch) * 64 + 4 * cq;
        const bool cv = c < n;                          // n % 4 == 0: all 4 columns or none
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
        auto off_of = [&](int p) { return (size_t)s * P * n + (size_t)p * n + (cv ? c : 0); };
        const f32x4v z4 = {0.0f, 0.0f, 0.0f, 0.0f};
        auto ld = [&](const float* __restrict__ base, int p) {
            return (cv && p < P) ? *(const f32x4v*)(base + off_of(p)) : z4;
        };
        auto st = [&](float* __restrict__ base, int p, f32x4v v) {
            if (cv && p < P) *(f32x4v*)(base + off_of(p)) = v;
        };
        const float* __restrict__ y1 = a.Y + (size_t)k * S;
        const float* __restrict__ yk = k > 0 ? a.Y + (size_t)(k - 1) * S : a.y0;
        const float* __restrict__ gYk = a.gY + (size_t)k * S;
        const float* __restrict__ Urk = a.Urec + (size_t)k * S;
        const float* __restrict__ Grk = a.Grec + (size_t)k * S;
        float* __restrict__ ybs = a.yb;
        float* __restrict__ Ubs = a.Ub;
        float* __restrict__ Gbs = a.Gb;
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            const int p = 4 * g + ag;
            if (4 * g < P && p < P) *(f32x4v*)(xs + p * 64 + 4 * cq) = ld(y1, p);
        }
        // the second phase's operands (y_k rows, Grec[k]) issued now, so that phase
        // does not start with another HBM round trip
        f32x4v ykr[NG], grr[NG];
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            ykr[g] = ld(yk, 4 * g + ag);
            grr[g] = ld(Grk, 4 * g + ag);
        }
    
        __builtin_amdgcn_wave_barrier();
        f32x4v ybr[NG], ubr[NG];
        // dual-update adjoint of iteration k (:95-99): the group's loads in flight together, then
        // the visit sums (LDS) under them
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            ybr[g] = ubr[g] = z4;
            if (4 * g >= P) continue;
            const int p = 4 * g + ag;
            const f32x4v gy = ld(gYk, p), ur = ld(Urk, p), gb = ld(Gbs, p);
            ubr[g] = ld(Ubs, p);
            ybr[g] = ld(ybs, p);
            const bool pv = p < P;
            const f32x4v d1 = pv ? visit_sum4(xs, vpl, vql, p, cq) : z4;
            const float et = hyp(k, pv ? p : 0, 3);
            const float rh1 = k + 1 < K ? hyp(k + 1, pv ? p : 0, 2) : 0.0f;
            f32x4v pe = z4, db = z4;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const bool md = a.variant == 0 || inside(d1[r], -20.0f, 20.0f);   // GNN clamp :229
                const float dcl = a.variant == 0 ? d1[r] : tclamp(d1[r], -20.0f, 20.0f);
                ybr[g][r] = ybr[g][r] + gy[r];                                   // + gY[k]
                const float wv = ur[r] + dcl * et;
                const float wb = inside(wv, -vclip, vclip) ? ubr[g][r] : 0.0f;
                pe[r] = wb * dcl;
                db[r] = md ? gb[r] * rh1 + wb * et : 0.0f;
                ubr[g][r] = wb;
            }
            if (!cv) pe = db = z4;
            if (pv) *(f32x4v*)(ds + p * 64 + 4 * cq) = db;
            group_accum(rw, pv ? p : 0, 3, pe, pv, lane);
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            const int p = 4 * g + ag;
            if (4 * g < P && p < P) *(f32x4v*)(xs + p * 64 + 4 * cq) = ykr[g];
        }
        __builtin_amdgcn_wave_barrier();
        // y_bar += 2 L d_bar; primal-update and gradient-clamp adjoint (:73-93)
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            if (4 * g >= P) continue;
            const int p = 4 * g + ag;
            const bool pv = p < P;
            const int pc = pv ? p : 0;
            const f32x4v gr = grr[g];
            f32x4v dk = k == 0 ? ld(a.d0, p) : z4;
            const f32x4v tv = pv ? visit_sum4(ds, vpl, vql, p, cq) : z4;
            if (k > 0 && pv) {
                dk = visit_sum4(xs, vpl, vql, p, cq);
                if (a.variant != 0) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) dk[r] = tclamp(dk[r], -20.0f, 20.0f);
                }
            }
            const float al = hyp(k, pc, 0);
            const float dg = a.deg[g0 + pc];
            const f32x4v y = *(const f32x4v*)(xs + pc * 64 + 4 * cq);
            f32x4v pa = z4, pt = z4, pr = z4, ubn, zbv, grbv;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float gv = tclamp(gr[r], -gclip, gclip);
                const float z = y[r] - al * gv;
                const float ybv = ybr[g][r] + tv[r];
                const float zb = inside(z, -vclip, vclip) ? ybv : 0.0f;
                pa[r] = -zb * gv;
                const float grb = inside(gr[r], -gclip, gclip) ? -al * zb : 0.0f;
                pt[r] = grb * sign_times(y[r], 1.0f);
                pr[r] = grb * dk[r];
                ubn[r] = ubr[g][r] + grb * dg;
                zbv[r] = zb;
                grbv[r] = grb;
            }
            st(Ubs, p, ubn);
            st(ybs, p, zbv);
            st(Gbs, p, grbv);
            if (!cv) pa = pt = pr = z4;
            group_accum(rw, pc, 0, pa, pv, lane);
            group_accum(rw, pc, 1, pt, pv, lane);
            group_accum(rw, pc, 2, pr, pv, lane);
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

static size_t lds_for(int P, int W) {
    return 4 * ((size_t)W * 2 * P * 64 + (size_t)W * P * 4 + (size_t)W * (P + 1 + (2 * P * P + 3) / 4));
}
// waves per workgroup of the update kernel: 4, or fewer where four waves' LDS would not fit
int adjoint_waves(int P) {
    if (P <= 16) return adj::WAVES;
    for (int W = adj::WAVES; W > 1; W /= 2)
        if (lds_for(P, W) <= 160 * 1024) return W;
    return 1;
}
size_t adjoint_lds_bytes(int P) { return lds_for(P, adjoint_waves(P)); }
int adjoint_workgroups(int B, int n, int P) {
    const long items = (long)B * ((n + 63) / 64);
    const int W = adjoint_waves(P);
    return (int)((items + W - 1) / W);
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
    const int W = adjoint_waves(a.P);
    auto kern = a.P <= 8 ? adj::adj_update_v4<8>
              : a.P <= 16 ? adj::adj_update_v4<16>
              : W == 4 ? adj::adj_update_kernel<4> : W == 2 ? adj::adj_update_kernel<2> : adj::adj_update_kernel<1>;
    if (lds > 64 * 1024 &&
        (e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)) !=
            hipSuccess)
        return e;
    const int items = a.B * ((a.n + 63) / 64);
    const int nwg = adjoint_workgroups(a.B, a.n, a.P);
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
        hipLaunchKernelGGL(kern, dim3(nwg), dim3(64 * W), lds, st, a, k, items);
        if ((e = gnn_launch_gram(g, k, a.Gb, a.yb, 2, st)) != hipSuccess) return e;
    }
    if ((e = hipGetLastError()) != hipSuccess) return e;
    return launch_backward_reduce(a.partial, dhyp, nwg, a.K, a.P, a.hyp_rows, st);
}

}  // namespace dadmm
