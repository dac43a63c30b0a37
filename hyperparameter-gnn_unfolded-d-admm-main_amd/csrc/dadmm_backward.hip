// dadmm_backward.hip — the adjoint of the fused unfolded D-ADMM forward for gfx950 (MI355X).
//
// Computes dL/dhyp [K][H][4] (alpha, tau, rho, eta) for L = sum_k <gY[k], Y[k]>, i.e. what torch
// autograd returns for the hyper-parameter rows when a driver calls loss.backward() through
// DLASSO_unfolded.forward (unfolded_train_new.py:74-80; forward unfolded_DLASSO.py:53-107). The
// derivative follows torch's rules for the reference's eager ops: sign() has zero derivative,
// clamp(x, lo, hi) passes the gradient where lo <= x <= hi, delta_{k+1} = compute_delta(y_{k+1})
// = 2 (D - Adj) y_{k+1} is differentiated (the map is its own transpose), delta_0 is a random leaf,
// and b / y0 / U0 carry no gradient. The oracle is oracle.backward_np64 (pinned to torch autograd
// through the reference's op sequence, tests/test_oracle.py).
//
// Reverse sweep along the trajectory the recording forward stored (Y, Grec = pre-clamp gradient,
// Urec = U_k); each step reads Y[k], Y[k-1], Grec[k], Urec[k] and gY[k]. Per iteration k, with g = clamp(gr_k), z = y_k - alpha g, w = U_k + delta_{k+1} eta:
//   w_bar = U_bar [|w| <= vclip]            dEta   += w_bar delta_{k+1}
//   d_bar = rho_{k+1} gr_bar_{k+1} + w_bar eta     (GNN variant: masked by |2 L y_{k+1}| <= 20)
//   y_bar += gY[k] + 2 L d_bar
//   z_bar = y_bar [|z| <= vclip]            dAlpha -= z_bar g
//   gr_bar = -alpha z_bar [|gr| <= gclip]   dTau   += gr_bar sign(y_k);  dRho += gr_bar delta_k
//   U_bar = w_bar + deg gr_bar ;  y_bar = z_bar + A^T (A gr_bar)
// The masks are re-evaluated with the forward's own float operations (same consensus order, same
// two-rounding update), so they are exactly the forward's.
//
// Layout mirrors the forward: one workgroup = 16 samples x all P agents x all K
// iterations (reversed), 8 waves; a lane owns rows nb*16 + 4h + r of every agent of sample j, so
// the consensus and its adjoint are lane-local. The Gram product of gr_bar is the forward's GEMM
// pair with gr_bar as the B operand (LDS) and no -b seed. dhyp partial sums: per lane -> wave
// (shuffles) -> workgroup (LDS, fixed order) -> partial[wg][k][P][4]; bwd_reduce_kernel sums the
// workgroups in a fixed order (deterministic).

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dadmm_consensus.h"
#include "dadmm_internal.h"

namespace dadmm {
namespace bwd {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __amdgpu_buffer_rsrc_t rsrc_t;

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ rsrc_t make_rsrc(const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ f32x4 bload4(rsrc_t r, uint32_t voff, uint32_t soff) {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}
__device__ __forceinline__ float tclamp(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }
__device__ __forceinline__ bool inside(float x, float lo, float hi) { return x >= lo && x <= hi; }
typedef const __attribute__((address_space(4))) float cfloat;
// compiler-only barrier: bounds how far the scheduler hoists loads (register budget)
__device__ __forceinline__ void fence() { asm volatile("" ::: "memory"); }
// a per-iteration opaque copy of a wave-uniform value: keeps the shared graph's neighbour tests
// inside the loop (s_bitcmp + branch) instead of P*P hoisted 64-bit condition registers
__device__ __forceinline__ uint32_t fresh_s(uint32_t x) {
    asm volatile("" : "=s"(x) : "0"(x));
    return x;
}

// Decisions measured at H (round 6 removed the A/B switches):
//   * 4 waves per workgroup (one per SIMD, 512 registers: twice the rows per wave, room for more of
//     the five trajectory streams in flight): 1.22 vs 1.27-1.28 ms with 8 (adjoint_variants_r05j);
//   * GEMM2's A^T straight from L2 (the loads sit in the 512-register budget) instead of the
//     forward's LDS-DMA ring: 1.19-1.21 vs 1.22-1.23 ms (adjoint_variants_r05p);
//   * the elementwise phase walks the wave's T2 row tiles in a runtime loop and rotates the carried
//     state (y_bar, U_bar) so that the current tile's rows are always columns 0..3 of the register
//     arrays (static indices); the unrolled tile loop interleaved the two tiles' temporaries
//     (256 VGPRs + 231 spilled at H, this form 13);
//   * all five streams of a tile (Y[k], Urec, gY, Y[k-1] or d0, Grec) software-pipelined: the NEXT
//     tile's streams (after a wave's last tile: the first tile of iteration k - 1) issued at the
//     top of the current one, so the last tile's prefetch lands under the GEMM phases;
//   * the shared graph's consensus on row pairs with packed f32 instructions (consensus_fma2: the
//     same values as the forward's consensus_fma, so the re-evaluated masks are the forward's);
//   * the per-iteration dhyp wave sums on DPP moves (wave_sum_dpp): a fixed order, deterministic.
constexpr int WAVES = 4;
#define BWD_ROW(e, r) (r)
typedef __attribute__((address_space(3))) void lds_void;
__device__ __forceinline__ void wait_vm(int n) {   // s_waitcnt vmcnt(n), n folded at compile time
    switch (n) {
        case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
        case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    }
}

// GNN variant: delta = clamp(delta, -20, 20) (gnn_dlasso_models_progressive.py:229) in place;
// returns bit 4p+r set where the pre-clamp value was inside (the clamp passes the gradient)
template <int P>
__device__ __forceinline__ uint32_t clamp_delta(float (&dd)[P][4], int variant) {
    uint32_t bits = 0xffffffffu;
    if (variant != 0) {
#pragma unroll
        for (int p = 0; p < P; ++p)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                if (!inside(dd[p][r], -20.0f, 20.0f)) bits &= ~(1u << (4 * p + r));
                dd[p][r] = tclamp(dd[p][r], -20.0f, 20.0f);
            }
    }
    return bits;
}

template <int P, int NT, int GRAPH, int HALF>
__device__ __forceinline__ void body(const BackwardArgs& a, float* __restrict__ lds, const int w) {
    constexpr int AS = WAVES / 4;                   // GEMM1 agent stride
    constexpr int MP = M_PAD;
    constexpr int NP = NT * 64;
    constexpr int NB = NP / 16;
    constexpr int T2 = (NB + WAVES - 1) / WAVES;
    constexpr int E = T2 * 4;
    constexpr int TH = (P - HALF + AS - 1) / AS;
    constexpr int THA = TH > 0 ? TH : 1;
    constexpr int YS = NP + 4;
    constexpr int RS = MP + 4;
    float* __restrict__ Glds = lds;                 // [P][BT][YS]  gr_bar (GEMM B operand)
    float* __restrict__ Rlds = lds + P * BT * YS;   // [P][BT][RS]  A gr_bar
    float* __restrict__ red = Rlds + P * BT * RS;   // [WAVES][P][4] partial sums

    const int lane = threadIdx.x & 63;
    const int j = lane & 15;
    const int h = lane >> 4;
    const int s = blockIdx.x * BT + j;
    const bool sv = s < a.B;
    const int n = a.n, B = a.B, K = a.K;
    const int mb = w & 3;
    const bool has_tiles = w * T2 < NB;
    const uint32_t state_bytes = (uint32_t)((size_t)B * P * n * 4);
    const size_t S = (size_t)B * P * n;
    const rsrc_t rA = make_rsrc(a.A, (uint32_t)(P * MP * NP * 4));
    const rsrc_t rAt = make_rsrc(a.At, (uint32_t)(P * MP * NP * 4));

    uint32_t msk[P], ord[P];
    float dg[P];
#pragma unroll
    for (int p = 0; p < P; ++p) {
        if (GRAPH == GRAPH_SHARED) {
            msk[p] = __builtin_amdgcn_readfirstlane((uint32_t)a.nbr[p]);
            dg[p] = a.deg[p];
        } else {
            msk[p] = sv ? (uint32_t)a.nbr[(size_t)s * P + p] : 0u;
            dg[p] = sv ? a.deg[(size_t)s * P + p] : 0.0f;
        }
        ord[p] = (GRAPH == GRAPH_ORDERED && sv) ? a.nbr_order[(size_t)s * P + p] : 0u;
    }

    // carried state (registers): y_bar, U_bar, the adjoints w.r.t. y_{k+1}, U_{k+1}; d_bar (w.r.t.
    // delta_{k+1}) is rho_{k+1} * gr_bar_{k+1}, read back from this lane's Glds rows; delta_{k+1}
    // is re-formed from y_{k+1} = Y[k] (re-read: the register budget holds two [P][E] arrays)
    float yb[P][E], Ub[P][E];
#pragma unroll
    for (int tt = 0; tt < T2; ++tt) {
        const int n0 = (w * T2 + tt) * 16 + 4 * h;
#pragma unroll
        for (int p = 0; p < P; ++p) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                yb[p][4 * tt + r] = 0.0f;
                Ub[p][4 * tt + r] = 0.0f;
            }
            if (has_tiles) *(f32x4*)(Glds + (p * BT + j) * YS + n0) = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
        }
    }
    // the shared graph's edges as 0/1 multipliers (uniform), mf[a][b] = (b in N(a)); the adjoint
    // needs an undirected graph (dadmm_backward refuses others), for which this is the forward's
    // consensus_fma operand
    float mf[P][P];
#pragma unroll
    for (int q = 0; q < P; ++q)
#pragma unroll
        for (int p = 0; p < P; ++p) mf[q][p] = (GRAPH == GRAPH_SHARED && ((msk[q] >> p) & 1u)) ? 1.0f : 0.0f;
    [[maybe_unused]] f32x2_c mf2[P][P];
#pragma unroll
    for (int q = 0; q < P; ++q)
#pragma unroll
        for (int p = 0; p < P; ++p) mf2[q][p] = (f32x2_c){mf[q][p], mf[q][p]};
    auto cons = [&](const float (&x)[P][4], float (&o)[P][4], const uint32_t (&mk_)[P]) {
        if constexpr (GRAPH == GRAPH_SHARED) {
#pragma unroll
            for (int rp = 0; rp < 2; ++rp) {   // rows (2 rp, 2 rp + 1) packed
                f32x2_c yy[P], dd[P];
#pragma unroll
                for (int p = 0; p < P; ++p) yy[p] = (f32x2_c){x[p][2 * rp], x[p][2 * rp + 1]};
                consensus_fma2<P>(yy, dd, mf2);
#pragma unroll
                for (int p = 0; p < P; ++p) {
                    o[p][2 * rp] = dd[p][0];
                    o[p][2 * rp + 1] = dd[p][1];
                }
            }
        } else if constexpr (GRAPH == GRAPH_SHARED) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float yy[P][1], dd[P][1];
#pragma unroll
                for (int p = 0; p < P; ++p) yy[p][0] = x[p][r];
                consensus_fma<P>(yy, dd, mf);
#pragma unroll
                for (int p = 0; p < P; ++p) o[p][r] = dd[p][0];
            }
        } else {
            consensus_any<P, GRAPH>(x, o, mk_, ord);
        }
    };
    float rh_next[P];   // rho_{k+1} (0 at k = K-1: no later iteration reads delta_K)
#pragma unroll
    for (int p = 0; p < P; ++p) rh_next[p] = 0.0f;

    const uint32_t voffA = (uint32_t)(((16 * mb + j) * NP + 4 * h) * 4);
    const uint32_t voffAt = (uint32_t)((j * MP + 4 * h) * 4);
    const float* brow = Glds + j * YS + 4 * h;
    // the five streams of (iteration kk, tile tt_) into one set of registers; every load is
    // unconditional (branch-free: a load under a branch makes the compiler drain the queue)
    f32x4 cy1[P], cu[P], cg[P], cyk[P], cgr[P];
    // stream c of (iteration kk, tile tt_): 0 Y[kk], 1 Urec[kk], 2 gY[kk], 3 Y[kk-1] (d0 at kk = 0),
    // 4 Grec[kk]
    auto issue1 = [&](int c, int kk, int tt_, f32x4 (&dst)[P]) {
        const float* base = c == 0 ? a.Y + (size_t)kk * S
                          : c == 1 ? a.Urec + (size_t)kk * S
                          : c == 2 ? a.gY + (size_t)kk * S
                          : c == 3 ? (kk > 0 ? a.Y + (size_t)(kk - 1) * S : a.d0)
                                   : a.Grec + (size_t)kk * S;
        const rsrc_t rs = make_rsrc(base, state_bytes);
        const int n0_ = (w * T2 + tt_) * 16 + 4 * h;
        const uint32_t vr = n0_ < n ? (uint32_t)((s * P * n + n0_) * 4) : 0x80000000u;
#pragma unroll
        for (int p = 0; p < P; ++p) dst[p] = bload4(rs, vr, (uint32_t)(p * n * 4));
    };
    if (has_tiles) {
        issue1(0, K - 1, 0, cy1);
        issue1(1, K - 1, 0, cu);
        issue1(2, K - 1, 0, cg);
        issue1(3, K - 1, 0, cyk);
        issue1(4, K - 1, 0, cgr);
    }
    __syncthreads();

    for (int k = K - 1; k >= 0; --k) {
        uint32_t mk[P];
#pragma unroll
        for (int p = 0; p < P; ++p) {
            if constexpr (GRAPH == GRAPH_SHARED) mk[p] = fresh_s(msk[p]);
            else mk[p] = msk[p];
        }
        float al[P], ta[P], rh[P], et[P];
#pragma unroll
        for (int p = 0; p < P; ++p) {
            // through the scalar cache (constant address space: the table is read-only for the
            // launch), so the per-iteration hyper-parameters sit in SGPRs, not VGPRs
            const cfloat* hp = (const cfloat*)a.hyp + ((size_t)k * a.hyp_rows + (a.hyp_rows == 1 ? 0 : p)) * 4;
            al[p] = hp[0]; ta[p] = hp[1]; rh[p] = hp[2]; et[p] = hp[3];
        }
        float gclip, vclip;
        if (a.variant == 0) {
            gclip = fmaxf(1.0f, 30.0f - (float)k);          // unfolded_DLASSO.py:80
            vclip = fmaxf(10.0f, 200.0f - (float)(k * 3));  // unfolded_DLASSO.py:92
        } else {
            gclip = 10.0f;                                   // gnn_dlasso_models_progressive.py:212
            vclip = 100.0f;                                  // :224, :232
        }
        float part[P][4];
#pragma unroll
        for (int p = 0; p < P; ++p)
#pragma unroll
            for (int c = 0; c < 4; ++c) part[p][c] = 0.0f;

        // ---- elementwise adjoint of iteration k on this lane's rows ---------------------------
        if (has_tiles) {
            const rsrc_t ryk = make_rsrc(k > 0 ? a.Y + (size_t)(k - 1) * S : a.y0, state_bytes);
            [[maybe_unused]] const rsrc_t ry1 = make_rsrc(a.Y + (size_t)k * S, state_bytes);
            [[maybe_unused]] const rsrc_t rgr = make_rsrc(a.Grec + (size_t)k * S, state_bytes);
            [[maybe_unused]] const rsrc_t ruk = make_rsrc(a.Urec + (size_t)k * S, state_bytes);
            [[maybe_unused]] const rsrc_t rgy = make_rsrc(a.gY + (size_t)k * S, state_bytes);
            [[maybe_unused]] const rsrc_t rd0 = make_rsrc(a.d0, state_bytes);
#pragma unroll 1
            for (int tt = 0; tt < T2; ++tt) {
                const int n0 = (w * T2 + tt) * 16 + 4 * h;
                const bool ok = n0 < n;
                // one VGPR offset per row group; the agent's (uniform) offset rides in soffset.
                // Rows past n get an offset the buffer range check turns into zeros (no branches).
                const uint32_t vrow = ok ? (uint32_t)((s * P * n + n0) * 4) : 0x80000000u;
                // live ranges kept short (register budget): [P][4] temporaries t1, t2
                float t1[P][4], t2[P][4];
                // this tile's streams were issued a tile (or the GEMM phases) ago; each stream of
                // the next tile (after the last tile: iteration k - 1's first) is issued into the
                // same registers right after this tile's last read of it
                const bool last_t = tt + 1 == T2;
                const int nk = last_t ? (k > 0 ? k - 1 : 0) : k, ntt = last_t ? 0 : tt + 1;
#define py1 cy1
#define pu cu
#define pg cg
#define pyk cyk
#define pgr cgr
#define BWD_LD(pre, rs) (pre[p])
#define BWD_NEXT(c, arr) issue1(c, nk, ntt, arr)
                // t2 = delta_{k+1} formed from y_{k+1} exactly as the forward did
#pragma unroll
                for (int p = 0; p < P; ++p) {
                    const f32x4 v = BWD_LD(py1, ry1);
#pragma unroll
                    for (int r = 0; r < 4; ++r) t1[p][r] = v[r];
                }
                BWD_NEXT(0, cy1);
                cons(t1, t2, mk);
                const uint32_t md1 = clamp_delta(t2, a.variant);
                fence();
                // dual update adjoint (:98-99); t1 = d_bar
#pragma unroll
                for (int p = 0; p < P; ++p) {
                    const f32x4 vu = BWD_LD(pu, ruk);
                    const f32x4 vg = BWD_LD(pg, rgy);
                    const f32x4 gprev = *(const f32x4*)(Glds + (p * BT + j) * YS + n0);
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        [[maybe_unused]] const int e = 4 * tt + r;
                        yb[p][BWD_ROW(e, r)] = yb[p][BWD_ROW(e, r)] + vg[r];  // + gY[k]
                        const float wv = vu[r] + t2[p][r] * et[p];
                        const float wb = inside(wv, -vclip, vclip) ? Ub[p][BWD_ROW(e, r)] : 0.0f;
                        part[p][3] += wb * t2[p][r];
                        const float db = gprev[r] * rh_next[p] + wb * et[p];
                        t1[p][r] = ((md1 >> (4 * p + r)) & 1u) ? db : 0.0f;
                        Ub[p][BWD_ROW(e, r)] = wb;
                    }
                }
                BWD_NEXT(1, cu);
                BWD_NEXT(2, cg);
                cons(t1, t2, mk);   // t2 = 2 L d_bar
#pragma unroll
                for (int p = 0; p < P; ++p)
#pragma unroll
                    for (int r = 0; r < 4; ++r) yb[p][BWD_ROW(4 * tt + r, r)] += t2[p][r];
                fence();
                // t1 = y_k; t2 = delta_k (k > 0: formed from y_k as the forward did; k = 0: d0)
                if (k > 0) {
#pragma unroll
                    for (int p = 0; p < P; ++p)
#pragma unroll
                        for (int r = 0; r < 4; ++r) t1[p][r] = pyk[p][r];
                    cons(t1, t2, mk);
                    clamp_delta(t2, a.variant);
                } else {   // y_0 (the prefetch slot held d0)
#pragma unroll
                    for (int p = 0; p < P; ++p) {
                        const f32x4 v = bload4(ryk, vrow, (uint32_t)(p * n * 4));
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            t1[p][r] = v[r];
                            t2[p][r] = pyk[p][r];
                        }
                    }
                }
                BWD_NEXT(3, cyk);
                fence();
                // primal update + gradient clamp adjoint (:73-93)
#pragma unroll
                for (int p = 0; p < P; ++p) {
                    const f32x4 vgr = BWD_LD(pgr, rgr);
                    f32x4 gbv;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        [[maybe_unused]] const int e = 4 * tt + r;
                        const float yk = t1[p][r];
                        const float gr = vgr[r];
                        const float g = tclamp(gr, -gclip, gclip);
                        const float z = yk - al[p] * g;
                        const float zb = inside(z, -vclip, vclip) ? yb[p][BWD_ROW(e, r)] : 0.0f;
                        part[p][0] -= zb * g;
                        const float grb = inside(gr, -gclip, gclip) ? -al[p] * zb : 0.0f;
                        const float sg = sign_times(yk, 1.0f);
                        part[p][1] += grb * sg;
                        part[p][2] += grb * t2[p][r];
                        Ub[p][BWD_ROW(e, r)] = Ub[p][BWD_ROW(e, r)] + grb * dg[p];
                        yb[p][BWD_ROW(e, r)] = zb;
                        gbv[r] = ok ? grb : 0.0f;
                    }
                    *(f32x4*)(Glds + (p * BT + j) * YS + n0) = gbv;
                }
                BWD_NEXT(4, cgr);
#undef py1
#undef pu
#undef pg
#undef pyk
#undef pgr
#undef BWD_NEXT
                // rotate: the next tile's carried state moves to rows 0..3 (T2 rotations: identity)
#pragma unroll
                for (int p = 0; p < P; ++p)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float y0v = yb[p][r], u0v = Ub[p][r];
#pragma unroll
                        for (int t2 = 0; t2 + 1 < T2; ++t2) {
                            yb[p][4 * t2 + r] = yb[p][4 * (t2 + 1) + r];
                            Ub[p][4 * t2 + r] = Ub[p][4 * (t2 + 1) + r];
                        }
                        yb[p][4 * (T2 - 1) + r] = y0v;
                        Ub[p][4 * (T2 - 1) + r] = u0v;
                    }
            }
        }
        __syncthreads();

        // ---- GEMM1: R_p = A_p gr_bar_p (this wave: m-block mb, agents HALF + AS*i); the A rows
        //      of step t+1 load under the MFMAs of step t ----------------------------------------
        {
            f32x4 acc[THA], av[2][THA];
#pragma unroll
            for (int i = 0; i < TH; ++i) {
                acc[i] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
                av[0][i] = bload4(rA, voffA, (uint32_t)((HALF + AS * i) * MP * NP * 4));
            }
#pragma unroll
            for (int t = 0; t < NB; ++t) {
                if (t + 1 < NB) {
#pragma unroll
                    for (int i = 0; i < TH; ++i)
                        av[(t + 1) & 1][i] = bload4(rA, voffA + 64 * (t + 1),
                                                    (uint32_t)((HALF + AS * i) * MP * NP * 4));
                }
                fence();
#pragma unroll
                for (int i = 0; i < TH; ++i) {
                    const f32x4 bv = *(const f32x4*)(brow + (HALF + AS * i) * BT * YS + 16 * t);
#pragma unroll
                    for (int r = 0; r < 4; ++r) acc[i] = mfma4(av[t & 1][i][r], bv[r], acc[i]);
                }
            }
#pragma unroll
            for (int i = 0; i < TH; ++i)
                *(f32x4*)(Rlds + ((HALF + AS * i) * BT + j) * RS + 16 * mb + 4 * h) = acc[i];
        }
        __syncthreads();

        // ---- GEMM2: y_bar_p += A_p^T R_p on this wave's n-tiles, as (agent, tile) chains of 16
        //      MFMAs; the A^T rows of the next chain load under the current one ----------------
        if (has_tiles) {
            constexpr int NS = P * T2;
            f32x4 tring[2][MP / 16];
            auto load_at = [&](f32x4 (&slot)[MP / 16], int c) {
                const int p = c / T2, tt = c % T2;
                const uint32_t vAt = voffAt + (uint32_t)(16 * (w * T2 + tt) * MP * 4);
#pragma unroll
                for (int t = 0; t < MP / 16; ++t)
                    slot[t] = bload4(rAt, vAt + 64 * t, (uint32_t)(p * NP * MP * 4));
            };
            load_at(tring[0], 0);
#pragma unroll
            for (int c = 0; c < NS; ++c) {
                const int p = c / T2, tt = c % T2;
                if (c + 1 < NS) load_at(tring[(c + 1) & 1], c + 1);
                fence();
                f32x4 rv[MP / 16];
#pragma unroll
                for (int t = 0; t < MP / 16; ++t)
                    rv[t] = *(const f32x4*)(Rlds + (p * BT + j) * RS + 4 * h + 16 * t);
                f32x4 gc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
                for (int t = 0; t < MP / 16; ++t)
#pragma unroll
                    for (int r = 0; r < 4; ++r) gc = mfma4(tring[c & 1][t][r], rv[t][r], gc);
#pragma unroll
                for (int r = 0; r < 4; ++r) yb[p][4 * tt + r] += gc[r];
            }
        }


        // ---- dhyp partial sums of iteration k: lane -> wave -> workgroup --------------------
#pragma unroll
        for (int p = 0; p < P; ++p)
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                float v = part[p][c];
                v = wave_sum_dpp(v);
            
                if (lane == 0) red[(w * P + p) * 4 + c] = v;
            }
        __syncthreads();
        if ((int)threadIdx.x < P * 4) {
            float v = 0.0f;
#pragma unroll
            for (int ww = 0; ww < WAVES; ++ww) v += red[ww * P * 4 + threadIdx.x];
            a.partial[((size_t)blockIdx.x * K + k) * P * 4 + threadIdx.x] = v;
        }
#pragma unroll
        for (int p = 0; p < P; ++p) rh_next[p] = rh[p];
    }
}

template <int P, int NT, int GRAPH>
__global__ __launch_bounds__(WAVES * 64) __attribute__((amdgpu_waves_per_eu(1, 1)))
void backward_kernel(BackwardArgs a) {
    constexpr int NP = NT * 64;
    __shared__ __attribute__((aligned(16))) float lds[P * BT * ((NP + 4) + (M_PAD + 4)) + WAVES * P * 4];
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    body<P, NT, GRAPH, 0>(a, lds, w);
}

// dhyp[k][hh][c] = sum over workgroups (and over agents for H = 1) of partial[wg][k][p][c]; one
// wave per output, lanes stride the workgroups, fixed shuffle tree: deterministic.
__global__ __launch_bounds__(256) void reduce_kernel(const float* __restrict__ partial,
                                                     float* __restrict__ dhyp, int nwg, int K, int P,
                                                     int H) {
    const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (t >= K * H * 4) return;
    const int c = t & 3, hh = (t >> 2) % H, k = t / (4 * H);
    float v = 0.0f;
    for (int wg = lane; wg < nwg; wg += 64) {
        const float* row = partial + ((size_t)wg * K + k) * P * 4;
        if (H == P) {
            v += row[hh * 4 + c];
        } else {
            for (int p = 0; p < P; ++p) v += row[p * 4 + c];
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
    if (lane == 0) dhyp[t] = v;
}

template <int P, int NT, int GRAPH>
hipError_t launch(const BackwardArgs& a, hipStream_t stream) {
    const int grid = (a.B + BT - 1) / BT;
    hipLaunchKernelGGL((backward_kernel<P, NT, GRAPH>), dim3(grid), dim3(WAVES * 64), 0, stream, a);
    return hipGetLastError();
}

template <int P, int NT>
backward_fn_ptr pick_graph(int graph) {
    switch (graph) {
        case GRAPH_SHARED: return &launch<P, NT, GRAPH_SHARED>;
        case GRAPH_LANE: return &launch<P, NT, GRAPH_LANE>;
        case GRAPH_ORDERED: return &launch<P, NT, GRAPH_ORDERED>;
        default: return nullptr;
    }
}

template <int P>
backward_fn_ptr pick_nt(int nt, int graph) {
    if (nt == 1) return pick_graph<P, 1>(graph);
    if (nt == 2) return pick_graph<P, 2>(graph);
    if constexpr (P <= 5) {
        if (nt == 4) return pick_graph<P, 4>(graph);
    }
    return nullptr;
}

}  // namespace bwd

backward_fn_ptr find_backward(int P, int nt, int graph) {
    switch (P) {
        case 1: return bwd::pick_nt<1>(nt, graph);
        case 2: return bwd::pick_nt<2>(nt, graph);
        case 3: return bwd::pick_nt<3>(nt, graph);
        case 4: return bwd::pick_nt<4>(nt, graph);
        case 5: return bwd::pick_nt<5>(nt, graph);
        case 6: return bwd::pick_nt<6>(nt, graph);
        default: return nullptr;
    }
}

hipError_t launch_backward_reduce(const float* partial, float* dhyp, int nwg, int K, int P, int H,
                                  hipStream_t stream) {
    const int outs = K * H * 4;
    hipLaunchKernelGGL(bwd::reduce_kernel, dim3((outs + 3) / 4), dim3(256), 0, stream, partial, dhyp,
                       nwg, K, P, H);
    return hipGetLastError();
}

}  // namespace dadmm
