// dadmm_split.hip — the fused K-iteration forward for SMALL batches, columns split over workgroups.
//
// Reference semantics: unfolded_DLASSO.py:34-140 (DLASSO_unfolded.forward / compute_delta), the
// GNN variant's fixed clamps gnn_dlasso_models_progressive.py:205-232 — as dadmm_fused.hip.
//
// Why: dadmm_fused.hip gives one workgroup a 16-sample tile for all K iterations, so a batch of B
// samples fills ceil(B / 16) CUs: BASELINE configs[1] (B = 1024) runs 64 workgroups on 256 CUs at
// the per-tile time of the headline (0.50 ms per forward, 50 M ADMM-iters/s). Here a tile is cut
// into S = n_pad / 64 column slices, one workgroup each (B = 1024: 64 tiles x 4 = 256 workgroups):
//   * workgroup (tile, slice s) owns rows [64 s, 64 s + 64) of y, U, delta for all P agents of its
//     16 samples, and keeps its operator slice A_p[:, 64 s : 64 s + 64] (all P agents: 87 KB at
//     P = 5) RESIDENT IN LDS for the whole launch — no operand stream from L2 in the K loop;
//   * GEMM1 is split: each slice forms the partial c_s = A_p[:, slice] y_p[slice] (slice 0 seeds its
//     chains with -b), publishes it, and every slice sums R_p = ((c_0 + c_1) + c_2) + c_3 in that
//     fixed order (bit-identical in every slice; oracle_forward_f32_split restates it);
//   * GEMM2 G_p[slice] = A_p[:, slice]^T R_p, the gradient assembly, clamps, primal update, the
//     consensus (all P agents of a row live in this workgroup) and the dual update are
//     slice-local, exactly as in dadmm_fused.hip.
// The exchange (MI355X_MICROARCH.md "Workgroup dispatch ... inter-workgroup visibility", the R1
// form of cdna_hip_programming.md Guideline 16): a wave stores its 16 x 16 partial tile (1 KB,
// 16 B per lane) write-through (sc1), waits for it (s_waitcnt vmcnt), then one lane stores the
// tile's epoch word (sc1); the consumer wave of the same (agent, m-block) in every other slice
// polls those words with sc1 loads and then loads the tiles with sc1 loads (no acquire fence:
// every load of the handed-off bytes is an sc1 load to registers). Partials are double-buffered by
// epoch parity: a slice can run at most one epoch ahead of another (it cannot finish iteration k
// without every slice's partials of iteration k). Slices of one tile sit on blocks with equal
// blockIdx % 8 (one XCD under the observed round-robin placement: speed only, never correctness).
//
// Persistence and the exit condition: grid = G groups x S slices <= the CU count (one workgroup
// per CU by LDS), each group walking tiles g, g + G, ...; every wait is bounded (s_memrealtime): a
// wait that runs out (workgroups not co-resident: the device shared with other work) sets a
// launch-wide abort word and status bit 16, every wave then skips its remaining waits and runs to
// the end, and the caller's gated stepwise launch recomputes the batch exactly.
//
// Reduction order: every chain as dadmm_fused.hip (0,4,8,12, 1,5,... inside each 16-block, blocks
// ascending; -ffp-contract=off elsewhere), GEMM1 cut at slice boundaries as above.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dadmm_internal.h"
#include "dadmm_consensus.h"

namespace dadmm {
namespace split {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef __amdgpu_buffer_rsrc_t rsrc_t;
typedef __attribute__((address_space(1))) uint32_t gu32;
typedef const __attribute__((address_space(4))) float cfloat;

constexpr int NS = SPLIT_COLS;          // columns (rows of y) per slice
constexpr int WV = 8;                   // waves per workgroup (2 per SIMD)
// LDS row strides (floats). The operator slice is read two ways: GEMM1 takes A rows (ds_read_b128
// of 4 columns), GEMM2 takes A^T fragments (ds_read_b32 of one column, 4 rows apart per k-group):
// stride 68 keeps the b32 reads conflict-free (2 cycles) at a 2-way b128 conflict; 72 would swap
// them (scripts: the bank model of MI355X_MICROARCH.md §LDS).
constexpr int AST = NS + 4;
constexpr int YS = NS + 8;              // Ylds / Rlds: b128 reads conflict-free at 8 mod 64
constexpr int RS = M_PAD + 8;

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ rsrc_t make_rsrc(const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}
// aux: 16 = sc1 (write-through store / L1-bypassing load)
template <int AUX>
__device__ __forceinline__ f32x4 bload4(rsrc_t r, uint32_t voff) {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, AUX));
}
template <int AUX>
__device__ __forceinline__ void bstore4(f32x4 v, rsrc_t r, uint32_t voff) {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, v), r, voff, 0, AUX);
}
__device__ __forceinline__ float mclamp(float x, float lo, float hi) {
    return __builtin_amdgcn_fmed3f(x, lo, hi);
}
__device__ __forceinline__ bool finitef(float x) { return __builtin_isfinite(x); }

// Wait until the epoch words of every other slice of the wave's TH (agent, m-block) tiles reach
// `epoch`: lane t * S + s polls word s of tile t (sc1 loads; tile t's S words at words[t]), lanes
// of the wave's own slice skip, lane TH * S polls the launch-wide abort word. False when the
// launch is aborted (by this wave's deadline or another's). Wave-uniform.
template <int S, int TH>
__device__ __forceinline__ bool wait_tiles(const uint32_t* const (&words)[TH > 0 ? TH : 1], uint32_t epoch,
                                           uint32_t* abortw, uint64_t spin_ticks, int lane, int self) {
    const uint32_t* mine = nullptr;
#pragma unroll
    for (int t = 0; t < TH; ++t)
        if (lane >= t * S && lane < (t + 1) * S && lane - t * S != self) mine = words[t] + (lane - t * S);
    uint64_t t_end = 0;
    for (int spin = 0;; ++spin) {
        uint32_t v = epoch, ab = 0;
        if (mine != nullptr) v = __hip_atomic_load((gu32*)mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else if (lane == TH * S) ab = __hip_atomic_load((gu32*)abortw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (__ballot(v < epoch) == 0) return true;
        if (__ballot(ab != 0) != 0) return false;
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        if (spin == 0) t_end = now + spin_ticks;
        else if (now > t_end || spin > (1 << 22)) {   // (the count: a backstop for the clock)
            if (lane == 0) __hip_atomic_store((gu32*)abortw, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

// One wave's share of the split forward. HALF = w / 4: agents HALF, HALF + 2, ... (TH of them);
// GEMM1 m-block mb = w % 4 of those agents, GEMM2 / state n-tile nt = w % 4 of the slice.
template <int P, int NT, int GRAPH, int HALF>
__device__ __forceinline__ void split_body(const SplitArgs& sa, float* __restrict__ lds, const int w) {
    constexpr int S = NT;                            // slices of n_pad = 64 NT
    constexpr int NP = NT * 64;
    constexpr int TH = (P - HALF + 1) / 2;           // agents of this wave
    constexpr int THA = TH > 0 ? TH : 1;
    const FusedArgs& a = sa.f;
    float* __restrict__ Alds = lds;                          // [P][64 m][AST]  A_p[:, slice]
    float* __restrict__ Ylds = Alds + P * M_PAD * AST;       // [P][BT][YS]     y_k[slice]
    float* __restrict__ Rlds = Ylds + P * BT * YS;           // [P][BT][RS]     R_p = A_p y_p - b_p

    const int lane = threadIdx.x & 63;
    const int j = lane & 15, h = lane >> 4;
    const int mb = w & 3, nt = w & 3;
    const int G = sa.groups;
    // block -> (group g, slice): octets of 8 groups; inside an octet of width wd the blocks are
    // slice-major, so the S blocks of a group are wd apart (equal blockIdx % 8 for full octets)
    const int bid = blockIdx.x;
    const int oct = bid / (8 * S);
    const int r0 = bid - oct * 8 * S;
    const int wd = G - 8 * oct < 8 ? G - 8 * oct : 8;
    const int slice = r0 / wd;
    const int g = 8 * oct + r0 % wd;
    const int n = a.n, m = a.m, B = a.B;
    const uint32_t state_bytes = (uint32_t)((size_t)B * P * n * 4);

    // ---- the operator slice into LDS, once per launch (all 512 lanes) ----------------------
    for (int i = threadIdx.x; i < P * M_PAD * (NS / 4); i += WV * 64) {
        const int row = i / (NS / 4), c4 = i % (NS / 4);          // row = p * 64 + mi
        const f32x4 v = *(const f32x4*)(a.A + (size_t)row * NP + slice * NS + 4 * c4);
        *(f32x4*)(Alds + row * AST + 4 * c4) = v;
    }

    // the exchange: tile (g, slot, p, mb, s) of 256 floats (lane-linear 16 B), epoch words
    // [G][P][4][S], then the abort word
    const rsrc_t rX = make_rsrc(sa.xbuf, (uint32_t)((size_t)G * 2 * P * 4 * S * 1024));
    uint32_t* const abortw = sa.xflag + (size_t)G * P * 4 * S;
    auto xtile_off = [&](uint32_t slot, int p, int s2) -> uint32_t {
        return (uint32_t)((((((size_t)g * 2 + slot) * P + p) * 4 + mb) * S + s2) * 1024 + lane * 16);
    };
    auto flag_at = [&](int p) -> uint32_t* { return sa.xflag + (((size_t)g * P + p) * 4 + mb) * S; };

    uint32_t status = 0;
    bool aborted = false;
    {   // non-finite hyper-parameters make y_next NaN (reference guard :102): flag once
        bool bad_h = false;
        const int nh = a.K * a.hyp_rows * 4;
        for (int i = threadIdx.x; i < nh; i += WV * 64) bad_h |= !finitef(a.hyp[i]);
        status |= bad_h ? 8u : 0u;
    }
    const float dlim = a.variant != 0 ? 20.0f : __builtin_inff();

    int round = 0;
    for (int tile = g; tile < sa.tiles; tile += G, ++round) {
        const int s = tile * BT + j;                 // global sample
        const bool sv = s < B;
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
        // ---- state: rows n0 = 64 slice + 16 nt + 4h + r of this wave's agents ----------------
        const int n0 = slice * NS + 16 * nt + 4 * h;
        const bool rows_ok = n0 < n;
        float U[THA][4], D[THA][4];
        {
            const rsrc_t ry = make_rsrc(a.y0, state_bytes);
            const rsrc_t ru = make_rsrc(a.U0, state_bytes);
            const rsrc_t rd = make_rsrc(a.d0, state_bytes);
            bool bad_y = false, bad_u = false;
#pragma unroll
            for (int i = 0; i < TH; ++i) {
                const int p = HALF + 2 * i;
                const uint32_t off = (uint32_t)(((s * P + p) * n + n0) * 4);
                f32x4 vy = {0, 0, 0, 0}, vu = {0, 0, 0, 0}, vd = {0, 0, 0, 0};
                if (rows_ok) {
                    vy = bload4<0>(ry, off);
                    vu = bload4<0>(ru, off);
                    vd = bload4<0>(rd, off);
                }
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    bad_y |= !finitef(vy[r]);
                    bad_u |= !finitef(vu[r]);
                    U[i][r] = vu[r];
                    D[i][r] = vd[r];
                }
                *(f32x4*)(Ylds + (p * BT + j) * YS + 16 * nt + 4 * h) = vy;
            }
            // reference guards at the top of an iteration (:55-61) can only fire at k = 0 (see
            // dadmm_fused.hip); the caller's gated recomputation applies them
            status |= (bad_y ? 1u : 0u) | (bad_u ? 2u : 0u);
        }
        // -b seeds of this wave's GEMM1 chains (slice 0 only; the other slices' chains start at +0)
        f32x4 bseed[THA];
#pragma unroll
        for (int i = 0; i < TH; ++i) {
            const int p = HALF + 2 * i;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int mi = 16 * mb + 4 * h + r;
                bseed[i][r] = (slice == 0 && sv && mi < m) ? -a.b[((size_t)s * P + p) * m + mi] : 0.0f;
            }
        }
        const uint32_t voffY = (uint32_t)((s * P * n + n0) * 4);
        float et_prev[THA];
        float vclip_prev = 0.0f;
#pragma unroll
        for (int i = 0; i < TH; ++i) et_prev[i] = 0.0f;
        __syncthreads();

        for (int k = 0; k < a.K; ++k) {
            const uint32_t epoch = (uint32_t)(round * a.K + k + 1);
            const uint32_t slot = (epoch - 1) & 1u;
            float al[THA], ta[THA], rh[THA], et[THA];
#pragma unroll
            for (int i = 0; i < TH; ++i) {
                const int p = HALF + 2 * i;
                const cfloat* hp = (const cfloat*)a.hyp + ((size_t)k * a.hyp_rows + (a.hyp_rows == 1 ? 0 : p)) * 4;
                al[i] = hp[0]; ta[i] = hp[1]; rh[i] = hp[2]; et[i] = hp[3];
            }
            float gclip, vclip;
            if (a.variant == 0) {
                gclip = fmaxf(1.0f, 30.0f - (float)k);          // unfolded_DLASSO.py:80
                vclip = fmaxf(10.0f, 200.0f - (float)(k * 3));  // :92
            } else {
                gclip = 10.0f;                                   // gnn_dlasso_models_progressive.py:212
                vclip = 100.0f;                                  // :224, :232
            }

            // ---- GEMM1 partials c_s = A_p[:, slice] y_p[slice] (+ -b in slice 0), published one
            //      chain at a time: stored write-through (sc1); chain i-1's epoch word after chain
            //      i's store (every VMEM op but that store has completed: vmcnt counts in order) --
            f32x4 part[THA];
            // the wave's priority raised while it issues its MFMA chains (the arbiter then prefers
            // it, so the matrix pipe stays fed while the SIMD's other wave runs VALU work): 187.8-191.1
            // vs 192.3-196.9 us per configs[1] forward; the second-dispatched half raised for the
            // whole loop instead (dadmm_fused.hip's choice) measured 216-220 us
            __builtin_amdgcn_s_setprio(2);
#pragma unroll
            for (int i = 0; i < TH; ++i) {
                const int p = HALF + 2 * i;
                f32x4 acc = bseed[i];
#pragma unroll
                for (int t = 0; t < NS / 16; ++t) {
                    const f32x4 av = *(const f32x4*)(Alds + (p * M_PAD + 16 * mb + j) * AST + 16 * t + 4 * h);
                    const f32x4 bv = *(const f32x4*)(Ylds + (p * BT + j) * YS + 16 * t + 4 * h);
#pragma unroll
                    for (int r = 0; r < 4; ++r) acc = mfma4(av[r], bv[r], acc);
                }
                part[i] = acc;
                bstore4<16>(acc, rX, xtile_off(slot, p, slice));
                if (i > 0) {
                    asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
                    if (lane == 0)
                        __hip_atomic_store((gu32*)(flag_at(HALF + 2 * (i - 1)) + slice), epoch,
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            __builtin_amdgcn_s_setprio(0);
            if (TH > 0) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (lane == 0)
                    __hip_atomic_store((gu32*)(flag_at(HALF + 2 * (TH - 1)) + slice), epoch,
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }

            // ---- dual update deferred from iteration k-1 (:95-99), under the exchange: delta_k =
            //      2 L y_k for the wave's 4 rows (all P agents of a row are in Ylds), U_k = clamp(U
            //      + delta eta); needed only by this iteration's primal updates -------------------
            if (k > 0) {
                float yy[P][4], dd[P][4];
#pragma unroll
                for (int p = 0; p < P; ++p) {
                    const f32x4 v = *(const f32x4*)(Ylds + (p * BT + j) * YS + 16 * nt + 4 * h);
#pragma unroll
                    for (int r = 0; r < 4; ++r) yy[p][r] = v[r];
                }
                consensus_any<P, GRAPH>(yy, dd, msk, ord);
#pragma unroll
                for (int i = 0; i < TH; ++i) {
                    const int p = HALF + 2 * i;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float d = mclamp(dd[p][r], -dlim, dlim);
                        U[i][r] = mclamp(U[i][r] + d * et_prev[i], -vclip_prev, vclip_prev);
                        D[i][r] = d;
                    }
                }
            }

            // ---- R_p = ((c_0 + c_1) + c_2) + ... for the wave's (agent, m-block) tiles -> Rlds:
            //      one poll over all of them, then every remote partial load in flight at once
            //      (a per-agent pipeline with LDS arrival counters under GEMM2 measured slower:
            //      206 vs 198 us per forward at configs[1]) ----------------------
            {
                const uint32_t* words[THA];
#pragma unroll
                for (int i = 0; i < TH; ++i) words[i] = flag_at(HALF + 2 * i);
                if (!aborted) aborted = !wait_tiles<S, TH>(words, epoch, abortw, sa.spin_ticks, lane, slice);
            }
            f32x4 c[THA][S];
#pragma unroll
            for (int i = 0; i < TH; ++i)
#pragma unroll
                for (int s2 = 0; s2 < S; ++s2)
                    c[i][s2] = s2 == slice ? part[i] : bload4<16>(rX, xtile_off(slot, HALF + 2 * i, s2));
#pragma unroll
            for (int i = 0; i < TH; ++i) {
                const int p = HALF + 2 * i;
                f32x4 rsum = c[i][0];
#pragma unroll
                for (int s2 = 1; s2 < S; ++s2) rsum = rsum + c[i][s2];
                *(f32x4*)(Rlds + (p * BT + j) * RS + 16 * mb + 4 * h) = rsum;
            }
            __syncthreads();

            // ---- GEMM2 G_p[n-tile nt] = A_p[:, slice]^T R_p, gradient assembly, clamps, primal
            //      update (:69-93) -> Ylds and Y[k] ---------------------------------------------
            const rsrc_t rY = make_rsrc(a.Y + (size_t)k * B * P * n, state_bytes);
            bool bad_g = false;
            __builtin_amdgcn_s_setprio(2);
#pragma unroll
            for (int i = 0; i < TH; ++i) {
                const int p = HALF + 2 * i;
                f32x4 gp = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
                for (int t = 0; t < M_PAD / 16; ++t) {
                    const f32x4 rv = *(const f32x4*)(Rlds + (p * BT + j) * RS + 16 * t + 4 * h);
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        gp = mfma4(Alds[(p * M_PAD + 16 * t + 4 * h + r) * AST + 16 * nt + j], rv[r], gp);
                }
                float* yrow = Ylds + (p * BT + j) * YS + 16 * nt + 4 * h;
                const f32x4 yk = *(const f32x4*)yrow;
                f32x4 yn;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float yv = yk[r];
                    // grad = (AtAy - Atb) + sign(y)*tau + U*deg + delta*rho, left to right (:73-77)
                    float gr = gp[r];
                    gr = gr + sign_times(yv, ta[i]);
                    gr = gr + U[i][r] * dg[p];
                    gr = gr + D[i][r] * rh[i];
                    bad_g |= (gr != gr);                            // :84 guard (flag only)
                    gr = mclamp(gr, -gclip, gclip);                 // :80-81
                    float v = yv - al[i] * gr;                      // :89
                    yn[r] = mclamp(v, -vclip, vclip);               // :92-93
                }
                *(f32x4*)yrow = yn;
                bstore4<16>(yn, rY, rows_ok ? voffY + (uint32_t)(p * n * 4) : 0x80000000u);
            }
            __builtin_amdgcn_s_setprio(0);
            status |= bad_g ? 4u : 0u;
#pragma unroll
            for (int i = 0; i < TH; ++i) et_prev[i] = et[i];
            vclip_prev = vclip;
            __syncthreads();
        }

        if (a.U_out != nullptr) {
            // the dual update of the last iteration (deferred like the others)
            float yy[P][4], dd[P][4];
#pragma unroll
            for (int p = 0; p < P; ++p) {
                const f32x4 v = *(const f32x4*)(Ylds + (p * BT + j) * YS + 16 * nt + 4 * h);
#pragma unroll
                for (int r = 0; r < 4; ++r) yy[p][r] = v[r];
            }
            consensus_any<P, GRAPH>(yy, dd, msk, ord);
            const rsrc_t rU = make_rsrc(a.U_out, state_bytes);
#pragma unroll
            for (int i = 0; i < TH; ++i) {
                const int p = HALF + 2 * i;
                f32x4 v;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float d = mclamp(dd[p][r], -dlim, dlim);
                    v[r] = mclamp(U[i][r] + d * et_prev[i], -vclip_prev, vclip_prev);
                }
                if (rows_ok) bstore4<0>(v, rU, (uint32_t)(((s * P + p) * n + n0) * 4));
            }
        }
        __syncthreads();   // Ylds is rewritten by the next tile's initial state
    }
    if (aborted) status |= 16u;   // the exact guarded recomputation redoes the batch
    if (a.status != nullptr) {
        uint32_t wst = status;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) wst |= __shfl_xor(wst, off);
        if (lane == 0 && wst) atomicOr((unsigned int*)a.status, wst);
    }
}

template <int P, int NT, int GRAPH>
__global__ __launch_bounds__(WV * 64) void split_forward_kernel(SplitArgs sa) {
    __shared__ __attribute__((aligned(16))) float lds[P * M_PAD * AST + P * BT * (YS + RS)];
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (w < 4)
        split_body<P, NT, GRAPH, 0>(sa, lds, w);
    else
        split_body<P, NT, GRAPH, 1>(sa, lds, w);
}

template <int P, int NT, int GRAPH>
hipError_t launch_split(const SplitArgs& sa, hipStream_t stream) {
    hipLaunchKernelGGL((split_forward_kernel<P, NT, GRAPH>), dim3(sa.groups * NT), dim3(WV * 64), 0,
                       stream, sa);
    return hipGetLastError();
}

template <int P, int NT>
split_fn_ptr pick_graph(int graph) {
    switch (graph) {
        case GRAPH_SHARED: return &launch_split<P, NT, GRAPH_SHARED>;
        case GRAPH_LANE: return &launch_split<P, NT, GRAPH_LANE>;
        case GRAPH_ORDERED: return &launch_split<P, NT, GRAPH_ORDERED>;
        default: return nullptr;
    }
}

template <int P>
split_fn_ptr pick_nt(int nt, int graph) {
    if (nt == 2) return pick_graph<P, 2>(graph);
    if (nt == 4) return pick_graph<P, 4>(graph);
    return nullptr;
}

}  // namespace split

// Instantiated shapes: P = 1..6, n_pad = 128 or 256 (S = 2 or 4 slices of 64 columns), m_pad = 64.
split_fn_ptr find_split(int P, int nt, int graph) {
    switch (P) {
        case 1: return split::pick_nt<1>(nt, graph);
        case 2: return split::pick_nt<2>(nt, graph);
        case 3: return split::pick_nt<3>(nt, graph);
        case 4: return split::pick_nt<4>(nt, graph);
        case 5: return split::pick_nt<5>(nt, graph);
        case 6: return split::pick_nt<6>(nt, graph);
        default: return nullptr;
    }
}

}  // namespace dadmm
