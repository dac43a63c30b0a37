// dadmm_stream.hip — the whole K-iteration forward in ONE launch for the shapes whose per-sample
// state does not fit on chip (BASELINE configs[2]: P = 16, n = 512, m = 64): the state streams
// through HBM exactly once per iteration, R_k stays in registers between iterations.
//
// Reference semantics: unfolded_DLASSO.py:53-107 / :127-140 (and the GNN variant's clamps,
// gnn_dlasso_models_progressive.py:205-232), in the order of oracle_forward_f32.
//
// Workgroup = 16 samples (the MFMA N dimension) x all P agents, 8 waves; wave w owns agents
// w, w + 8 (PW per wave). It walks the columns in 32-column blocks ("steps"), phase after phase:
//   phase -1:       GEMM1 only: R_0 = A_p y_0 - b_p accumulated block by block;
//   phase k < K:    per block: delta_k from y_k of every agent (visit lists over the LDS block;
//                   k = 0: d0), the deferred dual update U_k = clamp(U_{k-1} + delta_k eta_{k-1})
//                   (k = 0: U0), G = A_p^T R_k (GEMM2, R_k held in registers), the gradient, the
//                   primal update y_{k+1} -> Y[k], and GEMM1 of the NEXT iteration on the fly:
//                   R_{k+1} += A_p[:, block] y_{k+1}[block] (y_{k+1} goes from the update's
//                   registers straight into the MFMA B operand);
//   phase K:        the final dual update U_K -> U_out (only when U_out is requested).
// The fma chains are the oracle's: GEMM1 rows from -b over the columns in ascending 16-blocks,
// 0,4,8,12,1,5,... inside each; GEMM2 columns from +0 over the rows the same way. Because a
// block's GEMM1 continues the same accumulator chain in ascending column order, accumulating
// R_{k+1} across the blocks of iteration k is the oracle's chain exactly.
//
// HBM per sample-iteration: y_k read once (the block of every agent, staged in LDS by LDS-DMA,
// three blocks in flight), U_{k-1} read and U_k written, y_{k+1} written, b once per iteration —
// SURVEY.md §8(d)'s algorithmic 4 P (4n + m) bytes; no delta / R round trips, no second y read.
// The operator (A_p and A_p^T, 2 x 128 KB per agent at configs[2]) is read from L2.
//
// Guards: like the fused and tiled kernels, this path ORs the status bits of every case where one
// of the reference's batch-global NaN/Inf guards would fire, and the caller's gated stepwise
// recomputation redoes such a batch exactly. On guard-free inputs the output is bit-identical to
// oracle_forward_f32 and to the other paths.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <type_traits>

#include "dadmm_internal.h"

namespace dadmm {
namespace stream {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __amdgpu_buffer_rsrc_t rsrc_t;
typedef __attribute__((address_space(3))) void lds_void;

constexpr int NW = 8;            // waves per workgroup (the default form; 16: one agent per wave)
constexpr int CT = 2;            // 16-column MFMA tiles per step
constexpr int CW = 16 * CT;      // columns per step
constexpr int SLOTS = 3;         // y-block ring: the block of step bs + 2 is loaded during step bs
// Decisions measured at configs[2] (round 6 removed the A/B switches):
//   * the wave's priority raised while it issues an MFMA chain (the arbiter then prefers it, so
//     the matrix pipe is fed while the other wave of the SIMD runs its VALU work): 6.03-6.07 vs
//     6.09-6.14 ms, bit-identical (profiles/r03/stream_prio_r03.jsonl);
//   * GEMM2's A^T fragments read from the A_pad copy (4-byte loads, four 64-byte row segments per
//     instruction) instead of At_pad: the tile's GEMM1 reads the same 4 KB of A, so the operator
//     kept in L2 halves: 5.85-5.90 vs 6.04-6.10 ms (profiles/r04/variants_r04c.txt);
//   * default cache policy on the state streams (non-temporal: 6.04 vs 5.96 ms); the stores of a
//     tile issued right after it (behind the next tile's loads: 17 spilled VGPRs, 5.99-6.04 vs
//     5.87-5.89 ms); the two waves of a SIMD in the same phase order; no extra operand prefetch.
#define DADMM_STR_(x) #x
#define DADMM_STR(x) DADMM_STR_(x)

__device__ __forceinline__ rsrc_t make_rsrc(const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// A raw buffer descriptor as four SGPRs (for inline asm): base, stride 0, num_records = bytes,
// the gfx950 default data format (the word __builtin_amdgcn_make_buffer_rsrc takes).
__device__ __forceinline__ i32x4 rsrc_words(const void* base, uint32_t bytes) {
    const uint64_t b = (uint64_t)base;
    return (i32x4){(int)(uint32_t)b, (int)(uint32_t)(b >> 32) & 0xffff, (int)bytes, 0x00020000};
}
// LDS-DMA of 16 bytes per lane into LDS at m0 + 16 lane, issued from inline asm: the compiler's
// wait analysis then does not treat every later LDS read as a possible alias of the copy (it would
// wait for the whole copy before the first such read, i.e. two steps too early); the kernel waits
// for its copies itself (wait_prev_step). The compiler's own vmcnt waits stay correct: a copy it
// does not count only makes them wait longer. (m0 is a reserved register, so the compiler warns
// about the clobber; no other instruction of this kernel reads m0 — checked in its ISA.)
__device__ __forceinline__ void dma16(uint32_t lds_addr, uint32_t voff, i32x4 rsrc) {
    asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen" " lds"
                 :
                 : "s"(lds_addr), "v"(voff), "s"(rsrc)
                 : "memory", "m0");
}
// a - b on both halves (v_pk_add_f32 with the second operand negated: a + (-b) == a - b exactly)
__device__ __forceinline__ f32x2 pk_sub(f32x2 a, f32x2 b) {
    f32x2 r;
    asm("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float tclamp(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }
__device__ __forceinline__ bool finitef(float x) { return __builtin_isfinite(x); }
__device__ __forceinline__ bool finite4(f32x4 v) {
    return finitef(v[0]) && finitef(v[1]) && finitef(v[2]) && finitef(v[3]);
}

__device__ __forceinline__ void clips(int variant, int k, float& gclip, float& vclip) {
    if (variant == 0) {
        gclip = fmaxf(1.0f, 30.0f - (float)k);          // unfolded_DLASSO.py:80
        vclip = fmaxf(10.0f, 200.0f - (float)(k * 3));  // unfolded_DLASSO.py:92
    } else {
        gclip = 10.0f;                                   // gnn_dlasso_models_progressive.py:212
        vclip = 100.0f;                                  // :224, :232
    }
}

// Visit-table row length: an agent's list holds <= 2 P entries (each neighbour from both ends of
// the edge, a self-loop twice). Rows are padded with the agent itself (a term y_p - y_p = +0,
// which leaves the accumulator unchanged: it starts at +0 and is never -0) to a multiple of 4
// entries whose count / 4 is odd (the 16 samples' rows then sit in distinct LDS banks). An entry
// is the byte offset q * 2048 of neighbour q's rows in a ring slot: a visit is one address add.
__host__ __device__ constexpr int vt_stride(int P) {
    return 4 * (((2 * P + 3) / 4) | 1);
}
constexpr int slot_floats(int NWT, int PW) { return NWT * PW * CT * 64 * 4; }
size_t lds_bytes(int NWT, int PW, int P) {
    const int PA = NWT * PW;
    return 4 * (size_t)SLOTS * slot_floats(NWT, PW) + 4 * (size_t)PA * BT * vt_stride(P) + 4 * (size_t)PA;
}

// Step bs's block in the ring: chunk (q, ct, bq, j) = 16 bytes of agent q, sample j, columns
// c0 + 16 ct + 4 bq .. + 3, at chunk index ((q CT + ct) 4 + bq) 16 + j. One LDS-DMA instruction
// fills the 64 chunks of one (q, ct) with lane l = 16 bq + j (lane-linear, the DMA's constraint),
// and a lane's own read of agent q is chunk (q CT + ct) 64 + lane: conflict-free for any per-lane q.
//
// A wave's work in a step is PW x CT tiles (agent, 16 columns); the global operands of a tile (its
// A^T and A rows, U_{k-1}, d0) are fetched into a two-deep register ring during the previous tile
// (across steps and phases), so they land under that tile's MFMAs and the next consensus walk.
struct Ring {
    f32x4 at[4], am[4], u, d;
};

// At the top of step bs the DMA of step bs (issued at the top of step bs - 2) and every store of
// step bs - 2 must have completed. Vector-memory operations complete in issue order, so it
// suffices to wait until no more than the count of operations step bs - 1 issues at least are
// outstanding: per previous phase kind (a wave with one agent, the last two steps without DMA).
__device__ __forceinline__ void wait_prev_step(int kprev, int K) {
    if (kprev < 0) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
    else if (kprev < K - 1) asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
    else if (kprev == K - 1) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
}

template <int NWT, int PW, bool REC = false>
__global__ __launch_bounds__(64 * NWT) void stream_kernel(TiledArgs a) {
    constexpr int NW = NWT;
    constexpr bool RING = NWT == 8;   // the operand ring one tile ahead (two waves per SIMD)
    extern __shared__ __attribute__((aligned(16))) float lds[];
    constexpr int PA = NW * PW;
    constexpr int SF = slot_floats(NWT, PW);
    const int P = a.P, n = a.n, m = a.m, B = a.B, NP = a.n_pad, K = a.K, H = a.hyp_rows;
    const int DP = vt_stride(P);
    uint32_t* vt = (uint32_t*)(lds + SLOTS * SF);        // [PA][BT][DP] visit rows (byte offsets)
    int* dmx = (int*)(vt + PA * BT * DP);                // [PA] longest row of each agent
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int j = lane & 15, bq = lane >> 4;             // sample in the tile, 4-column group
    const int s0 = blockIdx.x * BT, s = s0 + j;
    const bool sok = s < B;
    const int sc = sok ? s : 0;
    const size_t S = (size_t)B * P * n;
    const uint32_t s_bytes = (uint32_t)(S * 4);          // one iterate (< 2^31: the ABI checks)
    const int NB = NP / CW;
    const int kend = a.U_out != nullptr ? K : K - 1;     // phase K: the final dual update only
    uint32_t status = 0;

    // ---- the tile's visit lists -> LDS rows (padded with the agent itself)
    if (threadIdx.x < PA) dmx[threadIdx.x] = 0;
    __syncthreads();
    if (threadIdx.x < PA * BT) {
        const int p = threadIdx.x / BT, sl = threadIdx.x % BT;
        uint32_t* row = vt + (p * BT + sl) * DP;
        int len = 0;
        if (p < P && s0 + sl < B) {
            const int g = a.graph_shared ? p : (s0 + sl) * P + p;
            const int v0 = a.vptr[g];
            len = a.vptr[g + 1] - v0;
            if (len > DP) {   // cannot come from a graph on P nodes; the exact path takes it
                len = DP;
                status |= 16u;
            }
            for (int t = 0; t < len; ++t) row[t] = (uint32_t)a.vq[v0 + t] * (CT * 64 * 16);
        }
        for (int t = len; t < DP; ++t) row[t] = (uint32_t)p * (CT * 64 * 16);
        atomicMax(&dmx[p], len);
    }

    float dg[PW];
#pragma unroll
    for (int ai = 0; ai < PW; ++ai) {
        const int p = w + NW * ai;
        dg[ai] = (sok && p < P) ? a.deg[(a.graph_shared ? 0 : s * P) + p] : 0.0f;
    }
    auto col_ok = [&](int c0, int ct) { return sok && c0 + 16 * ct + 4 * bq < n; };
    auto elem = [&](int p, int c0, int ct) {   // [s][p][col] of this lane's 4 columns
        return ((size_t)sc * P + p) * n + c0 + 16 * ct + 4 * bq;
    };

    // LDS-DMA of step bs's block (this wave's own agents; agents >= P and samples >= B get an
    // offset past the range, which the hardware returns as zeros)
    auto dma = [&](int k, int blk, float* slot) {
        const float* src = k <= 0 ? a.y0 : a.Y + (size_t)(k - 1) * S;
        const i32x4 r = rsrc_words(src, (k <= kend) ? s_bytes : 0u);
#pragma unroll
        for (int ai = 0; ai < PW; ++ai) {
            const int q = w + NW * ai;
#pragma unroll
            for (int ct = 0; ct < CT; ++ct) {
                const uint32_t off = (q < P && col_ok(blk * CW, ct))
                                         ? (uint32_t)(elem(q, blk * CW, ct) * 4) : 0x80000000u;
                dma16((uint32_t)(uintptr_t)(lds_void*)(slot + 4 * ((q * CT + ct) * 64)), off, r);
            }
        }
    };
    // operator buffers: per-lane offsets fixed for the whole launch, the rest in SGPRs
    // Every operand load is issued unconditionally (a zero-size descriptor where a phase or an absent
    // agent p >= P needs none: it returns zeros without a memory access), so that no ring register
    // is merged from two different loads across a branch (each such merge costs a full vmcnt wait).
    // (descriptors are built per use from a selected base and size: selecting between descriptor
    // values puts them on the stack)
    const uint32_t at_bytes = (uint32_t)((size_t)P * NP * 64 * 4);
    // launch-constant descriptors; a phase or lane without the operand gets an out-of-range offset
    // (zeros, no memory access) instead of a different descriptor
    const rsrc_t dA = make_rsrc(a.A, at_bytes);
    const rsrc_t dd0 = make_rsrc(a.d0, s_bytes), db = make_rsrc(a.b, (uint32_t)((size_t)B * P * m * 4));
    const uint32_t vam = (uint32_t)((j * NP + 4 * bq) * 4);
    // the global operands of tile i = (agent i / CT, columns 16 (i % CT)) of step bs: fetch_a (A^T
    // rows, U_{k-1}, d0) is issued at the start of the previous tile, fetch_m (A rows, needed only at
    // the tile's end) after the previous tile's GEMM2, when its A^T registers are free
    auto fetch_a = [&](int k, int c0, int i, Ring& r) {
        const int ai = i / CT, ct = i % CT;
        const int p = w + NW * ai;
        const bool pin = p < P;
        const int pc = pin ? p : 0;
        // lane (j, bq), m-block t: A_p rows 16 t + 4 bq + r, column c0 + 16 ct + j
        const uint32_t voa = (k >= 0 && k < K && pin) ? (uint32_t)(((4 * bq) * NP + j) * 4) : 0x80000000u;
        const uint32_t sba = (uint32_t)((((size_t)pc * 64) * NP + c0 + 16 * ct) * 4);
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int r4 = 0; r4 < 4; ++r4)
                r.at[t][r4] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                    dA, voa, sba + (uint32_t)((16 * t + r4) * NP * 4), 0));   // row step in soffset
        const uint32_t off = (pin && col_ok(c0, ct)) ? (uint32_t)(elem(pc, c0, ct) * 4) : 0x80000000u;
        // U_{k-1} (k = 0: U0 itself; k = 1: U_0 = U0)
        r.u = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
            make_rsrc(k <= 1 ? a.U0 : a.Ubuf[0], s_bytes), k >= 0 ? off : 0x80000000u, 0, 0));
        r.d = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(dd0, k == 0 ? off : 0x80000000u, 0,
                                                                              0));
    };
    auto fetch_m = [&](int k, int c0, int i, Ring& r) {
        const int ai = i / CT, ct = i % CT;
        const int p = w + NW * ai;
        const bool pin = p < P;
        const int pc = pin ? p : 0;
        const bool ok = k < K - 1 && pin;
#pragma unroll
        for (int t = 0; t < 4; ++t)
            r.am[t] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                dA, ok ? vam + (uint32_t)(16 * t * NP * 4) : 0x80000000u,
                (uint32_t)((((size_t)pc * 64) * NP + c0 + 16 * ct) * 4), 0));
    };

    f32x4 Rk[PW][4], Rn[PW][4];
#pragma unroll
    for (int ai = 0; ai < PW; ++ai)
#pragma unroll
        for (int t = 0; t < 4; ++t) Rk[ai][t] = Rn[ai][t] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
    bool bad_y0 = false, bad_u0 = false, bad_g = false, bad_y = false, bad_h = false;
    float al[PW], ta[PW], rh[PW], etp[PW];
    float gclip = 0.0f, vclip = 0.0f, vclip_prev = 0.0f;

    // tile i of step bs (phase k, columns c0), operands in r; pre() issues the next tile's A^T rows,
    // U and d0 after the consensus walk, mid() its A rows after GEMM2.
    // Straight-line in every phase: no global load or store sits under a branch (a zero-size descriptor
    // or an out-of-range offset disables one), because the compiler's wait analysis turns a memory
    // operation on one path of a merge into a full vmcnt wait after it. GEMM2 and the update run
    // in the phases without a primal update too (on A^T = 0; nothing is stored).
    auto compute = [&](int k, int c0, const float* ys, int i, Ring& r, auto&& pre, auto&& mid) {
        const int ai = i / CT, ct = i % CT;
        const int p = w + NW * ai;
        const bool okc = p < P && col_ok(c0, ct);   // agents p >= P: work on zeros, nothing stored
        const uint32_t soff = okc ? (uint32_t)(elem(p, c0, ct) * 4) : 0x80000000u;
        const f32x4 yo = *(const f32x4*)(ys + 4 * ((p * CT + ct) * 64 + lane));
        // delta_k = compute_delta(y_k) (unfolded_DLASSO.py:127-140): acc + (y_p - y_q) over p's visit
        // row, four entries per LDS word (no walk in phases -1 and 0)
        const int D = (k >= 1) ? __builtin_amdgcn_readfirstlane(dmx[p]) : 0;   // 0 for p >= P
        const uint32_t* vrow = vt + (p * BT + j) * DP;
        const char* ybase = (const char*)(ys + 4 * (ct * 64 + lane));
        auto walk = [&]() {
            f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
            for (int t4 = 0; t4 < D; t4 += 4) {
                const uint4 qo = *(const uint4*)(vrow + t4);
                const uint32_t qa[4] = {qo.x, qo.y, qo.z, qo.w};
                f32x4 yqs[4];   // the four neighbour reads in flight together
#pragma unroll
                for (int u = 0; u < 4; ++u) yqs[u] = *(const f32x4*)(ybase + qa[u]);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const f32x4 yq = yqs[u];
                    const f32x2 d0 = pk_sub((f32x2){yo[0], yo[1]}, (f32x2){yq[0], yq[1]});
                    const f32x2 d1 = pk_sub((f32x2){yo[2], yo[3]}, (f32x2){yq[2], yq[3]});
                    acc = acc + (f32x4){d0[0], d0[1], d1[0], d1[1]};
                }
            }
            return acc;
        };
        // GEMM2: A_p^T R_k, this tile's columns (16 dependent MFMAs, no input from the walk).
        // (The two waves of a SIMD taking the walk and GEMM2 in opposite orders measured 6.18-6.31
        // vs 6.13-6.19 ms.)
        auto gemm2 = [&]() {
            __builtin_amdgcn_s_setprio(1);
            f32x4 g = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int r4 = 0; r4 < 4; ++r4) g = mfma4(r.at[t][r4], Rk[ai][t][r4], g);
            __builtin_amdgcn_s_setprio(0);
            return g;
        };
        const f32x4 acc = walk();
        const f32x4 gc = gemm2();
        // the next tile's A^T rows, U, d0 and A rows: issued at one program point (outside the branch)
        pre();
        mid();
        f32x4 dv = k == 0 ? r.d : acc;
        if (k >= 1 && a.variant != 0) {
#pragma unroll
            for (int r4 = 0; r4 < 4; ++r4) dv[r4] = tclamp(dv[r4], -20.0f, 20.0f);   // :229
        }
        // the dual update of iteration k - 1 (:98-99), deferred to here (k = 0: U0 as given)
        f32x4 uv;
#pragma unroll
        for (int r4 = 0; r4 < 4; ++r4) {
            const float un = tclamp(r.u[r4] + dv[r4] * etp[ai], -vclip_prev, vclip_prev);
            uv[r4] = k >= 1 ? un : r.u[r4];
        }
        bad_u0 |= k == 0 && okc && !finite4(uv);
        // U_k after the next tile's A rows are issued: vector-memory operations complete in order,
        // so a load issued after a store waits for it
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, uv),
                                               make_rsrc(k == K ? a.U_out : a.Ubuf[0], s_bytes),
                                               k >= 1 ? soff : 0x80000000u, 0, 0);
        const bool upd = k >= 0 && k < K;
        f32x4 yn, grc;
#pragma unroll
        for (int r4 = 0; r4 < 4; ++r4) {   // :69-93, left to right
            const float y = yo[r4];
            float gr = gc[r4] + sign_times(y, ta[ai]);
            gr = gr + uv[r4] * dg[ai];
            gr = gr + dv[r4] * rh[ai];
            grc[r4] = gr;
            bad_g |= upd && okc && gr != gr;
            gr = tclamp(gr, -gclip, gclip);
            const float v = tclamp(y - al[ai] * gr, -vclip, vclip);
            bad_y |= upd && okc && !finitef(v);
            yn[r4] = okc ? v : 0.0f;
        }
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, yn),
                                               make_rsrc(a.Y + (size_t)(upd ? k : 0) * S, s_bytes),
                                               upd ? soff : 0x80000000u, 0, 0);
        if constexpr (REC) {   // the adjoint's trajectory: Grec[k] (pre-clamp gradient), Urec[k] = U_k
            const size_t kS = (size_t)(upd ? k : 0) * S;
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, grc),
                                                   make_rsrc(a.Grec + kS, s_bytes), upd ? soff : 0x80000000u, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, uv),
                                                   make_rsrc(a.Urec + kS, s_bytes), upd ? soff : 0x80000000u, 0, 0);
        }
        bad_y0 |= k == -1 && okc && !finite4(yo);   // the :55 guard on y_0
        // GEMM1: R_{k+1} += A_p[:, tile] y_{k+1}[tile] (phase -1: R_0 from y_0)
        const f32x4 gin = k == -1 ? yo : yn;
        if (k < K - 1) {
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int r4 = 0; r4 < 4; ++r4) Rn[ai][t] = mfma4(r.am[t][r4], gin[r4], Rn[ai][t]);
            __builtin_amdgcn_s_setprio(0);
        }
    };

    Ring r0, r1;
    dma(-1, 0, lds);          // (NB >= 4: stream_applies)
    dma(-1, 1, lds + SF);
    if constexpr (RING) {
        fetch_a(-1, 0, 0, r0);
        fetch_m(-1, 0, 0, r0);
    }
    int bs = 0;
    int slot = 0;                                        // bs % SLOTS
    int dk = -1, dblk = 2;                               // phase / block of step bs + 2
    for (int k = -1; k <= kend; ++k) {
        // phase setup: hyper-parameters, clips, R_k <- R_{k+1}, the GEMM1 chains from -b
        const int kc = k < 0 ? 0 : (k < K ? k : K - 1), kp = k < 1 ? 0 : k - 1;
        float gtmp;
        clips(a.variant, kc, gclip, vclip);
        clips(a.variant, kp, gtmp, vclip_prev);
#pragma unroll
        for (int ai = 0; ai < PW; ++ai) {
            const int p = w + NW * ai;
            const int hp = H == 1 ? 0 : (p < P ? p : 0);
            const float* hk = a.hyp + ((size_t)kc * H + hp) * 4;
            al[ai] = hk[0]; ta[ai] = hk[1]; rh[ai] = hk[2];
            if (k >= 0 && k < K && p < P)
                bad_h |= !(finitef(hk[0]) && finitef(hk[1]) && finitef(hk[2]) && finitef(hk[3]));
            etp[ai] = a.hyp[((size_t)kp * H + hp) * 4 + 3];
        }
        if (k >= 0) {
#pragma unroll
            for (int ai = 0; ai < PW; ++ai)
#pragma unroll
                for (int t = 0; t < 4; ++t) Rk[ai][t] = Rn[ai][t];
        }
        {   // (unconditional: Rn is dead in phases K - 1 and K)
            const bool bk = k < K - 1;
#pragma unroll
            for (int ai = 0; ai < PW; ++ai) {
                const int p = w + NW * ai;
#pragma unroll
                for (int t = 0; t < 4; ++t)
#pragma unroll
                    for (int r4 = 0; r4 < 4; ++r4) {
                        const int row = 16 * t + 4 * bq + r4;
                        const uint32_t boff = (bk && sok && p < P && row < m)
                                                  ? (uint32_t)((((size_t)s * P + p) * m + row) * 4) : 0x80000000u;
                        Rn[ai][t][r4] = -__builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(db, boff, 0, 0));
                    }
            }
        }
        for (int blk = 0; blk < NB; ++blk, ++bs) {
            // step bs's block has landed (every wave's DMA), every wave is done with step bs - 1's
            // slot, and this wave's stores of step bs - 2 have completed (the ring reads Y[k - 1]'s
            // block NB - 2 >= 2 steps after it was written)
            {
                if (bs > 0) wait_prev_step(blk > 0 ? k : k - 1, K);
                __syncthreads();
            }
            // step bs + 2's block (past the last step: a zero-size descriptor, zeros into a slot no
            // step reads)
            dma(dk, dblk, lds + (slot == 0 ? 2 : slot - 1) * SF);
            if (++dblk == NB) {
                dblk = 0;
                ++dk;
            }
            const float* ys = lds + slot * SF;
            const int c0 = blk * CW;
            const int nk = blk + 1 == NB ? k + 1 : k, nc0 = blk + 1 == NB ? 0 : c0 + CW;   // next step
            // the PW x CT tiles of the step, each a compile-time index (static ring slots)
            auto tile = [&](auto ic) {
                constexpr int i = decltype(ic)::value;
                if constexpr (!RING) {   // four waves per SIMD: A^T / U / d0 loaded at the tile's start,
                    fetch_a(k, c0, i, r0);   // A after GEMM2 (into the A^T registers' room)
                    compute(k, c0, ys, i, r0, [] {}, [&] { fetch_m(k, c0, i, r0); });
                    return;
                }
                Ring& cur = (i & 1) ? r1 : r0;
                Ring& nxt = (i & 1) ? r0 : r1;
                constexpr bool last = i + 1 == PW * CT;
                const int tk = last ? nk : k, tc0 = last ? nc0 : c0;
                constexpr int ni = last ? 0 : i + 1;
                // (past the last step the fetch reads harmless valid memory or nothing)
                compute(k, c0, ys, i, cur, [&] { fetch_a(tk, tc0, ni, nxt); },
                        [&] { fetch_m(tk, tc0, ni, nxt); });
            };
            tile(std::integral_constant<int, 0>{});
            tile(std::integral_constant<int, 1>{});
            if constexpr (PW == 2) {
                tile(std::integral_constant<int, 2>{});
                tile(std::integral_constant<int, 3>{});
            }
            slot = slot == SLOTS - 1 ? 0 : slot + 1;
        }
    }
    status |= (bad_y0 ? 1u : 0u) | (bad_u0 ? 2u : 0u) | (bad_g ? 4u : 0u) | ((bad_y || bad_h) ? 8u : 0u);
    if (a.status != nullptr) {
        uint32_t ws = status;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) ws |= __shfl_xor(ws, o);
        if (lane == 0 && ws) atomicOr((unsigned int*)a.status, ws);
    }
}

}  // namespace stream

// The streamed single-launch form applies to m <= 64 rows per agent, P <= 16 agents, and at least
// four 32-column blocks (the ring reads Y[k - 1]'s block >= 2 steps after it was written).
// waves per workgroup: DADMM_STREAM_WAVES=16 runs one agent per wave (P <= 16, 128 VGPRs, four
// waves per SIMD) instead of the default 8 waves with two agents each
static int stream_waves(int P) {
    const char* e = getenv("DADMM_STREAM_WAVES");
    return (e != nullptr && atoi(e) == 16 && P <= 16) ? 16 : stream::NW;
}

bool stream_applies(const TiledArgs& a) {
    const int nw = stream_waves(a.P);
    return a.m_pad == 64 && a.P >= 1 && a.P <= 2 * stream::NW && a.n_pad % stream::CW == 0 &&
           a.n_pad / stream::CW >= 4 && stream::lds_bytes(nw, (a.P + nw - 1) / nw, a.P) <= 160 * 1024;
}

hipError_t launch_stream(const TiledArgs& a, hipStream_t st) {
    const int nw = stream_waves(a.P);
    const int PW = (a.P + nw - 1) / nw;
    const void* kern = nw == 16 ? (const void*)stream::stream_kernel<16, 1>
                                : (PW == 1 ? (const void*)stream::stream_kernel<8, 1> : (const void*)stream::stream_kernel<8, 2>);
    const size_t lds = stream::lds_bytes(nw, PW, a.P);
    hipError_t e = hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    const int grid = (a.B + BT - 1) / BT;
    if (a.Grec != nullptr) {   // recording (8 waves)
        const void* rk = PW == 1 ? (const void*)stream::stream_kernel<8, 1, true> : (const void*)stream::stream_kernel<8, 2, true>;
        const size_t rl = stream::lds_bytes(8, (a.P + 7) / 8, a.P);
        if ((e = hipFuncSetAttribute(rk, hipFuncAttributeMaxDynamicSharedMemorySize, (int)rl)) != hipSuccess) return e;
        if (a.P <= 8)
            hipLaunchKernelGGL((stream::stream_kernel<8, 1, true>), dim3(grid), dim3(64 * 8), rl, st, a);
        else
            hipLaunchKernelGGL((stream::stream_kernel<8, 2, true>), dim3(grid), dim3(64 * 8), rl, st, a);
        return hipGetLastError();
    }
    if (nw == 16)
        hipLaunchKernelGGL((stream::stream_kernel<16, 1>), dim3(grid), dim3(64 * 16), lds, st, a);
    else if (PW == 1)
        hipLaunchKernelGGL((stream::stream_kernel<8, 1>), dim3(grid), dim3(64 * 8), lds, st, a);
    else
        hipLaunchKernelGGL((stream::stream_kernel<8, 2>), dim3(grid), dim3(64 * 8), lds, st, a);
    return hipGetLastError();
}

}  // namespace dadmm
