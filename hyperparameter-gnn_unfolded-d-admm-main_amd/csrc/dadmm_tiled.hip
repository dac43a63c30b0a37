// dadmm_tiled.hip — one launch per iteration for the shapes the fused kernel cannot hold on chip
// (many agents / long signals, e.g. BASELINE configs[2]: P = 16, n = 512; configs[4]: P = 50,
// n = 1024): the state lives in HBM, every (16-sample tile, agent) workgroup does a whole
// iteration of its agent in one pass.
//
// Reference semantics: unfolded_DLASSO.py:53-107 / :127-140 (and the GNN variant's clamps,
// gnn_dlasso_models_progressive.py:205-232). Iteration k of workgroup (tile, p):
//   delta_k[p] = sum over p's visit list of (y_p - y_q), from y_k of the neighbours: formed for
//                every agent of a sample at once by consensus_kernel (one pass over y_k, the
//                sample's rows staged in LDS) and read here as one more stream (k = 0: d0);
//   U_k[p]     = clamp(U_{k-1}[p] + delta_k[p] eta_{k-1}, +-vclip_{k-1})   (the dual update of
//                iteration k-1, deferred to here as in the fused kernel; k = 0: U0);
//   R          = A_p y_k - b_p;  G = A_p^T R                (f32 MFMA fma chains, the fused
//                kernel's / the oracle's order);
//   y_{k+1}    = clamp(y_k - alpha clamp(G + sign(y) tau + U_k deg + delta_k rho)) -> Y[k].
// So per unit of work the HBM traffic is read y_k, U_{k-1}, b, write y_{k+1}, U_k: SURVEY.md
// §8(d)'s algorithmic 4 P (4n + m) bytes (the neighbour tiles come from L2).
//
// Guards: like the fused kernel, this path does not apply the reference's batch-global NaN/Inf
// guards; it ORs the status bits of every case where one would fire, and the caller enqueues the
// gated stepwise recomputation behind it (dadmm_forward_stepwise, DADMM_GATE_ON). On guard-free
// inputs its output is bit-identical to the stepwise path and to oracle_forward_f32.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "dadmm_internal.h"

namespace dadmm {
namespace tiled {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __amdgpu_buffer_rsrc_t rsrc_t;

__device__ __forceinline__ rsrc_t make_rsrc(const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ f32x4 bload4(rsrc_t r, uint32_t voff) {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, 0));
}

constexpr int THREADS = 256;   // 4 waves: GEMM1 = one 16-row m-block per wave
constexpr int WAVES = 4;

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float tclamp(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }
__device__ __forceinline__ bool finitef(float x) { return __builtin_isfinite(x); }

__device__ __forceinline__ void clips(int variant, int k, float& gclip, float& vclip) {
    if (variant == 0) {
        gclip = fmaxf(1.0f, 30.0f - (float)k);          // unfolded_DLASSO.py:80
        vclip = fmaxf(10.0f, 200.0f - (float)(k * 3));  // unfolded_DLASSO.py:92
    } else {
        gclip = 10.0f;                                   // gnn_dlasso_models_progressive.py:212
        vclip = 100.0f;                                  // :224, :232
    }
}

constexpr int HALVES = 2;            // 16-sample MFMA column blocks per workgroup (32 samples):
                                     // every A / A^T operand load feeds two fma chains
constexpr int ST = HALVES * BT;      // samples per workgroup
// MB = m-groups of 64 rows per agent (m_pad = 64 MB; MB in {1, 2}). The update phase works in
// chunks of CH = 2 / MB n-tiles, so that a chunk's A^T rows (CH x 4 MB vectors) take the same
// registers for both; with MB = 2 the GEMM2 B operand (R) is read from LDS, not held.
// MB = 1: chunks of one n-tile, double-buffered (chunk c + 1's loads in flight
// under chunk c's update) in the registers one 2-tile chunk took (160 VGPRs instead of 192)
template <int MB>
struct Chunk {                       // one chunk's operands
    static constexpr bool DB = MB == 1;
    static constexpr int CH = DB ? 1 : 2 / MB;   // n-tiles per chunk of the update phase
    static constexpr int RG = CH * HALVES;       // row groups per chunk
    f32x4 yp[RG], up[RG], dv[RG];
    f32x4 atv[CH][4 * MB];
};

// blockIdx -> (tile, agent) so that the P workgroups of one sample tile run on the same XCD
// (dispatch is round-robin over the 8 XCDs, each with its own L2): the neighbour tiles a
// workgroup reads for delta are its siblings' own tiles, hot in that L2.
__device__ __forceinline__ int xcd_swizzle(int bid, int G) {
    constexpr int NX = 8;
    const int xcd = bid % NX, i = bid / NX, q = G / NX, r = G % NX;
    return xcd < r ? xcd * (q + 1) + i : r * (q + 1) + (xcd - r) * q + i;
}

typedef __attribute__((address_space(3))) void lds_void;

// STAGE (n_pad <= STAGE_NP_MAX): the workgroup's y_k tile [ST][n_pad] is copied HBM -> LDS by
// buffer_load ... lds (no VGPRs, the whole 64 KB in flight at once) at the start of the
// iteration; GEMM1's B operand and the update phase's own rows are then read from LDS. The
// image is lane-linear (the DMA's constraint), so the bank swizzle is applied on the source:
// 16-byte chunk c of row sl is stored at chunk c ^ (sl & 15) of that row, and the 16 lanes of an
// MFMA column block (16 samples, one chunk each) hit 16 distinct chunks of an aligned 256 B run.
constexpr int STAGE_NP_MAX = 512;

// k >= 0: one iteration (see header). k == K: the final dual update only (U_K into U_out).
// Workgroup = (32-sample tile, agent p).
// amdgpu_waves_per_eu(2): keeps VGPRs + AGPRs <= 256 (two workgroups per CU); without it the
// allocator lands at 249 + 8 and the kernel runs at one wave per SIMD (0.40 -> 0.53 ms/iteration)
// RONLY (the column-split path): GEMM1 only, R_k -> a.R [B][P][m_pad]; the update runs in
// colupdate_kernel
template <bool STAGE, int MB, bool RONLY = false>
__global__ __launch_bounds__(THREADS) __attribute__((amdgpu_waves_per_eu(2))) void iter_kernel(TiledArgs a, int k) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    constexpr int MP = 64 * MB;                      // padded rows per agent (a.m_pad)
    constexpr int CH = Chunk<MB>::CH, RG = Chunk<MB>::RG;
    const int P = a.P, n = a.n, m = a.m, B = a.B, NP = a.n_pad;
    const int wg = xcd_swizzle(blockIdx.x, gridDim.x);
    const int tile = wg / P, p = wg % P;
    const int RS = MP + 4;
    float* Ylds = lds;                               // [ST][NP] swizzled y_k tile (STAGE)
    float* Rlds = lds + (STAGE ? ST * NP : 0);       // [ST][RS]
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int j = lane & 15, h = lane >> 4;
    const size_t S = (size_t)B * P * n;
    const float* yk = k == 0 ? a.y0 : a.Y + (size_t)(k - 1) * S;   // y_k of every agent
    const bool final_only = k == a.K;
    const int H = a.hyp_rows;
    const int hp = H == 1 ? 0 : p;
    uint32_t status = 0;

    // update-phase operands; chunk 0 is issued now, so that it lands with the y tile
    const float* Uprev = a.Ubuf[(k + 1) & 1];     // U_{k-1}   (k = 0: unused)
    const float* usrc = k == 0 ? a.U0 : Uprev;
    const float* dsrc = k == 0 ? a.d0 : a.delta;  // delta_k
    const int ntw = (NP / 16 - w + WAVES - 1) / WAVES;   // n-tiles of this wave: w, w + 4, ...
    const float* atbase = a.At + ((size_t)p * NP + j) * MP + 4 * h;
    const bool ylds = STAGE && !final_only;       // own rows from the staged tile
    size_t srow[HALVES];
#pragma unroll
    for (int hh = 0; hh < HALVES; ++hh) {
        const int s = tile * ST + hh * BT + j;
        srow[hh] = (size_t)(s < B ? s : 0) * P;
    }
    auto load_chunk = [&](int c0, Chunk<MB>& c) {
#pragma unroll
        for (int i = 0; i < CH; ++i) {
            const int nb = w + WAVES * (c0 + i);
            const int n0 = 16 * nb + 4 * h;
            const bool tile_ok = c0 + i < ntw;
            if (!final_only && tile_ok) {
#pragma unroll
                for (int t = 0; t < MP / 16; ++t)
                    c.atv[i][t] = *(const f32x4*)(atbase + (size_t)16 * nb * MP + 16 * t);
            }
#pragma unroll
            for (int hh = 0; hh < HALVES; ++hh) {
                const int g = i * HALVES + hh;
                const int s = tile * ST + hh * BT + j;
                const size_t off = (srow[hh] + p) * n + n0;
                c.yp[g] = c.up[g] = c.dv[g] = (f32x4){0, 0, 0, 0};
                if (tile_ok && s < B && n0 < n) {
                    if (!ylds) c.yp[g] = *(const f32x4*)(yk + off);
                    c.up[g] = *(const f32x4*)(usrc + off);
                    c.dv[g] = *(const f32x4*)(dsrc + off);
                }
            }
        }
    };
    Chunk<MB> cA;
    if (!RONLY && ntw > 0) load_chunk(0, cA);

    if constexpr (STAGE) {
        if (!final_only) {
            const rsrc_t ry = make_rsrc(yk, (uint32_t)(S * 4));
            const int CPR = NP / 4;                   // 16-byte chunks per row (a multiple of 16)
            for (int base = w * 64; base < ST * CPR; base += WAVES * 64) {
                const int lc = base + lane;
                const int sl = lc / CPR, c = (lc % CPR) ^ (sl & 15);
                const int s = tile * ST + sl;
                const uint32_t off = (s < B && 4 * c < n)
                                         ? (uint32_t)((((size_t)s * P + p) * n + 4 * c) * 4)
                                         : 0x80000000u;   // past the range: the DMA writes zeros
                __builtin_amdgcn_raw_ptr_buffer_load_lds(ry, (lds_void*)(Ylds + 4 * base), 16, off,
                                                         0, 0, 0);
            }
        }
    }

    if (!final_only) {
        if (k == 0) {   // :55 guard on y0 (the only iteration where it can fire)
            const int nc4 = n / 4;
            bool bad = false;
            for (int idx = threadIdx.x; idx < ST * nc4; idx += THREADS) {
                const int s2 = tile * ST + idx / nc4, c = 4 * (idx % nc4);
                if (s2 < B) {
                    const f32x4 v = *(const f32x4*)(yk + ((size_t)s2 * P + p) * n + c);
                    bad |= !(finitef(v[0]) && finitef(v[1]) && finitef(v[2]) && finitef(v[3]));
                }
            }
            status |= bad ? 1u : 0u;
        }
        // GEMM1: R = A_p y - b_p, one fma chain per row from -b (wave w = m-blocks w, w + 4, ...
        // of the MB m-groups), one chain per 16-sample half sharing every A load
        if constexpr (STAGE) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's DMA has landed
            __syncthreads();                                     // ... and every other wave's
        }
#pragma unroll
        for (int mg = 0; mg < MB; ++mg) {
            const int mq = w + WAVES * mg;                   // this pass's m-block
            f32x4 acc[HALVES];
#pragma unroll
            for (int hh = 0; hh < HALVES; ++hh) {
                const int s = tile * ST + hh * BT + j;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int mi = 16 * mq + 4 * h + r;
                    acc[hh][r] = (s < B && mi < m) ? -a.b[((size_t)s * P + p) * m + mi] : 0.0f;
                }
            }
            if (16 * mq < m) {
                // the B operand (y_k, 16 columns per half) from the staged LDS tile (STAGE), else
                // straight from L2/HBM through a buffer
                // descriptor: columns past n and samples past B get an offset past the range, which
                // the hardware returns as 0 (the padded operator columns are 0 too) - no branches
                const float* arow = a.A + ((size_t)p * MP + 16 * mq + j) * NP + 4 * h;
                const rsrc_t ry = make_rsrc(yk, (uint32_t)(S * 4));
                uint32_t yoff[HALVES];
#pragma unroll
                for (int hh = 0; hh < HALVES; ++hh) {
                    const int s = tile * ST + hh * BT + j;
                    yoff[hh] = s < B ? (uint32_t)((((size_t)s * P + p) * n + 4 * h) * 4) : 0x80000000u;
                }
                auto ldb = [&](int hh, int t) -> f32x4 {
                    if constexpr (STAGE)
                        return *(const f32x4*)(Ylds + (hh * BT + j) * NP + 4 * ((4 * t + h) ^ j));
                    else
                        return bload4(ry, 16 * t + 4 * h < n ? yoff[hh] + 64u * t : 0x80000000u);
                };
                // operand ring of depth D: the loads of step t + D are issued right after step t's
                // MFMAs (pinned there by a scheduling barrier); T = NP / 16 is a multiple of D. The
                // steady loop is straight-line, two groups per trip (the compiler's waits at a loop
                // head drain the queue), so the waits count the D - 1 younger steps in flight.
                constexpr int D = 4;
                const int T = NP / 16;
                f32x4 ar[D], br[D][HALVES];
                auto load = [&](int u, int t) {
                    ar[u] = *(const f32x4*)(arow + 16 * t);
#pragma unroll
                    for (int hh = 0; hh < HALVES; ++hh) br[u][hh] = ldb(hh, t);
                };
                auto step = [&](int u) {
#pragma unroll
                    for (int hh = 0; hh < HALVES; ++hh)
#pragma unroll
                        for (int r = 0; r < 4; ++r) acc[hh] = mfma4(ar[u][r], br[u][hh][r], acc[hh]);
                };
#pragma unroll
                for (int u = 0; u < D; ++u) load(u, u);
                int t0 = 0;
                for (; t0 + 3 * D <= T; t0 += 2 * D) {
#pragma unroll
                    for (int u = 0; u < 2 * D; ++u) {
                        step(u % D);
                        load(u % D, t0 + u + D);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                }
                if (t0 + 2 * D <= T) {
#pragma unroll
                    for (int u = 0; u < D; ++u) {
                        step(u);
                        load(u, t0 + u + D);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                    t0 += D;
                }
#pragma unroll
                for (int u = 0; u < D; ++u) step(u);   // the last D steps (T % D == 0)
            }
#pragma unroll
            for (int hh = 0; hh < HALVES; ++hh) {
                if constexpr (RONLY) {
                    const int s = tile * ST + hh * BT + j;
                    if (s < B) *(f32x4*)(a.R + ((size_t)s * P + p) * MP + 16 * mq + 4 * h) = acc[hh];
                } else {
                    *(f32x4*)(Rlds + (hh * BT + j) * RS + 16 * mq + 4 * h) = acc[hh];
                }
            }
        }
    }
    if constexpr (RONLY) {
        if (a.status != nullptr) {
            uint32_t ws = status;
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) ws |= __shfl_xor(ws, o);
            if (lane == 0 && ws) atomicOr((unsigned int*)a.status, ws);
        }
        return;
    }
    __syncthreads();

    float al = 0, ta = 0, rh = 0, et = 0, et_prev = 0, gclip = 0, vclip = 0, vclip_prev = 0;
    if (!final_only) {
        const float* hk = a.hyp + ((size_t)k * H + hp) * 4;
        al = hk[0]; ta = hk[1]; rh = hk[2]; et = hk[3];
        status |= (finitef(al) && finitef(ta) && finitef(rh) && finitef(et)) ? 0u : 8u;
        clips(a.variant, k, gclip, vclip);
    }
    if (k > 0) {
        et_prev = a.hyp[((size_t)(k - 1) * H + hp) * 4 + 3];
        float gtmp;
        clips(a.variant, k - 1, gtmp, vclip_prev);
    }
    float* Ucur = final_only ? a.U_out : a.Ubuf[k & 1];   // U_k

    // per-lane data of the two samples this lane serves
    float dg[HALVES];
    f32x4 rv[HALVES][MB == 1 ? 4 : 1];   // MB = 1: GEMM2's B operand held; MB = 2: read from LDS
#pragma unroll
    for (int hh = 0; hh < HALVES; ++hh) {
        const int s = tile * ST + hh * BT + j;
        const int g0 = a.graph_shared ? 0 : s * P;
        dg[hh] = s < B ? a.deg[g0 + p] : 0.0f;
        if (MB == 1 && !final_only) {
#pragma unroll
            for (int t = 0; t < 4; ++t)
                rv[hh][t] = *(const f32x4*)(Rlds + (hh * BT + j) * RS + 16 * t + 4 * h);
        }
    }
    bool bad_u0 = false, bad_g = false, bad_y = false;
    auto compute_chunk = [&](int c0, Chunk<MB>& c) {
        int n0[CH];
        bool okr[RG];
        size_t off[RG];
        f32x4 uv[RG];
#pragma unroll
        for (int i = 0; i < CH; ++i) {
            n0[i] = 16 * (w + WAVES * (c0 + i)) + 4 * h;
#pragma unroll
            for (int hh = 0; hh < HALVES; ++hh) {
                const int g = i * HALVES + hh;
                const int s = tile * ST + hh * BT + j;
                okr[g] = c0 + i < ntw && s < B && n0[i] < n;
                off[g] = (srow[hh] + p) * n + n0[i];
                if (ylds && okr[g])
                    c.yp[g] = *(const f32x4*)(Ylds + (hh * BT + j) * NP + 4 * ((n0[i] >> 2) ^ j));
            }
        }
#pragma unroll
        for (int g = 0; g < RG; ++g) {
            if (!okr[g]) continue;
            if (k == 0) {
                uv[g] = c.up[g];
#pragma unroll
                for (int r = 0; r < 4; ++r) bad_u0 |= !finitef(uv[g][r]);
            } else {
                if (a.variant != 0) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) c.dv[g][r] = tclamp(c.dv[g][r], -20.0f, 20.0f);   // :229
                }
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    uv[g][r] = tclamp(c.up[g][r] + c.dv[g][r] * et_prev, -vclip_prev, vclip_prev);
            }
            *(f32x4*)(Ucur + off[g]) = uv[g];          // U_k (the ping-pong buffer / U_out)
        }
        if (final_only) return;
        // GEMM2 rows of these tiles + gradient assembly + primal update (:69-93)
#pragma unroll
        for (int g = 0; g < RG; ++g) {
            const int hh = g % HALVES, i = g / HALVES;
            if (c0 + i >= ntw) continue;
            f32x4 gc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
            for (int t = 0; t < MP / 16; ++t) {
                const f32x4 rt = MB == 1 ? rv[hh][t & 3]
                                         : *(const f32x4*)(Rlds + (hh * BT + j) * RS + 16 * t + 4 * h);
#pragma unroll
                for (int r = 0; r < 4; ++r) gc = mfma4(c.atv[i][t][r], rt[r], gc);
            }
            if (okr[g]) {
                f32x4 yn;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float y = c.yp[g][r];
                    const float st = sign_times(y, ta);   // sign(y) * tau
                    float gr = gc[r] + st;
                    gr = gr + uv[g][r] * dg[hh];
                    gr = gr + c.dv[g][r] * rh;
                    bad_g |= gr != gr;
                    gr = tclamp(gr, -gclip, gclip);
                    const float v = tclamp(y - al * gr, -vclip, vclip);
                    bad_y |= !finitef(v);
                    yn[r] = v;
                }
                *(f32x4*)(a.Y + (size_t)k * S + off[g]) = yn;
            }
        }
    };
    if constexpr (Chunk<MB>::DB) {
        Chunk<MB> cB;
        for (int c0 = 0; c0 < ntw; c0 += 2 * CH) {
            if (c0 + CH < ntw) load_chunk(c0 + CH, cB);
            compute_chunk(c0, cA);
            if (c0 + CH < ntw) {
                if (c0 + 2 * CH < ntw) load_chunk(c0 + 2 * CH, cA);
                compute_chunk(c0 + CH, cB);
            }
        }
    } else {
        for (int c0 = 0; c0 < ntw; c0 += CH) {
            if (c0 > 0) load_chunk(c0, cA);
            compute_chunk(c0, cA);
        }
    }
    status |= (bad_u0 ? 2u : 0u) | (bad_g ? 4u : 0u) | (bad_y ? 8u : 0u);
    if (a.status != nullptr) {
        uint32_t ws = status;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) ws |= __shfl_xor(ws, o);
        if (lane == 0 && ws) atomicOr((unsigned int*)a.status, ws);
    }
}

// delta_k = compute_delta(y_k) (unfolded_DLASSO.py:127-140) for every agent of one sample over a
// block of CB columns: the sample's P rows and its visit lists are staged in LDS (one coalesced
// pass over y_k), then wave w forms agent p = w, w + 4, ... by its visit list in the reference's
// order, one fp32 add chain per column from 0 (bit-identical to the fused / stepwise consensus).
constexpr int CB = 256;
// visit entries per sample: every node lists each neighbour twice (both ends of an edge), <= 2 P^2
size_t consensus_lds_bytes(int P) { return 4 * (size_t)P * CB + 4 * (size_t)(P + 1) + 2 * (size_t)P * P; }
__global__ __launch_bounds__(THREADS) void consensus_kernel(TiledArgs a, const float* __restrict__ y) {
    extern __shared__ __attribute__((aligned(16))) float ys[];   // [P][CB]
    const int P = a.P, n = a.n;
    int32_t* vp = (int32_t*)(ys + P * CB);                       // [P + 1] list starts (local)
    uint8_t* vq = (uint8_t*)(vp + P + 1);                        // <= 2 P^2 entries
    const int ncb = (n + CB - 1) / CB;
    const int s = blockIdx.x / ncb, c0 = (blockIdx.x % ncb) * CB;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const float* ys_g = y + (size_t)s * P * n;
    // the sample's rows: up to 4 chunks per thread loaded before any is stored (one round trip
    // for P <= 16), then the rest if P is larger
    constexpr int CPT = 4;
    {
        f32x4 v[CPT];
#pragma unroll
        for (int u = 0; u < CPT; ++u) {
            const int idx = threadIdx.x + u * THREADS;
            const int p = idx / (CB / 4), c = c0 + 4 * (idx % (CB / 4));
            v[u] = (p < P && c < n) ? *(const f32x4*)(ys_g + (size_t)p * n + c)
                                    : (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
        }
#pragma unroll
        for (int u = 0; u < CPT; ++u) {
            const int idx = threadIdx.x + u * THREADS;
            const int p = idx / (CB / 4), c = c0 + 4 * (idx % (CB / 4));
            if (p < P && c < n) *(f32x4*)(ys + p * CB + (c - c0)) = v[u];
        }
    }
    for (int idx = threadIdx.x + CPT * THREADS; idx < P * (CB / 4); idx += THREADS) {
        const int p = idx / (CB / 4), c = c0 + 4 * (idx % (CB / 4));
        if (c < n) *(f32x4*)(ys + p * CB + (c - c0)) = *(const f32x4*)(ys_g + (size_t)p * n + c);
    }
    const int g0 = a.graph_shared ? 0 : s * P;
    const int vbase = a.vptr[g0], vend = a.vptr[g0 + P];
    for (int i = threadIdx.x; i <= P; i += THREADS) vp[i] = a.vptr[g0 + i] - vbase;
    for (int i = threadIdx.x; i < vend - vbase; i += THREADS) vq[i] = a.vq[vbase + i];
    __syncthreads();
    const int c = c0 + 4 * lane;
    if (c >= n) return;
    for (int p = w; p < P; p += WAVES) {
        const int v0 = vp[p], v1 = vp[p + 1];
        const f32x4 yp = *(const f32x4*)(ys + p * CB + 4 * lane);
        f32x4 dv = {0.0f, 0.0f, 0.0f, 0.0f};
        for (int t = v0; t < v1; ++t) {
            const f32x4 yq = *(const f32x4*)(ys + (int)vq[t] * CB + 4 * lane);
#pragma unroll
            for (int r = 0; r < 4; ++r) dv[r] = dv[r] + (yp[r] - yq[r]);
        }
        *(f32x4*)(a.delta + ((size_t)s * P + p) * n + c) = dv;
    }
}


// ---- column-split path: GEMM1 per (tile, agent), then one update kernel per (tile, column block)
// that holds every agent of its samples, so the consensus is formed in LDS and neither delta_k
// nor a second copy of y_k goes through HBM. Per iteration: iter_kernel<., ., RONLY> reads y_k and
// b and writes R_k (m_pad floats per sample-agent), colupdate_kernel reads y_k, U_{k-1} and R_k
// and writes y_{k+1} and U_k: the algorithmic streams plus R.
//
// Workgroup = (ST2 = 32 samples, CW columns) x all P agents. y_k[s][*][c0, c0 + CW) is copied
// HBM -> LDS by LDS-DMA (row sl = one sample, P CW floats, 16-byte chunk c stored at chunk
// c ^ (sl & 15) of its row: the 16 lanes of an MFMA column block read 16 distinct chunks of an
// aligned 256 B run). Wave w takes agents w, w + 4, ...; per agent it holds R_p of both 16-sample
// halves (GEMM2's B operand) and per 16-column n-tile A_p^T's rows (its A operand). A lane
// (j, h) owns columns c0 + 16 nt + 4h .. + 3 of sample j of each half: delta_k by the sample's
// visit list over the LDS rows (the consensus kernel's order), the deferred dual update, the
// GEMM2 chain and the primal update, exactly as iter_kernel.
constexpr int ST2 = 2 * BT;
size_t colsplit_lds_bytes(int P, int CW, int vcap) {
    return 4 * (size_t)ST2 * P * CW + 4 * (size_t)(ST2 * P + 1) + (size_t)vcap + 4;
}
constexpr int AMAX = 4;     // agents per wave of the column-split path (P <= 16)
template <int MB, int NT>   // NT = CW / 16 n-tiles per column block
__global__ __launch_bounds__(THREADS) void colupdate_kernel(TiledArgs a, int k, int vcap) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    constexpr int MP = 64 * MB, TM = MP / 16;
    constexpr int CW = 16 * NT;
    const int P = a.P, n = a.n, B = a.B, NP = a.n_pad, H = a.hyp_rows;
    const int ncb = (n + CW - 1) / CW;
    const int wg = xcd_swizzle(blockIdx.x, gridDim.x);   // a tile's column blocks on one XCD
    const int tile = wg / ncb, c0 = (wg % ncb) * CW;
    const int s0 = tile * ST2, ns = min(ST2, B - s0);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int j = lane & 15, h = lane >> 4;
    const int CQ = CW / 4, RC = P * CQ;                  // 16-byte chunks per agent / per LDS row
    float* ys = lds;                                     // [ST2][RC] chunks, swizzled
    int32_t* vp = (int32_t*)(ys + (size_t)ST2 * RC * 4); // visit-list starts, local
    uint8_t* vql = (uint8_t*)(vp + ST2 * P + 1);
    const size_t S = (size_t)B * P * n;
    const float* yk = k == 0 ? a.y0 : a.Y + (size_t)(k - 1) * S;
    const bool final_only = k == a.K;

    {   // y_k block -> LDS (no VGPRs held; past-the-range offsets return zeros)
        const rsrc_t ry = make_rsrc(yk, (uint32_t)(S * 4));
        for (int base = w * 64; base < ST2 * RC; base += WAVES * 64) {
            const int lc = base + lane;
            const int sl = lc / RC, cs = (lc % RC) ^ (sl & 15);
            const int p = cs / CQ, c = c0 + 4 * (cs % CQ);
            const uint32_t off = (sl < ns && c < n)
                                     ? (uint32_t)((((size_t)(s0 + sl) * P + p) * n + c) * 4)
                                     : 0x80000000u;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(ry, (lds_void*)(ys + 4 * base), 16, off, 0, 0, 0);
        }
    }
    // visit lists of the tile's samples (one list for a shared graph)
    const int nl = a.graph_shared ? P : ns * P;
    const int g0 = a.graph_shared ? 0 : s0 * P;
    const int vbase = a.vptr[g0];
    const int nent = a.vptr[g0 + nl] - vbase;
    // (vcap + 4 <= 8 KB: every thread's loads are issued before its LDS stores, one round trip)
    const int vsh = vbase & 3;                           // lists copied as aligned 32-bit words
    const bool vin = nent + vsh <= vcap;
    {
        constexpr int VPW = (ST2 * 16 + 1 + THREADS - 1) / THREADS;   // list starts per thread
        constexpr int VQW = 8192 / 4 / THREADS;                       // list words per thread
        int pv[VPW];
        uint32_t qv[VQW];
        const uint32_t* vq32 = (const uint32_t*)(a.vq + (vbase - vsh));
        const int nw = vin ? (nent + vsh + 3) / 4 : 0;
#pragma unroll
        for (int u = 0; u < VPW; ++u) {
            const int i = threadIdx.x + u * THREADS;
            pv[u] = i <= nl ? a.vptr[g0 + i] : 0;
        }
#pragma unroll
        for (int u = 0; u < VQW; ++u) {
            const int i = threadIdx.x + u * THREADS;
            qv[u] = i < nw ? vq32[i] : 0u;
        }
#pragma unroll
        for (int u = 0; u < VPW; ++u) {
            const int i = threadIdx.x + u * THREADS;
            if (i <= nl) vp[i] = pv[u] - vbase;
        }
#pragma unroll
        for (int u = 0; u < VQW; ++u) {
            const int i = threadIdx.x + u * THREADS;
            if (i < nw) ((uint32_t*)vql)[i] = qv[u];
        }
    }
    const uint8_t* vq = vin ? (const uint8_t*)vql + vsh : a.vq + vbase;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    auto yl = [&](int sl, int p, int g) -> f32x4 {   // columns c0 + 4g .. of agent p, sample row sl
        return *(const f32x4*)(ys + 4 * ((size_t)sl * RC + ((p * CQ + g) ^ (sl & 15))));
    };
    float vclip_prev = 0.0f, gtmp;
    if (k > 0) clips(a.variant, k - 1, gtmp, vclip_prev);
    float gclip = 0.0f, vclip = 0.0f;
    if (!final_only) clips(a.variant, k, gclip, vclip);
    const float* usrc = k == 0 ? a.U0 : a.Ubuf[0];
    float* Ucur = final_only ? a.U_out : a.Ubuf[0];       // in place: U_{k-1} -> U_k
    float* Yk = a.Y + (size_t)k * S;
    uint32_t status = 0;
    bool bad_u0 = false, bad_g = false, bad_y = false;

#pragma unroll
    for (int ai = 0; ai < AMAX; ++ai) {
        const int p = w + WAVES * ai;
        if (p >= P) break;
        const int hp = H == 1 ? 0 : p;
        float al = 0, ta = 0, rh = 0, et_prev = 0;
        if (!final_only) {
            const float* hk = a.hyp + ((size_t)k * H + hp) * 4;
            al = hk[0]; ta = hk[1]; rh = hk[2];
            const float et = hk[3];
            status |= (finitef(al) && finitef(ta) && finitef(rh) && finitef(et)) ? 0u : 8u;
        }
        if (k > 0) et_prev = a.hyp[((size_t)(k - 1) * H + hp) * 4 + 3];
        // every global operand of this agent is issued first (R_p, A_p^T rows, U_{k-1}, d0); the
        // consensus over the LDS block runs under their latency
        f32x4 rv[HALVES][TM], at[NT][TM], up[NT][HALVES], dv[NT][HALVES], yv[NT][HALVES];
        float dg[HALVES];
        bool okr[NT][HALVES];
        size_t off[NT][HALVES];
#pragma unroll
        for (int hh = 0; hh < HALVES; ++hh) {
            const int s = s0 + hh * BT + j;
            dg[hh] = s < B ? a.deg[(a.graph_shared ? 0 : s * P) + p] : 0.0f;
#pragma unroll
            for (int t = 0; t < TM; ++t)
                rv[hh][t] = (!final_only && s < B)
                                ? *(const f32x4*)(a.R + ((size_t)s * P + p) * MP + 16 * t + 4 * h)
                                : (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
        }
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
            const int col = c0 + 16 * nt + 4 * h;
            if (!final_only) {
                const float* atp = a.At + ((size_t)p * NP + c0 + 16 * nt + j) * MP + 4 * h;
#pragma unroll
                for (int t = 0; t < TM; ++t) at[nt][t] = *(const f32x4*)(atp + 16 * t);
            }
#pragma unroll
            for (int hh = 0; hh < HALVES; ++hh) {
                const int sl = hh * BT + j, s = s0 + sl;
                okr[nt][hh] = s < B && col < n;
                off[nt][hh] = ((size_t)(okr[nt][hh] ? s : 0) * P + p) * n + (okr[nt][hh] ? col : 0);
                up[nt][hh] = dv[nt][hh] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
                if (okr[nt][hh]) {
                    up[nt][hh] = *(const f32x4*)(usrc + off[nt][hh]);
                    if (k == 0) dv[nt][hh] = *(const f32x4*)(a.d0 + off[nt][hh]);
                }
                yv[nt][hh] = yl(sl, p, 4 * nt + h);
            }
        }
        if (k > 0) {   // delta_k = compute_delta(y_k) (unfolded_DLASSO.py:127-140), both halves'
                       // lists walked together, each element's chain in its list's order
            int v0[HALVES], len[HALVES], lmax = 0;
#pragma unroll
            for (int hh = 0; hh < HALVES; ++hh) {
                const int sl = hh * BT + j;
                const int li = a.graph_shared ? p : sl * P + p;
                v0[hh] = vp[li];
                len[hh] = s0 + sl < B ? vp[li + 1] - v0[hh] : 0;
                lmax = max(lmax, len[hh]);
            }
            for (int t = 0; t < lmax; ++t) {
#pragma unroll
                for (int hh = 0; hh < HALVES; ++hh) {
                    if (t < len[hh]) {
                        const int q = (int)vq[v0[hh] + t];
#pragma unroll
                        for (int nt = 0; nt < NT; ++nt) {
                            const f32x4 yq = yl(hh * BT + j, q, 4 * nt + h);
#pragma unroll
                            for (int r = 0; r < 4; ++r)
                                dv[nt][hh][r] = dv[nt][hh][r] + (yv[nt][hh][r] - yq[r]);
                        }
                    }
                }
            }
            if (a.variant != 0) {
#pragma unroll
                for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                    for (int hh = 0; hh < HALVES; ++hh)
#pragma unroll
                        for (int r = 0; r < 4; ++r)
                            dv[nt][hh][r] = tclamp(dv[nt][hh][r], -20.0f, 20.0f);   // :229
            }
        }
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
#pragma unroll
            for (int hh = 0; hh < HALVES; ++hh) {
                const bool ok = okr[nt][hh];
                f32x4 uv;
                if (k == 0) {
                    uv = up[nt][hh];
#pragma unroll
                    for (int r = 0; r < 4; ++r) bad_u0 |= ok && !finitef(uv[r]);
                } else {
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        uv[r] = tclamp(up[nt][hh][r] + dv[nt][hh][r] * et_prev, -vclip_prev, vclip_prev);
                }
                if (ok) *(f32x4*)(Ucur + off[nt][hh]) = uv;           // U_k
                if (final_only) continue;
                f32x4 gc = {0.0f, 0.0f, 0.0f, 0.0f};                  // GEMM2 rows of this n-tile
#pragma unroll
                for (int t = 0; t < TM; ++t)
#pragma unroll
                    for (int r = 0; r < 4; ++r) gc = mfma4(at[nt][t][r], rv[hh][t][r], gc);
                if (ok) {
                    f32x4 yn;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float y = yv[nt][hh][r];
                        const float st = sign_times(y, ta);
                        float gr = gc[r] + st;
                        gr = gr + uv[r] * dg[hh];
                        gr = gr + dv[nt][hh][r] * rh;
                        bad_g |= gr != gr;
                        gr = tclamp(gr, -gclip, gclip);
                        const float v = tclamp(y - al * gr, -vclip, vclip);
                        bad_y |= !finitef(v);
                        yn[r] = v;
                    }
                    *(f32x4*)(Yk + off[nt][hh]) = yn;
                }
            }
        }
    }
    status |= (bad_u0 ? 2u : 0u) | (bad_g ? 4u : 0u) | (bad_y ? 8u : 0u);
    if (a.status != nullptr) {
        uint32_t ws = status;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) ws |= __shfl_xor(ws, o);
        if (lane == 0 && ws) atomicOr((unsigned int*)a.status, ws);
    }
}

}  // namespace tiled

size_t tiled_lds_bytes(int n_pad, int m_pad) {
    const size_t stage = n_pad <= tiled::STAGE_NP_MAX ? 4 * (size_t)tiled::ST * n_pad : 0;
    return stage + 4 * (size_t)(tiled::ST * (m_pad + 4));
}

// DADMM_TILED_SPLIT=1 in the environment selects the column-split form (iter_kernel<., ., RONLY> +
// colupdate_kernel) instead of the two-launch (consensus + iteration kernel) form. Bit-identical;
// measured slower at configs[2] (7.4 vs 6.9 ms per forward), so off by default.
// the column block of the split path: the widest of 64 / 32 / 16 columns whose LDS (y block of
// 32 samples x P agents + visit lists) keeps two workgroups per CU, else the narrowest that fits
// one; 0 = the split path does not apply. The swizzle needs P CW / 4 to be a multiple of 16.
static int colsplit_width(int P, int vcap) {
    int best = 0;
    for (int cw : {64, 32, 16}) {
        if ((P * cw / 4) % 16 != 0) continue;
        const size_t l = tiled::colsplit_lds_bytes(P, cw, vcap);
        if (l <= 80 * 1024) return cw;
        if (l <= 160 * 1024) best = cw;
    }
    return best;
}

static hipError_t launch_colsplit(const TiledArgs& a, int CW, int vcap, hipStream_t stream) {
    const size_t lds = tiled_lds_bytes(a.n_pad, a.m_pad);
    const bool stage = a.n_pad <= tiled::STAGE_NP_MAX;
    auto gk = a.m_pad == 64 ? (stage ? tiled::iter_kernel<true, 1, true> : tiled::iter_kernel<false, 1, true>)
                            : (stage ? tiled::iter_kernel<true, 2, true> : tiled::iter_kernel<false, 2, true>);
    decltype(&tiled::colupdate_kernel<1, 1>) uk;
    if (a.m_pad == 64)
        uk = CW == 64 ? tiled::colupdate_kernel<1, 4> : CW == 32 ? tiled::colupdate_kernel<1, 2> : tiled::colupdate_kernel<1, 1>;
    else
        uk = CW == 64 ? tiled::colupdate_kernel<2, 4> : CW == 32 ? tiled::colupdate_kernel<2, 2> : tiled::colupdate_kernel<2, 1>;
    const size_t ulds = tiled::colsplit_lds_bytes(a.P, CW, vcap);
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute((const void*)gk, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    if (ulds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute((const void*)uk, hipFuncAttributeMaxDynamicSharedMemorySize, (int)ulds);
        if (e != hipSuccess) return e;
    }
    const int gitems = ((a.B + tiled::ST - 1) / tiled::ST) * a.P;
    const int uitems = ((a.B + tiled::ST2 - 1) / tiled::ST2) * ((a.n + CW - 1) / CW);
    for (int k = 0; k <= a.K; ++k) {
        if (k == a.K && a.U_out == nullptr) break;   // k == K: the final dual update (U_out)
        if (k < a.K)
            hipLaunchKernelGGL(gk, dim3(gitems), dim3(tiled::THREADS), lds, stream, a, k);
        hipLaunchKernelGGL(uk, dim3(uitems), dim3(tiled::THREADS), ulds, stream, a, k, vcap);
    }
    return hipGetLastError();
}

hipError_t launch_tiled(const TiledArgs& a, hipStream_t stream) {
    // the single-launch streamed form (dadmm_stream.hip) wherever it applies; DADMM_TILED_STREAM=0
    // selects the per-iteration launches below (A/B timing, tests of both forms)
    const char* senv = getenv("DADMM_TILED_STREAM");
    if ((senv == nullptr || atoi(senv) != 0) && stream_applies(a)) return launch_stream(a, stream);
    const size_t lds = tiled_lds_bytes(a.n_pad, a.m_pad);
    const char* env = getenv("DADMM_TILED_SPLIT");
    const bool split = env != nullptr && atoi(env) != 0;
    // the column-split update reads the visit lists as 32-bit words: a word-aligned base only
    // (a sharded view gb.vq[base:] may start anywhere; it takes the two-launch form)
    const bool vq_words = ((uintptr_t)a.vq & 3u) == 0;
    if (split && vq_words && a.R != nullptr && a.n_pad % 64 == 0 && (a.m_pad == 64 || a.m_pad == 128) &&
        lds <= 160 * 1024) {
        const int vcap = 8192;
        const int CW = a.P <= tiled::AMAX * tiled::WAVES ? colsplit_width(a.P, vcap) : 0;
        if (CW > 0) return launch_colsplit(a, CW, vcap, stream);
    }
    if (lds > 160 * 1024) return hipErrorInvalidConfiguration;
    if (a.n_pad % 64 != 0) return hipErrorInvalidValue;   // the swizzle and GEMM ring assume it
    if (a.m_pad != 64 && a.m_pad != 128) return hipErrorInvalidValue;   // MB in {1, 2}
    const bool stage = a.n_pad <= tiled::STAGE_NP_MAX;
    auto kern = a.m_pad == 64 ? (stage ? tiled::iter_kernel<true, 1> : tiled::iter_kernel<false, 1>)
                              : (stage ? tiled::iter_kernel<true, 2> : tiled::iter_kernel<false, 2>);
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute((const void*)kern,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    const int items = ((a.B + tiled::ST - 1) / tiled::ST) * a.P;
    const size_t S = (size_t)a.B * a.P * a.n;
    const int citems = a.B * ((a.n + tiled::CB - 1) / tiled::CB);
    const size_t clds = tiled::consensus_lds_bytes(a.P);
    if (clds > 160 * 1024) return hipErrorInvalidConfiguration;
    if (clds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute((const void*)tiled::consensus_kernel,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)clds);
        if (e != hipSuccess) return e;
    }
    for (int k = 0; k <= a.K; ++k) {
        if (k == a.K && a.U_out == nullptr) break;   // k == K: the final dual update (U_out)
        if (k > 0)   // delta_k from y_k = Y[k-1]
            hipLaunchKernelGGL(tiled::consensus_kernel, dim3(citems), dim3(tiled::THREADS), clds,
                               stream, a, (const float*)(a.Y + (size_t)(k - 1) * S));
        hipLaunchKernelGGL(kern, dim3(items), dim3(tiled::THREADS), lds, stream, a, k);
    }
    return hipGetLastError();
}

}  // namespace dadmm
