// dadmm_hyper.hip — the GNN hypernetwork of DLASSO_GNNHyp3_Progressive, inference mode, as
// f32 MFMA GEMMs with fused epilogues (gnn_dlasso_models_progressive.py:9-72 GNNHypernetwork3,
// :93-123 decoder / fc, :165-196 the hyper-parameter head).
//
// Per iteration the hypernetwork is (B samples of P nodes, h = GHyp_hidden):
//   x0 = cat(AtAy_k, Atb)                         [B*P, 2n]
//   x_i = BN_i(leaky(A_hat (x_{i-1} W_i^T) + b_i))  i = 1..5   (GCNConv -> leaky_relu -> bn_i;
//                                                   Dropout is the identity in eval mode)
//   e = LayerNorm(x_5)                            per node, 4h
//   d = LReLU(LN(e.view(B, P*4h) D1^T + c1)) ... three decoder blocks
//   hyp = head(sigmoid(d fc^T + f))               clamp [1e-4, 0.9999], * max, clamp <= 0.9999
// The reference runs it per sample through torch_geometric (from_networkx + GCNConv) in a Python
// loop; here every stage is ONE launch over the whole batch:
//   linear_kernel<MB, EPI_GCN>  : Z = X W^T on v_mfma_f32_16x16x4_f32 (exact f32 fma chains), then
//                                 in the epilogue, per sample, the normalised-adjacency mix
//                                 sum_q A_hat[p][q] Z[q] + bias, leaky_relu, BatchNorm (running
//                                 statistics) — the tile holds whole samples, so the mix never
//                                 leaves the workgroup;
//   linear_kernel<MB, EPI_BIAS> : decoder linears;
//   linear_kernel<MB, EPI_HEAD> : fc + sigmoid + clamps + maxima, written as hyp_k [B][4][H]
//                                 (the reference's view(B, 4, H) layout);
//   rownorm_kernel              : LayerNorm (+ LeakyReLU) of every row, one wave per row.
// Tile: 32*WR rows (whole samples for the GCN epilogue) x 64 output columns, 4 waves in a 2 x 2
// layout; operands stream through an LDS-DMA ring on long K loops, a per-wave register ring on
// short ones.
// Numerics: f32 throughout; results match torch's eager hypernetwork to f32 rounding (the sums
// run in a different order than hipBLASLt's), not bit-for-bit.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "dadmm_internal.h"

namespace dadmm {
namespace hyper {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int THREADS = 256;
constexpr int TN = 64;            // output columns per workgroup (4 waves x 16)
constexpr int ZS = TN + 4;        // LDS row stride of the GCN epilogue tile (float4 rows)

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
// scheduling barrier: pins where the ring's loads issue (between the steps' MFMAs)
__device__ __forceinline__ void mem_fence() { __builtin_amdgcn_sched_barrier(0); }

// Main-loop operand staging. DMA = 1: the workgroup's A rows and W columns of a k-step go HBM/L2
// -> LDS once (LDS-DMA, lane-linear 1 KB fragment images, DQ k-steps in flight) and every wave
// reads its MFMA fragments from there; DMA = 0: each wave streams its own fragments into a
// register ring (the two waves that share a row block, or a column block, both fetch it).
constexpr int HYPER_DMA_MIN = 32;  // k-steps per workgroup from which the DMA ring is used
constexpr int HYPER_DQ = 4;
constexpr int HYPER_D1 = 4;
typedef __amdgpu_buffer_rsrc_t rsrc_t;
typedef __attribute__((address_space(3))) void lds_void;
__device__ __forceinline__ rsrc_t make_rsrc(const void* base, size_t bytes) {
    const uint32_t nb = bytes > 0xFFFFFFF0ull ? 0xFFFFFFF0u : (uint32_t)bytes;
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)nb, 0x00020000);
}
// one lane-linear 1 KB LDS-DMA: lane l's 16 bytes from voff land at lds + 16 l
__device__ __forceinline__ void dma16(rsrc_t r, float* lds, uint32_t voff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)lds, 16, voff, 0, 0, 0);
}
// s_waitcnt vmcnt(n) for a runtime n (the wait counts of the DMA ring depend on the wave)
__device__ __forceinline__ void wait_vm(int n) {
    switch (n) {
        case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
        case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
        case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
        case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
        case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
        case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
        case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
        case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
        case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
        case 11: asm volatile("s_waitcnt vmcnt(11)" ::: "memory"); break;
        case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
        case 13: asm volatile("s_waitcnt vmcnt(13)" ::: "memory"); break;
        case 14: asm volatile("s_waitcnt vmcnt(14)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(15)" ::: "memory"); break;
    }
}
// this wave's LDS reads done, then the workgroup barrier (no vmcnt drain: DMAs stay in flight)
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// XCD-aware tile order: the dispatcher deals blocks round-robin over the 8 XCDs (each with its
// own L2); consecutive tile numbers — the column tiles of one row tile, which read the same input
// rows — are given to blocks of one XCD.
__device__ __forceinline__ int xcd_tile(int bid, int G) {
    constexpr int NX = 8;
    const int xcd = bid % NX, i = bid / NX, q = G / NX, r = G % NX;
    return xcd < r ? xcd * (q + 1) + i : r * (q + 1) + (xcd - r) * q + i;
}

// Workgroup tile: 32 WR rows x 64 columns, 4 waves in a 2 x 2 layout; wave (wr, wc) owns row
// blocks wr WR .. wr WR + WR - 1 and column blocks 2 wc, 2 wc + 1 (16 x 16 each, WR x 2 MFMA
// accumulators). Operands stream from L2 into a register ring D k-steps (16 k) deep; rows past the
// tile / columns past N load clamped (valid) rows whose results are never stored, so the main loop
// has no masks; a K tail that is not a multiple of 16 runs as one masked step.
// KS = 2 (small grids, register ring only): 8 waves, the two halves of the tile's k-steps on two
// wave sets (kh = 0: the first half), added through LDS once (first half + second half) before the
// epilogue, which then runs on all 512 threads. Each wave's dependent chain is half as long; the
// result differs from the KS = 1 chain by that one association (launch_hyper decides KS from the
// GEMM shape alone, so every caller of one shape gets the same bits).
template <int WR, int EPI, bool SPLIT, bool DMA, int KS>
__global__ __launch_bounds__(THREADS * KS) void linear_kernel(HyperArgs a) {
    static_assert(KS == 1 || (KS == 2 && !DMA), "the K split runs on the register ring");
    constexpr int NT = THREADS * KS;               // threads per workgroup
    // register ring depth (k-steps in flight; 2 waves/SIMD); HYPER_D1: the depth of the
    // one-row-block tiles (small batches: one workgroup per CU, latency-bound K loops)
    [[maybe_unused]] constexpr int D = WR >= 5 ? 3 : (WR == 1 ? HYPER_D1 : 4);
    constexpr int TM = 32 * WR;                    // rows per workgroup tile
    extern __shared__ __attribute__((aligned(16))) float zt[];   // GCN epilogue (dynamic)
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int j = lane & 15, h = lane >> 4;
    const int wq = w & 3, kh = KS == 2 ? (w >> 2) : 0;   // the wave's tile position, its k half
    const int wr = wq >> 1, wcol = wq & 1;

    const int gm = a.gm, gn = a.gn;
    const int tl = xcd_tile(blockIdx.x, gridDim.x);
    const int ct = tl % gn, rt = (tl / gn) % gm, split = tl / (gn * gm);

    constexpr bool GCN = EPI == HYPER_EPI_GCN || EPI == HYPER_EPI_GCN_TRAIN || EPI == HYPER_EPI_GCN_BWD;
    int row0, rows_t, s0 = 0;
    if (GCN) {
        s0 = rt * a.S_t;
        const int ns = a.B - s0 < a.S_t ? a.B - s0 : a.S_t;
        row0 = s0 * a.P;
        rows_t = ns * a.P;
    } else {
        row0 = rt * TM;
        rows_t = a.rows - row0 < TM ? a.rows - row0 : TM;
    }
    const int col0 = ct * TN;
    const int K = a.K, K1 = a.K1;
    // k-steps of this split: [t_begin, t_end) of the full steps, plus the tail step in the last
    const int KF = K / 16;                          // full 16-wide steps
    const int per = (KF + a.splits - 1) / a.splits;
    int t_begin = split * per;
    int t_end = t_begin + per < KF ? t_begin + per : KF;
    if constexpr (KS == 2) {   // the wave set's half (the first half the longer one)
        const int mid = t_begin + (t_end - t_begin + 1) / 2;
        if (kh == 0) t_end = mid;
        else t_begin = mid;
    }
    const bool tail = (K & 15) != 0 && split == a.splits - 1 && kh == KS - 1;

    // operand rows (clamped into range)
    size_t oa[WR], ob[WR];
#pragma unroll
    for (int i = 0; i < WR; ++i) {
        int r = 16 * (wr * WR + i) + j;
        r = r < rows_t ? r : rows_t - 1;
        oa[i] = (size_t)(row0 + r) * a.ld1 + 4 * h;
        ob[i] = (size_t)(row0 + r) * a.ld2 + 4 * h;
    }
    size_t ow[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        int n = col0 + 16 * (2 * wcol + c) + j;
        n = n < a.N ? n : a.N - 1;
        ow[c] = (size_t)n * a.ldw + 4 * h;
    }

    const f32x4 zero = {0.0f, 0.0f, 0.0f, 0.0f};
    f32x4 acc[WR][2];
#pragma unroll
    for (int i = 0; i < WR; ++i) acc[i][0] = acc[i][1] = zero;

    auto mma = [&](const f32x4 (&av)[WR], const f32x4 (&bv)[2]) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int i = 0; i < WR; ++i)
#pragma unroll
                for (int c = 0; c < 2; ++c) acc[i][c] = mfma4(av[i][r], bv[c][r], acc[i][c]);
    };
    // steps [tb, te) of one input segment: X columns 16 t - koff at x + o[i]. The steady-state
    // loop is straight-line (no conditional loads), so the compiler's vmcnt waits count exactly
    // the D - 1 younger steps in flight instead of draining the queue every step.
    auto segment = [&](const float* __restrict__ x, const size_t (&o)[WR], int koff, int tb, int te) {
        f32x4 ar[D][WR], br[D][2];
        auto load = [&](int u, int t) {
#pragma unroll
            for (int i = 0; i < WR; ++i) ar[u][i] = *(const f32x4*)(x + o[i] + (16 * t - koff));
#pragma unroll
            for (int c = 0; c < 2; ++c) br[u][c] = *(const f32x4*)(a.W + ow[c] + 16 * t);
        };
        if (te - tb < D) {   // short segment: no ring
            for (int t = tb; t < te; ++t) {
                load(0, t);
                mma(ar[0], br[0]);
            }
            return;
        }
#pragma unroll
        for (int u = 0; u < D; ++u) load(u, tb + u);
        // one group: D steps, each followed by the loads of the step D ahead (pinned there)
        auto group = [&](int t0) {
#pragma unroll
            for (int u = 0; u < D; ++u) {
                mma(ar[u], br[u]);
                load(u, t0 + u + D);
                mem_fence();
            }
        };
        // two groups per trip: the compiler's waits at the loop head are conservative (they
        // drain the queue), so a longer body exposes that latency less often
        int t0 = tb;
        for (; t0 + 3 * D <= te; t0 += 2 * D) {
            group(t0);
            group(t0 + D);
        }
        if (t0 + 2 * D <= te) {
            group(t0);
            t0 += D;
        }
        // te - t0 in [D, 2D): one group with its remaining prefetches, then the last steps
#pragma unroll
        for (int u = 0; u < D; ++u) {
            mma(ar[u], br[u]);
            if (t0 + u + D < te) load(u, t0 + u + D);
        }
        t0 += D;
#pragma unroll
        for (int u = 0; u < D; ++u)
            if (t0 + u < te) mma(ar[u], br[u]);
    };
    // GCN_BWD: the block's saved M tile [rows][64] and its samples' BatchNorm statistics go
    // HBM -> LDS (LDS-DMA) now, under the GEMM, into a region past the ring and the epilogue tile
    // (the epilogue then never waits on memory; its loads were the fused kernel's critical path)
    [[maybe_unused]] float* pf = nullptr;
    [[maybe_unused]] const int SR = (a.S_t + 3) & ~3;
    if constexpr (EPI == HYPER_EPI_GCN_BWD) {
        constexpr int RING = DMA ? HYPER_DQ * (2 * WR + 4) * 256 : 0;   // floats
        const int epi = TM * ZS + ((a.S_t * a.P * a.P + 3) & ~3) + 4 * TN;
        pf = zt + (RING > epi ? RING : epi);
        float* pst = pf + TM * TN;                                   // mean [SR][64], var [SR][64]
        const rsrc_t rm = make_rsrc(a.save_m, (size_t)a.B * a.P * a.N * 4);
        const rsrc_t rmu = make_rsrc(a.save_mean, (size_t)a.B * a.N * 4);
        const rsrc_t rva = make_rsrc(a.save_var, (size_t)a.B * a.N * 4);
        const int rr = lane >> 4, c4 = 4 * (lane & 15);   // lane-linear: 4 rows x 64 columns per copy
        for (int q = w; 4 * q < rows_t; q += 4 * KS)
            dma16(rm, pf + q * 256, (uint32_t)(((size_t)(row0 + 4 * q + rr) * a.N + col0 + c4) * 4));
        const int nsm = rows_t / a.P;
        for (int q = w; 4 * q < nsm; q += 4 * KS) {
            const uint32_t o = (uint32_t)(((size_t)(s0 + 4 * q + rr) * a.N + col0 + c4) * 4);
            dma16(rmu, pst + q * 256, o);
            dma16(rva, pst + SR * TN + q * 256, o);
        }
    }
    if constexpr (DMA) {
        // ring slot: the tile's NBA row blocks, then its 4 column blocks (16 x 16 floats each, as
        // lane-linear fragment images: lane (j, h) of block q holds row/column 16 q + j, k 4h..4h+3)
        constexpr int DQ = HYPER_DQ;
        constexpr int NBA = 2 * WR, NB = NBA + 4, NBW = (NB + 3) / 4, SLOT = NB * 256;
        const int wu = __builtin_amdgcn_readfirstlane(w) & 3;   // provably uniform, in [0, 4)
        const int nbw = NB % 4 == 0 ? NB / 4 : (NB - wu + 3) / 4;   // blocks this wave copies per k-step
        const int T = t_end - t_begin, t1 = SPLIT ? K1 / 16 : KF;
        const int kq = 4 * (lane >> 4);
        const rsrc_t rx1 = make_rsrc(a.x1 + (size_t)row0 * a.ld1, (size_t)rows_t * a.ld1 * 4);
        const rsrc_t rx2 = make_rsrc(SPLIT ? a.x2 + (size_t)row0 * a.ld2 : a.x1, SPLIT ? (size_t)rows_t * a.ld2 * 4 : 0);
        const rsrc_t rw = make_rsrc(a.W, (size_t)a.N * a.ldw * 4);
        uint32_t o1[NBW], o2[NBW];
#pragma unroll
        for (int i = 0; i < NBW; ++i) {
            const int q = wu + 4 * i;
            if (q < NBA) {
                int r = 16 * q + j;
                r = r < rows_t ? r : rows_t - 1;
                o1[i] = (uint32_t)(((size_t)r * a.ld1 + kq) * 4);
                o2[i] = SPLIT ? (uint32_t)(((size_t)r * a.ld2 + kq) * 4) : 0u;
            } else {
                int nn = col0 + 16 * (q - NBA) + j;
                nn = nn < a.N ? nn : a.N - 1;
                o1[i] = o2[i] = (uint32_t)(((size_t)nn * a.ldw + kq) * 4);
            }
        }
        auto dma = [&](int t) {
            float* slot = zt + ((t - t_begin) % DQ) * SLOT;
            const bool seg2 = SPLIT && t >= t1;
            const uint32_t ka = seg2 ? (uint32_t)(64 * t - 4 * K1) : (uint32_t)(64 * t);
#pragma unroll
            for (int i = 0; i < NBW; ++i) {
                const int q = wu + 4 * i;
                if (q < NBA) {
                    if (seg2)
                        dma16(rx2, slot + q * 256, o2[i] + ka);
                    else
                        dma16(rx1, slot + q * 256, o1[i] + ka);
                } else if (q < NB) {
                    dma16(rw, slot + q * 256, o1[i] + (uint32_t)(64 * t));
                }
            }
        };
        auto frag = [&](f32x4 (&fa)[WR], f32x4 (&fb)[2], int t) {
            const float* slot = zt + ((t - t_begin) % DQ) * SLOT + 4 * lane;
#pragma unroll
            for (int i = 0; i < WR; ++i) fa[i] = *(const f32x4*)(slot + (wr * WR + i) * 256);
#pragma unroll
            for (int c = 0; c < 2; ++c) fb[c] = *(const f32x4*)(slot + (NBA + 2 * wcol + c) * 256);
        };
        // step u: wait for step u + 1's copies (this wave's: the count of its younger DMAs), the
        // barrier (every wave's), refill the slot step u - 1 left, then step u's MFMAs with step
        // u + 1's fragment reads issued after the first quarter of them. Branch-free but for the
        // refill (past the last step the wait is vmcnt(0) and the reads are of a stale slot, never
        // used), so the compiler's LDS-read waits are exact and no MFMA waits for the next reads.
        auto body = [&](int u, f32x4 (&fa)[WR], f32x4 (&fb)[2], f32x4 (&na)[WR], f32x4 (&nb)[2]) {
            int younger = DQ - 2 < T - 2 - u ? DQ - 2 : T - 2 - u;
            younger = younger > 0 ? younger : 0;
            wait_vm(nbw * younger);
            lds_barrier();
            if (u + DQ < T) dma(t_begin + u + DQ);
#pragma unroll
            for (int i = 0; i < WR; ++i)
#pragma unroll
                for (int c = 0; c < 2; ++c) acc[i][c] = mfma4(fa[i][0], fb[c][0], acc[i][c]);
            mem_fence();
            frag(na, nb, t_begin + u + 1);
            mem_fence();
#pragma unroll
            for (int r = 1; r < 4; ++r)
#pragma unroll
                for (int i = 0; i < WR; ++i)
#pragma unroll
                    for (int c = 0; c < 2; ++c) acc[i][c] = mfma4(fa[i][r], fb[c][r], acc[i][c]);
        };
        if (T > 0) {
            const int pre = T < DQ ? T : DQ;
            for (int u = 0; u < pre; ++u) dma(t_begin + u);
            wait_vm(nbw * (pre - 1));
            lds_barrier();
            f32x4 fa0[WR], fb0[2], fa1[WR], fb1[2];
            frag(fa0, fb0, t_begin);
            for (int u = 0; u < T; u += 2) {
                body(u, fa0, fb0, fa1, fb1);
                if (u + 1 < T) body(u + 1, fa1, fb1, fa0, fb0);
            }
            lds_barrier();   // the ring's last reads before the epilogue reuses the LDS
        }
    } else if constexpr (SPLIT) {   // cat(x1, x2): K1 is a multiple of 16 (checked by the launcher)
        const int t1 = K1 / 16;
        segment(a.x1, oa, 0, t_begin, t_end < t1 ? t_end : t1);
        segment(a.x2, ob, K1, t_begin > t1 ? t_begin : t1, t_end);
    } else {
        segment(a.x1, oa, 0, t_begin, t_end);
    }
    if (tail) {   // the last (K mod 16) columns: lanes past K load zeros
        const int t = KF, k = 16 * t + 4 * h;
        const bool kin = k < K;
        f32x4 av[WR], bv[2];
#pragma unroll
        for (int i = 0; i < WR; ++i) {
            const float* src = (SPLIT && k >= K1) ? a.x2 + ob[i] + (16 * t - K1)
                                                  : a.x1 + oa[i] + 16 * t;
            av[i] = kin ? *(const f32x4*)src : zero;
        }
#pragma unroll
        for (int c = 0; c < 2; ++c) bv[c] = kin ? *(const f32x4*)(a.W + ow[c] + 16 * t) : zero;
        mma(av, bv);
    }
    if constexpr (KS == 2) {   // acc = (first half) + (second half), on the kh = 0 waves
        __shared__ f32x4 kred[4 * 2 * WR * 64];
        if (kh == 1) {
#pragma unroll
            for (int i = 0; i < WR; ++i)
#pragma unroll
                for (int c = 0; c < 2; ++c) kred[((wq * WR + i) * 2 + c) * 64 + lane] = acc[i][c];
        }
        __syncthreads();
        if (kh == 0) {
#pragma unroll
            for (int i = 0; i < WR; ++i)
#pragma unroll
                for (int c = 0; c < 2; ++c) acc[i][c] = acc[i][c] + kred[((wq * WR + i) * 2 + c) * 64 + lane];
        }
    }

    // lane (j, h) holds rows 16 (wr WR + i) + 4 h + r of column col0 + 16 (2 wcol + c) + j
    // (KS = 2: the kh = 0 waves hold the sums)
    if constexpr (!GCN) {
        if (kh != 0) return;
        float* y = a.y + (size_t)split * a.split_stride;
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const int col = col0 + 16 * (2 * wcol + c) + j;
            if (col >= a.N) continue;
            float bv = 0.0f, mx = 1.0f;
            int ch = 0;
            if (EPI == HYPER_EPI_BIAS && a.bias != nullptr) bv = a.bias[col];
            if (EPI == HYPER_EPI_HEAD) {
                bv = a.bias[col];
                ch = col / a.H;                         // view(B, 4, H): channel of fc output col
                mx = a.maxv[ch];
            }
#pragma unroll
            for (int i = 0; i < WR; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int rr = 16 * (wr * WR + i) + 4 * h + r;
                    if (rr >= rows_t) continue;
                    float v = acc[i][c][r] + bv;
                    // y = addend + x W^T in place (the adjoint's gradient accumulation; unsplit only)
                    if (EPI == HYPER_EPI_BIAS && a.addend != nullptr)
                        v = a.addend[(size_t)(row0 + rr) * a.ld_add + col] + v;
                    if (EPI == HYPER_EPI_HEAD) {
                        // training: the logits too (the head's backward reads them)
                        if (a.save_m != nullptr) a.save_m[(size_t)(row0 + rr) * a.ldy + col] = v;
                        v = 1.0f / (1.0f + expf(-v));                  // torch.sigmoid  (:170)
                        v = fminf(fmaxf(v, 1e-4f), 0.9999f);          // clamp          (:171)
                        v = v * mx;                                   // * *_max        (:180-189)
                        if (ch > 0) v = fminf(v, 0.9999f);            // tau/rho/eta    (:194-196)
                    }
                    y[(size_t)(row0 + rr) * a.ldy + col] = v;
                }
        }
    } else {
        // GCN epilogue. LDS: Z tile [TM][ZS] (ZS = 68: float4 rows), the tile's normalised
        // adjacency blocks [S_t][P][P], per-column (bias, BN mean, BN scale, BN shift) [4][64].
        // Output (node p of sample s, columns c..c+3):
        //   BN(leaky(sum_q A_hat[s][p][q] Z[s, q][c] + bias[c])), BatchNorm on running statistics
        const int P = a.P;
        float* ahs = zt + TM * ZS;                     // [S_t][P][P]
        float* colp = ahs + ((a.S_t * P * P + 3) & ~3);
        if (kh == 0) {
#pragma unroll
            for (int i = 0; i < WR; ++i)
#pragma unroll
                for (int c = 0; c < 2; ++c)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        zt[(16 * (wr * WR + i) + 4 * h + r) * ZS + 16 * (2 * wcol + c) + j] = acc[i][c][r];
        }
        const int ns = rows_t / P;
        const float* agl = a.ahat + (a.ahat_per_sample ? (size_t)s0 * P * P : 0);
        if (a.ahat_per_sample) {
            for (int i = threadIdx.x; i < ns * P * P; i += NT) ahs[i] = agl[i];
        } else {
            for (int i = threadIdx.x; i < P * P; i += NT)
                for (int sl = 0; sl < ns; ++sl) ahs[sl * P * P + i] = agl[i];
        }
        const int cols = a.N - col0 < TN ? a.N - col0 : TN;
        // the mix sum_q A_hat[p][q] Z[q] of 4 nodes x 4 columns per task: each q reads four A_hat
        // words and one Z quad for 16 fma (one node x 4 columns per task read two LDS words per
        // 4 fma and made the epilogue as long as the 400-deep GEMM). emit(row, col, sums).
        auto mix = [&](auto&& emit) {
            const int ng = (P + 3) >> 2;
            for (int task = threadIdx.x; task < ns * ng * (TN / 4); task += NT) {
                const int cq = task % (TN / 4), rest = task / (TN / 4);
                const int g = rest % ng, sl = rest / ng;
                const int c = 4 * cq;
                if (c >= cols) continue;
                const float* at[4];                    // rows 4g..4g+3 (clamped: never emitted)
#pragma unroll
                for (int e = 0; e < 4; ++e) at[e] = ahs + (sl * P + (4 * g + e < P ? 4 * g + e : P - 1)) * P;
                const float* zc = zt + sl * P * ZS + c;
                f32x4 v[4] = {zero, zero, zero, zero};
                for (int q = 0; q < P; ++q) {
                    const f32x4 z = *(const f32x4*)(zc + q * ZS);
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] = __builtin_elementwise_fma((f32x4)(at[e][q]), z, v[e]);
                }
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    if (4 * g + e < P) emit(sl * P + 4 * g + e, c, v[e]);
            }
        };
        if constexpr (EPI == HYPER_EPI_GCN_BWD) {
            // the GCN block backward of the layer whose output gradient dy this GEMM produced (the
            // tile holds whole samples and 64 of its columns: everything gcn_bwd_kernel reads per
            // (sample, column)); the same operations in the same order as gcn_bwd_kernel's loop
            // form, so dz and the partial sums are bit-identical to the unfused pair of launches
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's prefetch copies landed
            __syncthreads();
            const float* pmu = pf + TM * TN;
            const float* pva = pmu + SR * TN;
            const uint32_t thr = drop_threshold(a.drop_p);
            const float scale = a.drop_p > 0.0f ? 1.0f / (1.0f - a.drop_p) : 1.0f;
            const float inv = 1.0f / (float)P;
            for (int task = threadIdx.x; task < ns * TN; task += NT) {
                const int sl = task / TN, c = task - sl * TN;
                if (c >= cols) continue;
                const int col = col0 + c, s = s0 + sl;
                const size_t rs = (size_t)row0 + (size_t)sl * P;
                const float mean = pmu[sl * TN + c];
                const float rstd = 1.0f / sqrtf(pva[sl * TN + c] + a.bn_eps);
                const float gam = a.bn_w[col];
                float* dc = zt + sl * P * ZS + c;
                const float* mc = pf + sl * P * TN + c;
                float sb = 0.0f, sg = 0.0f, sbias = 0.0f;
                for (int p = 0; p < P; ++p) {   // dxn = dropout'(dy), the two BatchNorm sums
                    const float mv = mc[p * TN];
                    const float t = mv > 0.0f ? mv : mv * a.slope;
                    const float xh = (t - mean) * rstd;
                    float g = dc[p * ZS];
                    if (a.drop_p > 0.0f)
                        g = drop_hash(a.seed, a.site, (uint32_t)(rs + p), (uint32_t)col) >= thr ? g * scale : 0.0f;
                    sb += g;
                    sg += g * xh;
                    dc[p * ZS] = g;
                }
                for (int p = 0; p < P; ++p) {   // BatchNorm and leaky_relu backward -> dM
                    const float mv = mc[p * TN];
                    const float t = mv > 0.0f ? mv : mv * a.slope;
                    const float xh = (t - mean) * rstd;
                    const float g = dc[p * ZS];
                    const float dt = a.bn_eval ? gam * rstd * g : gam * rstd * (g - sb * inv - xh * (sg * inv));
                    const float d = mv > 0.0f ? dt : dt * a.slope;
                    sbias += d;
                    dc[p * ZS] = d;
                }
                a.part[(size_t)s * a.N + col] = sg;                       // dgamma
                a.part[((size_t)a.B + s) * a.N + col] = sb;               // dbeta
                a.part[((size_t)2 * a.B + s) * a.N + col] = sbias;        // dbias (GCNConv.bias)
            }
            __syncthreads();
            // dZ[q] = sum_p A_hat[p][q] dM[p] (the mix, transposed), 4 columns per task
            for (int task = threadIdx.x; task < rows_t * (TN / 4); task += NT) {
                const int r = task / (TN / 4), c = 4 * (task - r * (TN / 4));
                if (c >= cols) continue;
                const int sl = r / P, q = r - sl * P;
                const float* ah = ahs + sl * P * P;
                const float* dm = zt + sl * P * ZS + c;
                f32x4 acc4 = zero;
                for (int p = 0; p < P; ++p) {
                    const f32x4 d4 = *(const f32x4*)(dm + p * ZS);
                    const float w = ah[p * P + q];
#pragma unroll
                    for (int e = 0; e < 4; ++e) acc4[e] += w * d4[e];
                }
                float* dst = a.y + (size_t)(row0 + r) * a.ldy + col0 + c;
                if (c + 4 <= cols) {
                    *(f32x4*)dst = acc4;
                } else {
                    for (int e = 0; e < cols - c; ++e) dst[e] = acc4[e];
                }
            }
            return;
        }
        if constexpr (EPI == HYPER_EPI_GCN_TRAIN) {
            // training: BatchNorm on each sample's own statistics over its P nodes, then Dropout
            //   pass 1: M = A_hat Z + bias (LDS mt, and saved for the backward)
            //   pass 2: per (sample, column): mean and biased variance of leaky(M) over the P nodes
            //   pass 3: y = Dropout((leaky(M) - mean) / sqrt(var + eps) * gamma + beta)
            float* mt = colp + 4 * TN;                 // [TM][ZS]
            float* smean = mt + TM * ZS;               // [S_t][TN]
            float* srstd = smean + a.S_t * TN;         // [S_t][TN]
            if (threadIdx.x < TN) {
                const int col = col0 + threadIdx.x < a.N ? col0 + threadIdx.x : a.N - 1;
                colp[threadIdx.x] = a.bias[col];
                colp[2 * TN + threadIdx.x] = a.bn_w[col];
                colp[3 * TN + threadIdx.x] = a.bn_b[col];
            }
            __syncthreads();
            mix([&](int r, int c, f32x4 v) {
                if (a.addend != nullptr) {   // layer 1's Atb half (formed once per forward)
                    const float* src = a.addend + (size_t)(row0 + r) * a.ld_add + col0 + c;
                    f32x4 ad = zero;
                    if (c + 4 <= cols) {
                        ad = *(const f32x4*)src;
                    } else {
                        for (int e = 0; e < cols - c; ++e) ad[e] = src[e];
                    }
                    v = v + ad;
                }
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = v[e] + colp[c + e];
                *(f32x4*)(mt + r * ZS + c) = v;
                float* dst = a.save_m + (size_t)(row0 + r) * a.N + col0 + c;
                if (c + 4 <= cols) {
                    *(f32x4*)dst = v;
                } else {
                    for (int e = 0; e < cols - c; ++e) dst[e] = v[e];
                }
            });
            __syncthreads();
            for (int task = threadIdx.x; task < ns * TN; task += NT) {
                const int sl = task / TN, c = task - sl * TN;
                if (c >= cols) continue;
                if (a.bn_mean != nullptr) {
                    // eval-mode BatchNorm (model.eval() with autograd): the running statistics,
                    // saved per sample like batch statistics for the backward
                    const float mean = a.bn_mean[col0 + c], var = a.bn_var[col0 + c];
                    smean[sl * TN + c] = mean;
                    srstd[sl * TN + c] = 1.0f / sqrtf(var + a.bn_eps);
                    a.save_mean[(size_t)(s0 + sl) * a.N + col0 + c] = mean;
                    a.save_var[(size_t)(s0 + sl) * a.N + col0 + c] = var;
                    continue;
                }
                const float* mc = mt + sl * P * ZS + c;
                float sum = 0.0f;
                for (int q = 0; q < P; ++q) {
                    const float t = mc[q * ZS];
                    sum += t > 0.0f ? t : t * a.slope;
                }
                const float mean = sum / (float)P;
                float sq = 0.0f;
                for (int q = 0; q < P; ++q) {
                    const float t = mc[q * ZS];
                    const float d = (t > 0.0f ? t : t * a.slope) - mean;
                    sq += d * d;
                }
                const float var = sq / (float)P;
                smean[sl * TN + c] = mean;
                srstd[sl * TN + c] = 1.0f / sqrtf(var + a.bn_eps);
                a.save_mean[(size_t)(s0 + sl) * a.N + col0 + c] = mean;
                a.save_var[(size_t)(s0 + sl) * a.N + col0 + c] = var;
            }
            __syncthreads();
            const uint32_t thr = drop_threshold(a.drop_p);
            const float scale = a.drop_p > 0.0f ? 1.0f / (1.0f - a.drop_p) : 1.0f;
            for (int task = threadIdx.x; task < rows_t * (TN / 4); task += NT) {
                const int r = task / (TN / 4), c = 4 * (task - r * (TN / 4));
                if (c >= cols) continue;
                const int sl = r / P;
                const f32x4 v = *(const f32x4*)(mt + r * ZS + c);
                f32x4 o;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float t = v[e] > 0.0f ? v[e] : v[e] * a.slope;
                    float u = (t - smean[sl * TN + c + e]) * srstd[sl * TN + c + e] * colp[2 * TN + c + e] +
                              colp[3 * TN + c + e];
                    if (a.drop_p > 0.0f) {
                        const bool keep = drop_hash(a.seed, a.site, (uint32_t)(row0 + r),
                                                    (uint32_t)(col0 + c + e)) >= thr;
                        u = keep ? u * scale : 0.0f;
                    }
                    o[e] = u;
                }
                float* dst = a.y + (size_t)(row0 + r) * a.ldy + col0 + c;
                if (c + 4 <= cols) {
                    *(f32x4*)dst = o;
                } else {
                    for (int e = 0; e < cols - c; ++e) dst[e] = o[e];
                }
            }
            return;
        }
        if (threadIdx.x < TN && !a.raw) {
            const int col = col0 + threadIdx.x < a.N ? col0 + threadIdx.x : a.N - 1;
            const float sc = (1.0f / sqrtf(a.bn_var[col] + a.bn_eps)) * a.bn_w[col];
            colp[threadIdx.x] = a.bias[col];
            colp[TN + threadIdx.x] = a.bn_mean[col];
            colp[2 * TN + threadIdx.x] = sc;
            colp[3 * TN + threadIdx.x] = a.bn_b[col];
        }
        __syncthreads();
        mix([&](int r, int c, const f32x4& v) {
            f32x4 o, ad = zero;
            if (a.addend != nullptr) {   // e.g. layer 1's Atb half, formed once per forward
                const float* src = a.addend + (size_t)(row0 + r) * a.ld_add + col0 + c;
                if (c + 4 <= cols) {
                    ad = *(const f32x4*)src;
                } else {
                    for (int e = 0; e < cols - c; ++e) ad[e] = src[e];
                }
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float t = a.addend != nullptr ? v[e] + ad[e] : v[e];
                if (!a.raw) {
                    t = t + colp[c + e];
                    t = t > 0.0f ? t : t * a.slope;
                    t = (t - colp[TN + c + e]) * colp[2 * TN + c + e] + colp[3 * TN + c + e];
                }
                o[e] = t;
            }
            float* dst = a.y + (size_t)(row0 + r) * a.ldy + col0 + c;
            if (c + 4 <= cols) {
                *(f32x4*)dst = o;
            } else {
                for (int e = 0; e < cols - c; ++e) dst[e] = o[e];
            }
        });
    }
}

// ---- GCN layer (inference) on v_mfma_f32_32x32x2_f32, round 4 --------------------------------
// linear_kernel's 16x16x4 tiles move 256 operand bytes per 2048-flop MFMA and its 160-row tiles
// ran the configs[4] 400-wide layers at ~0.43 of the f32 MFMA peak. Here: 256-row x 64-column
// tiles (5 whole samples of 50 nodes: 98 % of the rows used), 8 waves in a 4 x 2 layout, each
// wave 64 x 32 (two 32x32 accumulators, 4096 flop per MFMA from one A and one B VGPR). The k
// dimension streams in 16-wide stages through a DQ-deep LDS ring filled by LDS-DMA (A 16 KB +
// W 4 KB per stage, lane-linear 1 KB pieces whose 16-byte chunks are XOR-swizzled by row, so
// every ds_read_b128 fragment read is bank-conflict free); a lane's b128 read feeds four MFMAs
// (k = 4 kh + s within an 8-wide sub-step: the sum order differs from torch's, not the value
// beyond f32 rounding). Columns past K, rows past the tile and columns past N load as zeros
// (buffer range checks), so the loop is branch-free. The epilogue is linear_kernel's inference
// GCN epilogue (mix with A_hat, the optional addend, bias, leaky_relu, BatchNorm) on the 256-row
// Z tile.
constexpr int G32_TM = 256, G32_WAVES = 8, G32_DQ = 4;
constexpr int G32_STAGE = (G32_TM + TN) * 16;                  // floats per ring stage
// Measured and dropped: the per-sample mix sum_q A_hat[p][q] Z[q] on v_mfma_f32_16x16x4_f32
// instead of VALU fma: output blocks of 16 rows x 16 columns, each summing over the node range of
// the samples its rows belong to (A_hat entries of other samples are zero: a block-diagonal
// operand, ~1.3 samples' width per block), Z from LDS (row stride ZM = 80 floats: the four k rows
// of a fragment read land 16 banks apart), A_hat through the vector cache. Bit-identical to the
// VALU mix (an f32 MFMA is an fma chain in k order, and the zero entries leave it unchanged), but
// slower: 91.9-92.0 vs 84.1-84.2 ms at the configs[4] shard forward (per-lane A_hat gathers and
// one dependent chain per block; profiles/r04/variants_r04q_mfma_mix.txt), so off
__host__ __device__ constexpr size_t g32_lds_bytes(int S_t, int P) {
    const size_t ring = 4 * (size_t)G32_DQ * G32_STAGE;
    const size_t epi = 4 * ((size_t)G32_TM * ZS + 4 * TN);
    return ring > epi ? ring : epi;
}
typedef float f32x16 __attribute__((ext_vector_type(16)));
__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

__global__ __launch_bounds__(64 * G32_WAVES) void gcn32_kernel(HyperArgs a) {
    extern __shared__ __attribute__((aligned(16))) float zt[];
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wr = w >> 1, wc = w & 1;
    const int gn = a.gn;
    const int tl = xcd_tile(blockIdx.x, gridDim.x);
    const int ct = tl % gn, rt = tl / gn;
    const int P = a.P;
    const int s0 = rt * a.S_t;
    const int ns = a.B - s0 < a.S_t ? a.B - s0 : a.S_t;
    const int row0 = s0 * P, rows_t = ns * P;
    const int col0 = ct * TN;
    const int K = a.K, T = (K + 15) / 16;

    // LDS-DMA sources: wave w copies A pieces 2w, 2w + 1 (16 rows each) and, for w < 4, W piece w
    const rsrc_t rx = make_rsrc(a.x1 + (size_t)row0 * a.ld1, (size_t)rows_t * a.ld1 * 4);
    const rsrc_t rw = make_rsrc(a.W, (size_t)a.N * a.ldw * 4);
    const int pos = lane & 3;
    uint32_t oa[2], ka[2], ow = 0, kw = 0;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int r = 16 * (2 * w + i) + (lane >> 2);
        const int chunk = pos ^ ((r >> 2) & 3);
        oa[i] = r < rows_t ? (uint32_t)(((size_t)r * a.ld1 + 4 * chunk) * 4) : 0x80000000u;
        ka[i] = (uint32_t)(4 * chunk);                  // the chunk's first k within a stage
    }
    const bool wdma = w < 4;
    {
        const int c = 16 * (w & 3) + (lane >> 2);
        const int chunk = pos ^ ((c >> 2) & 3);
        ow = col0 + c < a.N ? (uint32_t)(((size_t)(col0 + c) * a.ldw + 4 * chunk) * 4) : 0x80000000u;
        kw = (uint32_t)(4 * chunk);
    }
    const int nper = wdma ? 3 : 2;                      // this wave's DMAs per stage
    auto dma = [&](int t) {
        float* st = zt + (t % G32_DQ) * G32_STAGE;
        const int k0 = 16 * t;
#pragma unroll
        for (int i = 0; i < 2; ++i)
            dma16(rx, st + (2 * w + i) * 256, (k0 + (int)ka[i] < K) ? oa[i] + 4u * k0 : 0x80000000u);
        if (wdma) dma16(rw, st + G32_TM * 16 + (w & 3) * 256, (k0 + (int)kw < K) ? ow + 4u * k0 : 0x80000000u);
    };
    // fragment reads of sub-step c (k 8c .. 8c + 7) of stage t: lane (i = lane & 31, kh = lane >> 5)
    const int fi = lane & 31, kh = lane >> 5;
    int fa[2], fb;
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
        const int R = 64 * wr + 32 * rb + fi;
        fa[rb] = 4 * R;
    }
    const int Cc = 32 * wc + fi;
    fb = 4 * Cc;
    auto swz = [](int rc) { return (rc >> 2) & 3; };
    const int sa0 = swz(64 * wr + fi), sb0 = swz(Cc);   // (32 rb does not change the swizzle)
    struct Frag {
        f32x4 a[2], b;
    };
    auto frag = [&](Frag& f, int t, int c) {
        const float* st = zt + (t % G32_DQ) * G32_STAGE;
        const int chunk = 2 * c + kh;
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) f.a[rb] = *(const f32x4*)(st + 4 * (fa[rb] + (chunk ^ sa0)));
        f.b = *(const f32x4*)(st + G32_TM * 16 + 4 * (fb + (chunk ^ sb0)));
    };
    f32x16 acc[2];
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[rb][e] = 0.0f;
    auto mma = [&](const Frag& f) {
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int rb = 0; rb < 2; ++rb) acc[rb] = mfma32(f.a[rb][s], f.b[s], acc[rb]);
    };
    if (T > 0) {
        const int pre = T < G32_DQ ? T : G32_DQ;
        for (int u = 0; u < pre; ++u) dma(u);
        wait_vm(nper * (pre - 1));
        lds_barrier();
        Frag f0, f1;
        frag(f0, 0, 0);
        for (int u = 0; u < T; ++u) {
            // stage u's sub-step 0 is in f0; read sub-step 1, then wait for stage u + 1 (this
            // wave's copies, then every wave's) and refill stage u's slot once all have read it
            frag(f1, u, 1);
            mma(f0);
            int younger = G32_DQ - 2 < T - 2 - u ? G32_DQ - 2 : T - 2 - u;
            younger = younger > 0 ? younger : 0;
            wait_vm(nper * younger);
            lds_barrier();
            if (u + G32_DQ < T) dma(u + G32_DQ);
            if (u + 1 < T) frag(f0, u + 1, 0);
            mma(f1);
        }
        lds_barrier();   // the ring's last reads before the epilogue reuses the LDS
    }
    // Z tile: acc[rb] register e = row (e & 3) + 8 (e >> 2) + 4 kh of row block rb, column fi
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int e = 0; e < 16; ++e)
            zt[(64 * wr + 32 * rb + (e & 3) + 8 * (e >> 2) + 4 * kh) * ZS + 32 * wc + fi] = acc[rb][e];
    const f32x4 zero = {0.0f, 0.0f, 0.0f, 0.0f};
    // A_hat read through the vector cache (the 16 lanes of a column quad group share each word):
    // the LDS then holds only the ring / Z tile, so two workgroups fit on a CU and one's epilogue
    // runs beside the other's MFMA loop
    const float* ahs = a.ahat + (a.ahat_per_sample ? (size_t)s0 * P * P : 0);
    const int ahs_stride = a.ahat_per_sample ? P * P : 0;
    float* colp = zt + G32_TM * ZS;
    if (threadIdx.x < TN && !a.raw) {
        const int col = col0 + threadIdx.x < a.N ? col0 + threadIdx.x : a.N - 1;
        const float sc = (1.0f / sqrtf(a.bn_var[col] + a.bn_eps)) * a.bn_w[col];
        colp[threadIdx.x] = a.bias[col];
        colp[TN + threadIdx.x] = a.bn_mean[col];
        colp[2 * TN + threadIdx.x] = sc;
        colp[3 * TN + threadIdx.x] = a.bn_b[col];
    }
    __syncthreads();
    const int cols = a.N - col0 < TN ? a.N - col0 : TN;
    const int ng = (P + 3) >> 2;
    for (int task = threadIdx.x; task < ns * ng * (TN / 4); task += 64 * G32_WAVES) {
        const int cq = task % (TN / 4), rest = task / (TN / 4);
        const int g = rest % ng, sl = rest / ng;
        const int c = 4 * cq;
        if (c >= cols) continue;
        const float* at[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) at[e] = ahs + sl * ahs_stride + (4 * g + e < P ? 4 * g + e : P - 1) * P;
        const float* zc = zt + sl * P * ZS + c;
        f32x4 v[4] = {zero, zero, zero, zero};
        int q = 0;
        // A_hat words four nodes at a time, the next four in flight under this group's fma (the
        // loads go through the vector cache: one dependent round trip per group without it)
        typedef float f32x4u __attribute__((ext_vector_type(4), aligned(4)));
        const int P4 = P & ~3;
        if (P4 > 0) {
            f32x4 an[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) an[e] = *(const f32x4u*)at[e];
            for (; q < P4; q += 4) {
                f32x4 ac[4];
                const int qn = q + 4 < P4 ? q + 4 : q;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    ac[e] = an[e];
                    an[e] = *(const f32x4u*)(at[e] + qn);
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const f32x4 z = *(const f32x4*)(zc + (q + u) * ZS);
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] = __builtin_elementwise_fma((f32x4)(ac[e][u]), z, v[e]);
                }
            }
        }
        for (; q < P; ++q) {
            const f32x4 z = *(const f32x4*)(zc + q * ZS);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = __builtin_elementwise_fma((f32x4)(at[e][q]), z, v[e]);
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            if (4 * g + e >= P) continue;
            const int r = sl * P + 4 * g + e;
            f32x4 o, ad = zero;
            if (a.addend != nullptr) {
                const float* src = a.addend + (size_t)(row0 + r) * a.ld_add + col0 + c;
                if (c + 4 <= cols) {
                    ad = *(const f32x4*)src;
                } else {
                    for (int q = 0; q < cols - c; ++q) ad[q] = src[q];
                }
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                float t = a.addend != nullptr ? v[e][q] + ad[q] : v[e][q];
                if (!a.raw) {
                    t = t + colp[c + q];
                    t = t > 0.0f ? t : t * a.slope;
                    t = (t - colp[TN + c + q]) * colp[2 * TN + c + q] + colp[3 * TN + c + q];
                }
                o[q] = t;
            }
            float* dst = a.y + (size_t)(row0 + r) * a.ldy + col0 + c;
            if (c + 4 <= cols) {
                *(f32x4*)dst = o;
            } else {
                for (int q = 0; q < cols - c; ++q) dst[q] = o[q];
            }
        }
    }
}

// LayerNorm over the C columns of every row (biased variance, like torch), then optionally
// LeakyReLU(slope); one wave per row, the row held in registers (C <= 64 * 4 * CH).
// CH: row chunks of 256 columns per lane (the launcher picks the smallest that holds C: fewer
// registers, more rows in flight — the 400-wide encoder norm ran at 2.3 TB/s with CH = 8)
template <int CH>
__global__ __launch_bounds__(THREADS) void rownorm_kernel(RowNormArgs a) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * (THREADS / 64) + (threadIdx.x >> 6);
    if (row >= a.rows) return;
    const float* x = a.x + (size_t)row * a.C;
    const int C4 = a.C / 4;
    f32x4 v[CH];
    float s = 0.0f;
#pragma unroll
    for (int u = 0; u < CH; ++u) {
        const int c4 = lane + 64 * u;
        v[u] = c4 < C4 ? *(const f32x4*)(x + 4 * c4) : (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
        if (c4 < C4) {
            // split-K partial sums of the producing linear, added in split order, then its bias
            for (int q = 1; q < a.nsum; ++q) v[u] += *(const f32x4*)(x + (size_t)q * a.sum_stride + 4 * c4);
            if (a.pre_bias != nullptr) v[u] += *(const f32x4*)(a.pre_bias + 4 * c4);
            if (a.drop_p > 0.0f) {   // training: Dropout on the LayerNorm input (:94-104)
                const uint32_t thr = drop_threshold(a.drop_p);
                const float scale = 1.0f / (1.0f - a.drop_p);
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    v[u][e] = drop_hash(a.seed, a.site, (uint32_t)row, (uint32_t)(4 * c4 + e)) >= thr
                                  ? v[u][e] * scale : 0.0f;
            }
            if (a.xd != nullptr) *(f32x4*)(a.xd + (size_t)row * a.C + 4 * c4) = v[u];
        }
        s += (v[u][0] + v[u][1]) + (v[u][2] + v[u][3]);
    }
    s = ln_row_sum(s);
    const float mean = s / (float)a.C;
    float q = 0.0f;
#pragma unroll
    for (int u = 0; u < CH; ++u) {
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
    const float rstd = 1.0f / sqrtf(q / (float)a.C + a.eps);
    float* y = a.y + (size_t)row * a.C;
#pragma unroll
    for (int u = 0; u < CH; ++u) {
        const int c4 = lane + 64 * u;
        if (c4 >= C4) continue;
        const f32x4 wv = *(const f32x4*)(a.weight + 4 * c4);
        const f32x4 bv = *(const f32x4*)(a.bias + 4 * c4);
        f32x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            float t = (v[u][e] - mean) * rstd * wv[e] + bv[e];
            if (a.act) t = t > 0.0f ? t : t * a.slope;
            o[e] = t;
        }
        *(f32x4*)(y + 4 * c4) = o;
    }
}

template <int WR, int EPI, bool SPLIT, bool DMA, int KS = 1>
hipError_t launch_one(int grid, const HyperArgs& a, hipStream_t st) {
    size_t lds = DMA ? 4 * (size_t)HYPER_DQ * (2 * WR + 4) * 256 : 0;   // the ring
    if (EPI == HYPER_EPI_GCN || EPI == HYPER_EPI_GCN_TRAIN || EPI == HYPER_EPI_GCN_BWD) {   // the epilogue (reuses the ring)
        size_t e = 4 * ((size_t)32 * WR * ZS + (((size_t)a.S_t * a.P * a.P + 3) & ~(size_t)3) + 4 * TN);
        if (EPI == HYPER_EPI_GCN_TRAIN) e += 4 * ((size_t)32 * WR * ZS + 2 * (size_t)a.S_t * TN);
        lds = e > lds ? e : lds;
        // the prefetched M tile and statistics, past both the ring and the epilogue tile
        if (EPI == HYPER_EPI_GCN_BWD) lds += 4 * ((size_t)32 * WR * TN + 2 * (size_t)((a.S_t + 3) & ~3) * TN);
    }
    // (KS = 2: plus the static 8 KB x WR of the K-half sums)
    if (lds + (KS == 2 ? (size_t)8192 * WR : 0) > 160 * 1024) return hipErrorInvalidConfiguration;
    if (lds > 64 * 1024 - (KS == 2 ? (size_t)8192 * WR : 0)) {
        hipError_t e = hipFuncSetAttribute((const void*)linear_kernel<WR, EPI, SPLIT, DMA, KS>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL((linear_kernel<WR, EPI, SPLIT, DMA, KS>), dim3(grid), dim3(THREADS * KS), lds, st, a);
    return hipGetLastError();
}

template <int EPI, bool SPLIT>
hipError_t launch_wr(int wr, bool dma, int ks, int grid, const HyperArgs& a, hipStream_t st) {
    constexpr bool GCN = EPI == HYPER_EPI_GCN || EPI == HYPER_EPI_GCN_TRAIN || EPI == HYPER_EPI_GCN_BWD;
    switch (wr) {
        case 1: return ks == 2 ? launch_one<1, EPI, SPLIT, false, 2>(grid, a, st) : launch_one<1, EPI, SPLIT, false>(grid, a, st);
        case 2: return dma ? launch_one<2, EPI, SPLIT, true>(grid, a, st) : launch_one<2, EPI, SPLIT, false>(grid, a, st);
        case 4: return dma ? launch_one<4, EPI, SPLIT, true>(grid, a, st) : launch_one<4, EPI, SPLIT, false>(grid, a, st);
        case 5:   // 160-row tiles: whole samples with little padding (3 x 50 nodes, 32 x 5)
            if constexpr (GCN)
                return dma ? launch_one<5, EPI, SPLIT, true>(grid, a, st) : launch_one<5, EPI, SPLIT, false>(grid, a, st);
            else
                return hipErrorInvalidValue;
        default: return hipErrorInvalidValue;
    }
}

// the LDS-DMA ring pays for its per-step barrier on long K loops (configs[4]: the 2n-deep first
// GCN layer 360 -> 310 us, the split-K decoder 247 -> 185 us) and not on short ones (the 400-deep
// GCN layers: 191 -> 200 us)
static bool use_dma(int K, int splits) {
    const int per = (K / 16 + splits - 1) / splits;
    return per >= HYPER_DMA_MIN;
}

template <int EPI>
hipError_t launch_epi(int wr, int ks, int grid, const HyperArgs& a, hipStream_t st) {
    const bool dma = use_dma(a.K, a.splits);
    if (a.K1 < a.K) return launch_wr<EPI, true>(wr, dma, ks, grid, a, st);
    return launch_wr<EPI, false>(wr, dma, ks, grid, a, st);
}

}  // namespace hyper

// Row tiling: the largest tile (32 WR rows; whole samples of P rows for the GCN epilogue) that
// still gives ~two workgroups per CU; smaller tiles for small batches.
static int pick_tiles(HyperArgs& a, int epi) {
    const bool gcn = epi == HYPER_EPI_GCN || epi == HYPER_EPI_GCN_TRAIN || epi == HYPER_EPI_GCN_BWD;
    const int unit = gcn ? a.P : 1;                             // rows per tiling unit
    const int units = gcn ? a.B : a.rows;
    a.gn = (a.N + hyper::TN - 1) / hyper::TN;
    if (gcn) {
        // whole samples per tile: the candidate that wastes the fewest padding rows among those
        // whose grid still gives ~two workgroups per CU (P = 50: 160-row tiles hold 150 rows,
        // 128-row tiles only 100)
        int best = 0;
        double best_fill = 0.0;
        for (int cand : {5, 4, 2, 1}) {
            const int su = 32 * cand / unit;
            if (su < 1) continue;
            const long gm = (units + su - 1) / su;
            if (gm * a.gn < 480) continue;
            const double fill = (double)(su * unit) / (32 * cand);
            if (fill > best_fill + 1e-9) {
                best_fill = fill;
                best = cand;
            }
        }
        if (best != 0) {
            a.S_t = 32 * best / unit;
            a.gm = (units + a.S_t - 1) / a.S_t;
            return best;
        }
    }
    int wr = 0;
    for (int cand = 4; cand >= 1; cand >>= 1) {
        const int su = 32 * cand / unit;
        if (su < 1) break;
        wr = cand;
        a.S_t = su;
        a.gm = (units + su - 1) / su;
        if ((long)a.gm * a.gn >= 480) break;   // ~2 workgroups per CU: balance + latency hiding
    }
    return wr;
}

// Split-K linears (the decoder's, HYPER_EPI_BIAS): the largest row tile whose grid, times the
// K splits that the deep K then allows, still gives ~two workgroups per CU. Big tiles cut the
// operand re-reads (x is read once per column tile, W once per row tile: configs[4]'s
// 1024 x 20000 x 400 decoder input moved 1.6 GB at 32-row tiles).
static int split_k(long tiles, int K) {
    int s = 1;
    // split K while the grid is under ~8 workgroups per CU and every split keeps >= 16 k-steps
    while (tiles * s * 2 <= 2048 && K / 16 / (s * 2) >= 16 && s < 32) s *= 2;
    return s;
}
static int pick_split_tiles(HyperArgs& a, int K, int& splits) {
    a.gn = (a.N + hyper::TN - 1) / hyper::TN;
    int wr = 0;
    for (int cand = 4; cand >= 1; cand >>= 1) {
        wr = cand;
        a.S_t = 32 * cand;
        a.gm = (a.rows + a.S_t - 1) / a.S_t;
        splits = split_k((long)a.gm * a.gn, K);
        if ((long)a.gm * a.gn * splits >= 480) break;
    }
    return wr;
}

// the 32x32x2 GCN kernel (gcn32_kernel) for inference GCN layers on an unsplit input whose grid
// of 256-row tiles still covers the CUs; DADMM_GCN32=0 in the environment selects linear_kernel
// (A/B timing)
static bool try_gcn32(HyperArgs& a, hipStream_t st, hipError_t& err) {
    static int enabled = -1;
    if (enabled < 0) {
        const char* e = getenv("DADMM_GCN32");
        enabled = (e != nullptr && e[0] == '0') ? 0 : 1;
    }
    // (small P: linear_kernel's 160-row tiles hold 32 whole samples with little padding and the mix
    // is short; at P = 5, B = 4096 gcn32 measured 14.2-14.3 vs 13.9 ms, profiles/r04/variants_r04v_p5.txt)
    if (!enabled || a.K1 < a.K || a.P < 32 || a.P > hyper::G32_TM) return false;
    const int S_t = hyper::G32_TM / a.P;
    const long gm = (a.B + S_t - 1) / S_t, gn = (a.N + hyper::TN - 1) / hyper::TN;
    if (gm * gn < 256) return false;
    const size_t lds = hyper::g32_lds_bytes(S_t, a.P);
    if (lds > 160 * 1024) return false;
    a.S_t = S_t;
    a.gm = (int)gm;
    a.gn = (int)gn;
    err = hipFuncSetAttribute((const void*)hyper::gcn32_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (err == hipSuccess) {
        hipLaunchKernelGGL(hyper::gcn32_kernel, dim3((unsigned)(gm * gn)), dim3(64 * hyper::G32_WAVES), lds, st, a);
        err = hipGetLastError();
    }
    return true;
}

// The K split over two wave sets of a workgroup (linear_kernel KS = 2): where the grid of 32-row
// tiles leaves the CUs idle (< ~2 workgroups per CU) and the register ring runs the whole K loop,
// each wave's dependent chain halves. Decided from the GEMM shape (rows, K, N) and the GCN P alone,
// so that a GCN layer's input-gradient GEMM gives the same bits fused with the block backward or
// alone. a.kwave: 0 = never (the decoder's linears), else the P whose whole-sample tiles pair
// with this GEMM (the split needs 32-row tiles of whole samples: P <= 32).
// DADMM_HYPER_KW=0 in the environment: never (A/B timing).
constexpr int HYPER_KW_MIN = 8;    // k-steps (16 k each) from which the K loop is split
static bool hyper_kwave(const HyperArgs& a, int epi, int rows) {
    static int enabled = -1;
    if (enabled < 0) {
        const char* e = getenv("DADMM_HYPER_KW");
        enabled = (e != nullptr && e[0] == '0') ? 0 : 1;
    }
    if (!enabled || a.kwave < 1 || a.kwave > 32 || a.splits > 1) return false;
    // (the inference GCN layer and the training forward's 200-deep one measured slower split: its
    // epilogue is shorter than the chain it would overlap; profiles/r05/kwave_r05kw.txt)
    if (epi == HYPER_EPI_GCN || (epi == HYPER_EPI_GCN_TRAIN && a.K < 256)) return false;
    const int steps = a.K / 16;
    if (steps < HYPER_KW_MIN || hyper::use_dma(a.K, 1)) return false;
    const long tiles = (long)((rows + 31) / 32) * ((a.N + hyper::TN - 1) / hyper::TN);
    return tiles < 480;
}

hipError_t launch_hyper(HyperArgs a, int epi, hipStream_t st) {
    const bool gcn = epi == HYPER_EPI_GCN || epi == HYPER_EPI_GCN_TRAIN || epi == HYPER_EPI_GCN_BWD;
    const int units = gcn ? a.B : a.rows;
    if (units <= 0 || a.N <= 0) return hipSuccess;
    if (a.K1 < a.K && (a.K1 & 15)) return hipErrorInvalidValue;
    hipError_t gerr = hipSuccess;
    if (epi == HYPER_EPI_GCN && try_gcn32(a, st, gerr)) return gerr;
    int wr = 0, ks = 1;
    if (hyper_kwave(a, epi, gcn ? a.B * a.P : a.rows)) {   // 32-row tiles (whole samples), K split in two
        ks = 2;
        wr = 1;
        a.gn = (a.N + hyper::TN - 1) / hyper::TN;
        a.S_t = gcn ? 32 / a.P : 32;
        a.gm = (units + a.S_t - 1) / a.S_t;
    } else if (epi == HYPER_EPI_BIAS && a.splits > 1) {
        int sp = 0;
        wr = pick_split_tiles(a, a.K, sp);
        if (sp != a.splits) wr = pick_tiles(a, epi);   // caller's own split count: plain tiling
    } else {
        wr = pick_tiles(a, epi);
    }
    if (wr == 0) return hipErrorInvalidValue;
    if (a.splits < 1) a.splits = 1;
    const int grid = a.gm * a.gn * a.splits;
    switch (epi) {
        case HYPER_EPI_BIAS: return hyper::launch_epi<HYPER_EPI_BIAS>(wr, ks, grid, a, st);
        case HYPER_EPI_GCN: return hyper::launch_epi<HYPER_EPI_GCN>(wr, ks, grid, a, st);
        case HYPER_EPI_HEAD: return hyper::launch_epi<HYPER_EPI_HEAD>(wr, ks, grid, a, st);
        case HYPER_EPI_GCN_TRAIN: return hyper::launch_epi<HYPER_EPI_GCN_TRAIN>(wr, ks, grid, a, st);
        case HYPER_EPI_GCN_BWD: return hyper::launch_epi<HYPER_EPI_GCN_BWD>(wr, ks, grid, a, st);
        default: return hipErrorInvalidValue;
    }
}

int hyper_linear_splits(int rows, int K, int N) {
    HyperArgs a{};
    a.rows = rows;
    a.N = N;
    if (rows <= 0 || N <= 0) return 1;
    int s = 1;
    pick_split_tiles(a, K, s);
    return s;
}

hipError_t launch_rownorm(const RowNormArgs& a, hipStream_t st) {
    if (a.rows <= 0) return hipSuccess;
    const int per = hyper::THREADS / 64;
    const dim3 grid((a.rows + per - 1) / per), block(hyper::THREADS);
    if (a.C <= 256)
        hipLaunchKernelGGL(hyper::rownorm_kernel<1>, grid, block, 0, st, a);
    else if (a.C <= 512)
        hipLaunchKernelGGL(hyper::rownorm_kernel<2>, grid, block, 0, st, a);
    else if (a.C <= 1024)
        hipLaunchKernelGGL(hyper::rownorm_kernel<4>, grid, block, 0, st, a);
    else
        hipLaunchKernelGGL(hyper::rownorm_kernel<8>, grid, block, 0, st, a);
    return hipGetLastError();
}

}  // namespace dadmm
