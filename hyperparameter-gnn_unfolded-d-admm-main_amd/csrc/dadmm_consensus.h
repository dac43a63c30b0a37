// dadmm_consensus.h — delta = compute_delta(y) = 2 (D - Adj) y, lane-local over the P agents of one
// sample, in the reference's accumulation order (unfolded_DLASSO.py:127-140). Shared by the fused
// forward and the fused adjoint (which must reproduce the forward's delta bit-for-bit to recover
// its clamp masks, and applies the same linear map to the adjoint: (2 (D - Adj))^T = 2 (D - Adj)).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dadmm_internal.h"

namespace dadmm {

// delta_p = 2 (L y)_p accumulated exactly as compute_delta (unfolded_DLASSO.py:127-140) does for
// one sample: the agents' loops run p' = 0..P-1 over graph.neighbors(p') in ascending order,
// each visit (p', q) doing delta[p'] += (y_p' - y_q); delta[q] -= (y_p' - y_q). Restricted to the
// updates of delta[p], in order: every q < p with p in N(q) (-=), then p's own neighbours
// (+=, a self-loop also takes its -= there), then every q > p with p in N(q) (-=).
// Every such update of delta[p] adds +-fl(y_a - y_b) for the pair's ordered difference
// d(a, b) = fl(y_a - y_b), a < b, and fl(y_b - y_a) == -d(a, b) exactly (round-to-nearest is
// symmetric), so acc - fl(y_q - y_p) == acc + fl(y_p - y_q): one subtraction per pair serves all
// four updates an undirected edge makes, bit-for-bit.
// `bit(q, p)` = p in N(q); E positions (rows) at a time.
template <int P, int E, typename BitFn>
__device__ __forceinline__ void consensus(const float (&yy)[P][E], float (&dl)[P][E], BitFn bit) {
    float acc[P][E];
#pragma unroll
    for (int p = 0; p < P; ++p)
#pragma unroll
        for (int e = 0; e < E; ++e) acc[p][e] = 0.0f;
    // contribution of pair (a, b) to agent p, as the reference's sequence for p orders it:
    //   q < p  (other's loop):  acc -= (y_q - y_p)  ==  acc - d(q, p)
    //   own loop, q < p:        acc += (y_p - y_q)  ==  acc - d(q, p)
    //   own loop, q > p:        acc += (y_p - y_q)  ==  acc + d(p, q)
    //   q > p  (other's loop):  acc -= (y_q - y_p)  ==  acc + d(p, q)
#pragma unroll
    for (int p = 0; p < P; ++p) {
#pragma unroll
        for (int q = 0; q < p; ++q)
            if (bit(q, p)) {
#pragma unroll
                for (int e = 0; e < E; ++e) acc[p][e] = acc[p][e] - (yy[q][e] - yy[p][e]);
            }
#pragma unroll
        for (int q = 0; q < P; ++q)
            if (bit(p, q)) {
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    if (q < p) acc[p][e] = acc[p][e] - (yy[q][e] - yy[p][e]);
                    else if (q > p) acc[p][e] = acc[p][e] + (yy[p][e] - yy[q][e]);
                    else acc[p][e] = (acc[p][e] + (yy[p][e] - yy[p][e])) - (yy[p][e] - yy[p][e]);
                }
            }
#pragma unroll
        for (int q = p + 1; q < P; ++q)
            if (bit(q, p)) {
#pragma unroll
                for (int e = 0; e < E; ++e) acc[p][e] = acc[p][e] + (yy[p][e] - yy[q][e]);
            }
    }
#pragma unroll
    for (int p = 0; p < P; ++p)
#pragma unroll
        for (int e = 0; e < E; ++e) dl[p][e] = acc[p][e];
}

// The shared-graph form without branches or selects, for a symmetric adjacency (an undirected
// graph: p in N(q) <=> q in N(p)): mf[a][b] (a < b) = 1.0f for an edge, else 0.0f, a uniform
// value held in an SGPR. Every update of delta[p] is acc + fl(y_p - y_q) (see above), written as
// fma(d, mf, acc): with mf = 1 that is exactly fl(acc + d); with mf = 0 it is acc + (+-0) = acc,
// because acc starts at +0 and a round-to-nearest sum is -0 only when both addends are -0, so acc
// is never -0. A self-loop's pair of updates, (acc + 0) - 0, leaves acc unchanged and is skipped.
// One subtraction per unordered pair, one v_fma_f32 per candidate visit, for finite y (a
// non-finite y is flagged before it can reach here).
__device__ __forceinline__ float fma_s(float d, float m, float acc) {   // d * m + acc, m in an SGPR
    float r;
    asm("v_fma_f32 %0, %1, %2, %3" : "=v"(r) : "v"(d), "s"(m), "v"(acc));
    return r;
}
__device__ __forceinline__ float fma_sn(float d, float m, float acc) {  // -d * m + acc
    float r;
    asm("v_fma_f32 %0, -%1, %2, %3" : "=v"(r) : "v"(d), "s"(m), "v"(acc));
    return r;
}
template <int P>
__device__ __forceinline__ void consensus_fma(const float (&yy)[P][1], float (&dl)[P][1],
                                              const float (&mf)[P][P]) {
    float d[P][P];   // d[a][b] = fl(y_a - y_b) for a < b
#pragma unroll
    for (int a2 = 0; a2 < P; ++a2)
#pragma unroll
        for (int b2 = a2 + 1; b2 < P; ++b2) d[a2][b2] = yy[a2][0] - yy[b2][0];
#pragma unroll
    for (int p = 0; p < P; ++p) {
        float acc = 0.0f;
        // the sequence of delta[p]: q < p (q's loop), then p's own loop (ascending), then q > p
        // (q's loop); d(p, q) = fl(y_p - y_q) = -d[q][p] for q < p (exact negation)
#pragma unroll
        for (int q = 0; q < p; ++q) acc = fma_sn(d[q][p], mf[q][p], acc);
#pragma unroll
        for (int q = 0; q < P; ++q) {
            if (q < p) acc = fma_sn(d[q][p], mf[q][p], acc);
            else if (q > p) acc = fma_s(d[p][q], mf[p][q], acc);
        }
#pragma unroll
        for (int q = p + 1; q < P; ++q) acc = fma_s(d[p][q], mf[p][q], acc);
        dl[p][0] = acc;
    }
}

// consensus_fma on two rows at once (v_pk_add_f32 / v_pk_fma_f32: each half rounded exactly as the
// scalar instruction, so the result is consensus_fma's bit for bit, at half the VALU issue). The
// multipliers mf2[a][b] = {mf, mf} are uniform (an SGPR pair per candidate pair).
typedef float f32x2_c __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2_c pk_sub_c(f32x2_c a, f32x2_c b) {   // a - b == a + (-b) exactly
    f32x2_c r;
    asm("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ f32x2_c pk_fma_s(f32x2_c d, f32x2_c m, f32x2_c acc) {    // d m + acc
    f32x2_c r;
    asm("v_pk_fma_f32 %0, %1, %2, %3" : "=v"(r) : "v"(d), "s"(m), "v"(acc));
    return r;
}
__device__ __forceinline__ f32x2_c pk_fma_sn(f32x2_c d, f32x2_c m, f32x2_c acc) {   // -d m + acc
    f32x2_c r;
    asm("v_pk_fma_f32 %0, %1, %2, %3 neg_lo:[1,0,0] neg_hi:[1,0,0]" : "=v"(r) : "v"(d), "s"(m), "v"(acc));
    return r;
}
template <int P>
__device__ __forceinline__ void consensus_fma2(const f32x2_c (&yy)[P], f32x2_c (&dl)[P],
                                               const f32x2_c (&mf)[P][P]) {
    f32x2_c d[P][P];
#pragma unroll
    for (int a2 = 0; a2 < P; ++a2)
#pragma unroll
        for (int b2 = a2 + 1; b2 < P; ++b2) d[a2][b2] = pk_sub_c(yy[a2], yy[b2]);
#pragma unroll
    for (int p = 0; p < P; ++p) {
        f32x2_c acc = {0.0f, 0.0f};
#pragma unroll
        for (int q = 0; q < p; ++q) acc = pk_fma_sn(d[q][p], mf[q][p], acc);
#pragma unroll
        for (int q = 0; q < P; ++q) {
            if (q < p) acc = pk_fma_sn(d[q][p], mf[q][p], acc);
            else if (q > p) acc = pk_fma_s(d[p][q], mf[p][q], acc);
        }
#pragma unroll
        for (int q = p + 1; q < P; ++q) acc = pk_fma_s(d[p][q], mf[p][q], acc);
        dl[p] = acc;
    }
}

// Per-lane (per-sample graph) form: the conditional adds become selects; pair differences are
// shared as above (the compiler CSEs yy[a] - yy[b] across the four uses).
template <int P, int E>
__device__ __forceinline__ void consensus_lane(const float (&yy)[P][E], float (&dl)[P][E],
                                               const uint32_t (&msk)[P]) {
    float d[P][P][E];   // d[a][b] = y_a - y_b for a < b
#pragma unroll
    for (int a = 0; a < P; ++a)
#pragma unroll
        for (int b2 = a + 1; b2 < P; ++b2)
#pragma unroll
            for (int e = 0; e < E; ++e) d[a][b2][e] = yy[a][e] - yy[b2][e];
#pragma unroll
    for (int p = 0; p < P; ++p) {
        float acc[E];
#pragma unroll
        for (int e = 0; e < E; ++e) acc[e] = 0.0f;
#pragma unroll
        for (int q = 0; q < p; ++q) {
            const bool on = (msk[q] >> p) & 1u;
#pragma unroll
            for (int e = 0; e < E; ++e) acc[e] = on ? acc[e] - d[q][p][e] : acc[e];
        }
#pragma unroll
        for (int q = 0; q < P; ++q) {
            const bool on = (msk[p] >> q) & 1u;
#pragma unroll
            for (int e = 0; e < E; ++e) {
                float t;
                if (q < p) t = acc[e] - d[q][p][e];
                else if (q > p) t = acc[e] + d[p][q][e];
                else t = (acc[e] + (yy[p][e] - yy[p][e])) - (yy[p][e] - yy[p][e]);
                acc[e] = on ? t : acc[e];
            }
        }
#pragma unroll
        for (int q = p + 1; q < P; ++q) {
            const bool on = (msk[q] >> p) & 1u;
#pragma unroll
            for (int e = 0; e < E; ++e) acc[e] = on ? acc[e] + d[p][q][e] : acc[e];
        }
#pragma unroll
        for (int e = 0; e < E; ++e) dl[p][e] = acc[e];
    }
}

// Per-lane graphs whose adjacency lists are not ascending: p's own loop follows the packed
// adjacency order ord[p] (4 bits per neighbour, cnt[p] entries) exactly as graph.neighbors(p).
template <int P, int E>
__device__ __forceinline__ void consensus_ordered(const float (&yy)[P][E], float (&dl)[P][E],
                                                  const uint32_t (&msk)[P],
                                                  const uint32_t (&ord)[P]) {
#pragma unroll
    for (int p = 0; p < P; ++p) {
        float acc[E];
#pragma unroll
        for (int e = 0; e < E; ++e) acc[e] = 0.0f;
#pragma unroll
        for (int q = 0; q < p; ++q) {
            const bool on = (msk[q] >> p) & 1u;
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const float t = acc[e] - (yy[q][e] - yy[p][e]);
                acc[e] = on ? t : acc[e];
            }
        }
        const int cnt = __builtin_popcount(msk[p]);
#pragma unroll
        for (int t = 0; t < P; ++t) {
            const bool on = t < cnt;
            const int q = (ord[p] >> (4 * t)) & 15;
#pragma unroll
            for (int e = 0; e < E; ++e) {
                float yq = yy[0][e];
#pragma unroll
                for (int qq = 1; qq < P; ++qq) yq = (q == qq) ? yy[qq][e] : yq;
                float v = acc[e] + (yy[p][e] - yq);
                if (q == p) v = v - (yy[p][e] - yy[p][e]);
                acc[e] = on ? v : acc[e];
            }
        }
#pragma unroll
        for (int q = p + 1; q < P; ++q) {
            const bool on = (msk[q] >> p) & 1u;
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const float t = acc[e] - (yy[q][e] - yy[p][e]);
                acc[e] = on ? t : acc[e];
            }
        }
#pragma unroll
        for (int e = 0; e < E; ++e) dl[p][e] = acc[e];
    }
}

template <int P, int GRAPH>
__device__ __forceinline__ void consensus_any(const float (&yy)[P][4], float (&dl)[P][4],
                                              const uint32_t (&msk)[P], const uint32_t (&ord)[P]) {
    if constexpr (GRAPH == GRAPH_SHARED)
        consensus<P, 4>(yy, dl, [&](int q, int p) { return ((msk[q] >> p) & 1u) != 0; });
    else if constexpr (GRAPH == GRAPH_LANE)
        consensus_lane<P, 4>(yy, dl, msk);
    else
        consensus_ordered<P, 4>(yy, dl, msk, ord);
}

}  // namespace dadmm
