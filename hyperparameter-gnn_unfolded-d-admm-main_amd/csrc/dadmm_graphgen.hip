// dadmm_graphgen.hip — per-sample Erdos-Renyi agent graphs generated on the device, straight into
// the layouts the kernels read (include/dadmm.h: neighbour masks, degrees, packed adjacency
// order, compute_delta visit lists).
//
// Replaces the host loop of the progressive driver (gnn_dlasso_progressive.py:181-191):
//     graph = nx.erdos_renyi_graph(P, prob)
//     if not nx.is_connected(graph):
//         components = list(nx.connected_components(graph))
//         for i in range(len(components) - 1):
//             graph.add_edge(list(components[i])[0], list(components[i + 1])[0])
// followed by ingestion (dadmm_hip/graph.py), which at configs[4] (P = 50, 1024 graphs per GPU)
// costs about as much as the forward itself.
//
// Graph model, per sample s: every pair u < v is an edge with probability `prob`, decided by a
// counter-based hash of (seed, s, u, v) — reproducible for any grid and restated in numpy by the
// tests — NOT networkx's Python RNG stream (the reference seeds nothing: its graphs are a
// distribution, not a sequence). Adjacency lists are in networkx's insertion order: the ER edges
// ascending, then the connectivity edges in the order they are added. Components are taken in
// networkx's order (by smallest node) and represented by their smallest node; networkx takes the
// first element of a Python set, which for these small-integer sets is usually, not always, the
// smallest — a difference in which edge joins two components, not in the graph distribution.
//
// One thread per sample (P <= 64: the adjacency is P 64-bit masks). Pass 0 writes masks,
// degrees, order nibbles and the per-sample visit-entry count; a single-workgroup scan turns
// the counts into offsets; pass 1 writes vptr and (when vq is given) the visit lists.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dadmm_internal.h"

namespace dadmm {
namespace gg {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// uniform in [0, 1) with 24 bits for pair (u, v), u < v, of sample s
__device__ __forceinline__ float pair_uniform(uint64_t seed, int s, int u, int v) {
    const uint64_t h = splitmix64(seed ^ splitmix64(((uint64_t)s << 12) | ((uint64_t)u << 6) | (uint64_t)v));
    return (float)(h >> 40) * (1.0f / 16777216.0f);
}

struct Sample {
    uint64_t er[64];          // ER neighbours of each node (ascending by construction)
    uint64_t all[64];         // ER + connectivity edges
    int8_t pa[64], pb[64];    // connectivity edges in insertion order
    int npatch;
};

__device__ void build(const GraphGenArgs& a, int s, Sample& g) {
    const int P = a.P;
    for (int p = 0; p < P; ++p) g.er[p] = 0;
    for (int u = 0; u < P; ++u)
        for (int v = u + 1; v < P; ++v)
            if (pair_uniform(a.seed, s, u, v) < a.prob) {
                g.er[u] |= 1ull << v;
                g.er[v] |= 1ull << u;
            }
    for (int p = 0; p < P; ++p) g.all[p] = g.er[p];
    g.npatch = 0;
    if (!a.connect) return;
    const uint64_t full = P == 64 ? ~0ull : ((1ull << P) - 1);
    uint64_t left = full;
    int prev = -1;
    while (left) {
        const int start = __builtin_ctzll(left);
        uint64_t comp = 1ull << start, frontier = comp;
        while (frontier) {                         // BFS over bitmasks
            uint64_t nxt = 0;
            for (uint64_t f = frontier; f; f &= f - 1) nxt |= g.er[__builtin_ctzll(f)];
            frontier = nxt & ~comp;
            comp |= nxt;
        }
        left &= ~comp;
        if (prev >= 0) {                           // join component i-1 to component i
            g.pa[g.npatch] = (int8_t)prev;
            g.pb[g.npatch] = (int8_t)start;
            ++g.npatch;
            g.all[prev] |= 1ull << start;
            g.all[start] |= 1ull << prev;
        }
        prev = start;
    }
}

// p's neighbours in adjacency (insertion) order: ER ones ascending, then its connectivity edges
template <typename F>
__device__ __forceinline__ void for_adjacency(const Sample& g, int p, F f) {
    for (uint64_t m = g.er[p]; m; m &= m - 1) f(__builtin_ctzll(m));
    for (int i = 0; i < g.npatch; ++i) {
        if (g.pa[i] == p) f(g.pb[i]);
        else if (g.pb[i] == p) f(g.pa[i]);
    }
}

__global__ __launch_bounds__(64) void gen_kernel(GraphGenArgs a, int pass) {
    const int s = blockIdx.x * 64 + threadIdx.x;
    if (s >= a.B) return;
    const int P = a.P;
    Sample g;
    build(a, s, g);
    if (pass == 0) {
        int cnt = 0;
        for (int p = 0; p < P; ++p) {
            const int d = __builtin_popcountll(g.all[p]);
            a.nbr[(size_t)s * P + p] = (int64_t)g.all[p];
            a.deg[(size_t)s * P + p] = (float)d;
            cnt += 2 * d;                          // each incident edge visited from both ends
            if (a.order != nullptr) {
                uint32_t o = 0;
                int t = 0;
                for_adjacency(g, p, [&](int q) {
                    if (t < 8) o |= (uint32_t)(q & 15) << (4 * t);
                    ++t;
                });
                a.order[(size_t)s * P + p] = (int32_t)o;
            }
        }
        a.counts[s] = cnt;
        return;
    }
    // pass 1: vptr from the scanned sample offsets, and the visit lists (graph.py _visit_lists):
    // N(p) below p ascending | N(p) in adjacency order | N(p) above p ascending
    int off = a.counts[s];
    for (int p = 0; p < P; ++p) {
        a.vptr[(size_t)s * P + p] = off;
        const uint64_t nb = g.all[p];
        const uint64_t below = nb & ((1ull << p) - 1), above = p == 63 ? 0 : nb & ~((2ull << p) - 1);
        if (a.vq != nullptr) {
            int o = off;
            for (uint64_t m = below; m; m &= m - 1) a.vq[o++] = (uint8_t)__builtin_ctzll(m);
            for_adjacency(g, p, [&](int q) { a.vq[o++] = (uint8_t)q; });
            for (uint64_t m = above; m; m &= m - 1) a.vq[o++] = (uint8_t)__builtin_ctzll(m);
        }
        off += 2 * __builtin_popcountll(nb);
    }
    if (s == a.B - 1) a.vptr[(size_t)a.B * P] = off;
}

// exclusive scan of counts[0..B) in place (one workgroup; B up to a few 100k)
__global__ __launch_bounds__(1024) void scan_kernel(int32_t* counts, int B) {
    __shared__ int32_t part[1024];
    const int t = threadIdx.x;
    const int chunk = (B + 1023) / 1024;
    const int lo = t * chunk, hi = lo + chunk < B ? lo + chunk : B;
    int sum = 0;
    for (int i = lo; i < hi; ++i) sum += counts[i];
    part[t] = sum;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {           // Hillis-Steele over the 1024 partials
        const int v = t >= d ? part[t - d] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    int run = t > 0 ? part[t - 1] : 0;
    for (int i = lo; i < hi; ++i) {
        const int c = counts[i];
        counts[i] = run;
        run += c;
    }
}

}  // namespace gg

hipError_t launch_graphgen(const GraphGenArgs& a, int pass, hipStream_t st) {
    const int grid = (a.B + 63) / 64;
    if (pass == 0) {
        hipLaunchKernelGGL(gg::gen_kernel, dim3(grid), dim3(64), 0, st, a, 0);
        hipLaunchKernelGGL(gg::scan_kernel, dim3(1), dim3(1024), 0, st, a.counts, a.B);
    }
    hipLaunchKernelGGL(gg::gen_kernel, dim3(grid), dim3(64), 0, st, a, 1);
    return hipGetLastError();
}

}  // namespace dadmm
