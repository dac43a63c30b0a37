// dadmm_internal.h — shared between the kernel translation units and the C-ABI layer.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dadmm {

constexpr int BT = 16;       // samples per workgroup of the fused kernel (MFMA N dimension)
constexpr int M_PAD = 64;    // padded rows per agent (4 m-blocks of 16 rows)
#ifndef DADMM_FUSED_WAVES
#define DADMM_FUSED_WAVES 8
#endif
constexpr int FUSED_WAVES = DADMM_FUSED_WAVES;  // waves per workgroup of the fused kernel

// Arguments of the fused kernel (device pointers; see include/dadmm.h for the layouts).
struct FusedArgs {
    const float* A;      // prepared operator: [P][M_PAD][n_pad]
    const float* At;     // prepared operator: [P][n_pad][M_PAD]
    const float* b;      // [B][P][m]
    const uint64_t* nbr; // [B][P] (or [P] for GRAPH_SHARED)
    const uint32_t* nbr_order;  // [B][P] packed adjacency order (GRAPH_ORDERED) or nullptr
    const float* deg;    // [B][P]
    const float* hyp;    // [K][hyp_rows][4]
    const float* y0;     // [B][P][n]
    const float* U0;
    const float* d0;
    float* Y;            // [K][B][P][n]
    float* U_out;        // [B][P][n] or nullptr
    int32_t* status;     // or nullptr
    int B, m, n, K, hyp_rows, variant;
};

typedef hipError_t (*fused_fn_ptr)(const FusedArgs&, hipStream_t);

// Returns the launcher for (P, n_pad = 64*nt) or nullptr when that shape is not instantiated.
enum { GRAPH_SHARED = 0, GRAPH_LANE = 1, GRAPH_ORDERED = 2 };
fused_fn_ptr find_fused(int P, int nt, int graph);

// Operator preparation kernel launcher (dadmm_prepare.hip).
hipError_t launch_prepare(const float* A, float* Apad, float* Atpad, int P, int m, int n,
                          int n_pad, hipStream_t stream);

inline int fused_nt(int n) {
    const int nt = (n + 63) / 64;
    return nt <= 1 ? 1 : (nt <= 2 ? 2 : (nt <= 4 ? 4 : nt));
}

}  // namespace dadmm
