// dadmm_internal.h — shared between the kernel translation units and the C-ABI layer.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dadmm {

// Sum of v over the wave's 64 lanes, in a fixed order, on DPP moves (quad perms, half-row and row
// mirrors: every lane ends with its 16-lane row's sum) and four readlanes: no LDS round trips (a
// __shfl_xor butterfly is six ds_bpermute round trips). Deterministic; the association differs
// from the butterfly's (f32 rounding). Uniform result.
template <int CTRL>
__device__ __forceinline__ float dpp_mov_f32(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float wave_sum_dpp(float v) {
    v = v + dpp_mov_f32<0xB1>(v);    // quad_perm [1,0,3,2]
    v = v + dpp_mov_f32<0x4E>(v);    // quad_perm [2,3,0,1]: every lane holds its quad's sum
    v = v + dpp_mov_f32<0x141>(v);   // row_half_mirror: its 8-lane group's
    v = v + dpp_mov_f32<0x140>(v);   // row_mirror: its 16-lane row's
    const auto lane_v = [&](int l) {
        return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
    };
    return (lane_v(0) + lane_v(16)) + (lane_v(32) + lane_v(48));
}
// Sum of v over each 16-lane row, in every lane of the row (the first four steps above).
__device__ __forceinline__ float row16_sum_dpp(float v) {
    v = v + dpp_mov_f32<0xB1>(v);
    v = v + dpp_mov_f32<0x4E>(v);
    v = v + dpp_mov_f32<0x141>(v);
    return v + dpp_mov_f32<0x140>(v);
}

// The LayerNorm row sums (rownorm forward / backward and the hypernetwork tail kernel's copies of
// them, which must reduce identically): wave_sum_dpp.
__device__ __forceinline__ float ln_row_sum(float v) {
    return wave_sum_dpp(v);
}


// sign(y) * t exactly as torch's eager ops give it (sign(+-0) = sign(NaN) = 0, so +0 there, else
// +-t), without branches: the sign bit of y moved onto t, then one select. (The nested-ternary
// form compiles to divergent branches, ~11 instructions per element in the middle of the MFMA
// chains.)
__device__ __forceinline__ float sign_times(float y, float t) {
    const float st = __uint_as_float(__float_as_uint(t) ^ (__float_as_uint(y) & 0x80000000u));
    return __builtin_fabsf(y) > 0.0f ? st : 0.0f;
}

constexpr int BT = 16;       // samples per workgroup of the fused kernel (MFMA N dimension)
constexpr int M_PAD = 64;    // rows per m-group (4 m-blocks of 16 rows); the fused kernels hold one
constexpr int M_MAX = 1024;  // rows per agent accepted by the ABI (the stepwise path: any m-group count)
// padded rows per agent of the prepared operator: whole m-groups of 64 rows
__host__ __device__ constexpr int m_pad_of(int m) { return (m + M_PAD - 1) / M_PAD * M_PAD; }
constexpr int FUSED_WAVES = 8;  // waves per workgroup of the fused kernel

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
    float* Grec;         // [K][B][P][n] pre-clamp gradients (recording launchers only)
    float* Urec;         // [K][B][P][n] U_k entering iteration k (recording launchers only)
    int B, m, n, K, hyp_rows, variant;
};

typedef hipError_t (*fused_fn_ptr)(const FusedArgs&, hipStream_t);

// Returns the launcher for (P, n_pad = 64*nt) or nullptr when that shape is not instantiated.
enum { GRAPH_SHARED = 0, GRAPH_LANE = 1, GRAPH_ORDERED = 2 };
fused_fn_ptr find_fused(int P, int nt, int graph);
// Same shapes, recording the adjoint's trajectory (a.Grec / a.Urec must be set).
fused_fn_ptr find_fused_rec(int P, int nt, int graph);

// ---- the column-split forward for small batches (dadmm_split.hip) ------------------------------
constexpr int SPLIT_COLS = 64;   // columns of n_pad per slice (one workgroup each)
struct SplitArgs {
    FusedArgs f;         // as the fused kernel (U_out / status optional; no recording)
    float* xbuf;         // [groups][2][P][4][S][256] GEMM1 partial tiles (no initialisation)
    uint32_t* xflag;     // [groups][P][4][S] epoch words + 1 abort word: ZEROED before every launch
    int groups;          // workgroup groups (S blocks each); grid = groups * S <= CUs
    int tiles;           // ceil(B / BT) 16-sample tiles, walked g, g + groups, ...
    uint64_t spin_ticks; // bound on one wait (s_memrealtime ticks, 100 MHz) before the abort
};
typedef hipError_t (*split_fn_ptr)(const SplitArgs&, hipStream_t);
// P = 1..6, n_pad = 64 * nt with nt in {2, 4}; nullptr otherwise
split_fn_ptr find_split(int P, int nt, int graph);

// ---- adjoint (dadmm_backward.hip) ---------------------------------------------------------------
struct BackwardArgs {
    const float* A;      // prepared operator [P][M_PAD][n_pad]
    const float* At;     // [P][n_pad][M_PAD]
    const uint64_t* nbr; // as FusedArgs
    const uint32_t* nbr_order;
    const float* deg;
    const float* hyp;    // [K][hyp_rows][4]
    const float* y0;     // [B][P][n]
    const float* d0;     // [B][P][n]
    const float* Y;      // [K][B][P][n] recorded trajectory
    const float* Grec;   // [K][B][P][n]
    const float* Urec;   // [K][B][P][n]
    const float* gY;     // [K][B][P][n] dL/dY
    float* partial;      // [ceil(B/BT)][K][P][4] per-workgroup sums
    int B, m, n, K, hyp_rows, variant;
};
typedef hipError_t (*backward_fn_ptr)(const BackwardArgs&, hipStream_t);
backward_fn_ptr find_backward(int P, int nt, int graph);
hipError_t launch_backward_reduce(const float* partial, float* dhyp, int nwg, int K, int P, int H,
                                  hipStream_t stream);

// ---- adjoint for every shape (dadmm_adjoint.hip) ------------------------------------------------
struct AdjArgs {
    const float* A;         // prepared operator [P][m_pad][n_pad]
    const float* At;        // [P][n_pad][m_pad]
    const int32_t* vptr;    // visit lists (as StepArgs)
    const uint8_t* vq;
    const float* deg;       // [G][P]
    const float* hyp;       // [K][hyp_rows][4]
    const float* y0;        // [B][P][n]
    const float* d0;        // [B][P][n]
    const float* Y;         // [K][B][P][n] recorded trajectory
    const float* Grec;      // [K][B][P][n]
    const float* Urec;      // [K][B][P][n]
    const float* gY;        // [K][B][P][n] dL/dY
    float* yb;              // scratch [B][P][n]: dL/dy
    float* Ub;              // scratch [B][P][n]: dL/dU
    float* Gb;              // scratch [B][P][n]: dL/d(pre-clamp gradient) of the later iteration
    float* partial;         // scratch [adjoint_workgroups(B, n, P)][K][P][4]
    int B, P, m, m_pad, n, n_pad, K, hyp_rows, variant, graph_shared;
};
size_t adjoint_lds_bytes(int P);
int adjoint_workgroups(int B, int n, int P);
int adjoint_waves(int P);
hipError_t launch_adjoint(const AdjArgs& a, float* dhyp, hipStream_t st);

// ---- GNN-model per-iteration path (dadmm_gnn.hip) -----------------------------------------------
// flag words (int32, zeroed by dadmm_gnn_begin): y0 guard, then U_k non-finite (k = 0..K),
// gradient NaN and y_next non-finite (k = 0..K-1), and the fused step's optimistic y_next /
// U_{k+1} flags (committed by its resolve launch when no gradient was NaN)
#define GNN_F_Y0 0
#define GNN_F_UBAD(k) (1 + 5 * (k))
#define GNN_F_GBAD(k) (2 + 5 * (k))
#define GNN_F_YNB(k) (3 + 5 * (k))
#define GNN_F_YNB_OPT(k) (4 + 5 * (k))
#define GNN_F_UNB_OPT(k) (5 + 5 * (k))
#define GNN_FLAG_WORDS(K) (5 * (K) + 4)

struct GnnArgs {
    const float* A;         // prepared operator [P][m_pad][n_pad]
    const float* At;        // [P][n_pad][m_pad]
    const float* b;         // [B][P][m]
    const int32_t* vptr;    // visit lists (as StepArgs)
    const uint8_t* vq;
    const float* deg;       // [G][P]
    const float* hyp;       // [B][4][hyp_rows] of the current iteration
    float* const* yptr;     // device table [K+1]: y0, y_1 .. y_K (Y[k] = y_{k+1})
    const float* yk;        // adjoint: y_k itself
    const float* AtAy;      // [B][P][n]
    const float* Atb;       // [B][P][n]
    const float* U;         // U_k (check0: U0)
    const float* D;         // delta_k
    float* U_next;          // U_{k+1}
    float* D_next;          // delta_{k+1}
    float* G;               // scratch [B][P][n]: clamped gradient of the iteration
    int32_t* flags;         // [GNN_FLAG_WORDS(K)]
    int32_t* status;        // nullable
    int B, P, m, m_pad, n, n_pad, K, hyp_rows, variant, graph_shared;
    const float* acc_add;   // gram mode 2 (out += A^T A x): then + acc_add [B][P][n] (nullable)
};
struct GnnGrads {
    const float* gy1;       // dL/dy_{k+1} (nullable = 0)
    const float* gU1;       // dL/dU_{k+1} (nullable)
    const float* gd1;       // dL/ddelta_{k+1} (nullable)
    float* gy;              // dL/dy_k (direct path; the AtAy path is the caller's gram)
    float* gU;              // dL/dU_k
    float* gd;              // dL/ddelta_k
    float* gAtAy;           // dL/dAtAy_k
    float* ghyp;            // dL/dhyp_k [B][4][hyp_rows]
    // training-backward epilogue (dadmm_gnn_step_backward_ex), all nullable
    const float* ghyp_add;  // added to dL/dhyp_k
    const float* hz;        // the head's logits [B][4 H]: with hdz, the head backward runs here
    float* hdz;             // d logits [B][4 H]
    float hmax[4];
};
hipError_t gnn_launch_zero(int32_t* p, int words, hipStream_t st);
hipError_t gnn_launch_check0(const GnnArgs& a, const float* y0, hipStream_t st);
hipError_t gnn_launch_gram(const GnnArgs& a, int k, const float* x_raw, float* out, int mode,
                           hipStream_t st);
hipError_t gnn_launch_step(const GnnArgs& a, int k, hipStream_t st);
hipError_t gnn_launch_finish(const GnnArgs& a, hipStream_t st);
hipError_t gnn_launch_step_backward(const GnnArgs& a, int k, const GnnGrads& gg, hipStream_t st);
size_t gnn_gram_lds(int m_pad);

// ---- one launch per iteration, state in HBM (dadmm_tiled.hip) ---------------------------------
struct TiledArgs {
    const float* A;         // prepared operator [P][m_pad][n_pad]
    const float* At;        // [P][n_pad][m_pad]
    const float* b;         // [B][P][m]
    const int32_t* vptr;    // visit lists (as StepArgs)
    const uint8_t* vq;
    const float* deg;       // [G][P]
    const float* hyp;       // [K][hyp_rows][4]
    const float* y0;        // [B][P][n]
    const float* U0;
    const float* d0;
    float* Y;               // [K][B][P][n]
    float* Ubuf[2];         // ping-pong U_k buffers [B][P][n] (scratch)
    float* delta;           // delta_k [B][P][n] (scratch, consensus_kernel)
    float* R;               // R_k = A_p y_k - b_p [B][P][m_pad] (scratch, the column-split path)
    float* U_out;           // [B][P][n] or nullptr
    int32_t* status;        // or nullptr (OR-ed DADMM_STATUS_* bits)
    int B, P, m, m_pad, n, n_pad, K, hyp_rows, variant, graph_shared;
    float* Grec;            // streamed form only, nullable: [K][B][P][n] pre-clamp gradients
    float* Urec;            //   and U_k entering iteration k (the adjoint's trajectory)
};
size_t tiled_lds_bytes(int n_pad, int m_pad);
hipError_t launch_tiled(const TiledArgs& a, hipStream_t stream);
// the whole forward in one launch, state streamed once per iteration (dadmm_stream.hip); U_k in
// place in a.Ubuf[0]
bool stream_applies(const TiledArgs& a);
hipError_t launch_stream(const TiledArgs& a, hipStream_t stream);

// ---- fused loss (dadmm_loss.hip) ----------------------------------------------------------------
struct LossArgs {
    const float* Y;         // [K][rows][n_store], rows = B * P
    const float* label;     // [B][n]
    float* partial;         // scratch: loss_scratch_floats(K, rows, n)
    float* losses;          // [K] per-layer losses (nullable)
    float* out;             // [2]: loss_mean, loss_final
    int32_t* flags;         // [2]: non-finite seen, fallback fired
    int K, P, n, n_store;
    int64_t rows;
};
size_t loss_scratch_floats(int K, int64_t rows, int n);
hipError_t launch_loss(const LossArgs& a, hipStream_t st);
hipError_t launch_loss_grad(const LossArgs& a, const float* gout, float* dY, hipStream_t st);

// ---- GNN hypernetwork, inference mode (dadmm_hyper.hip) ------------------------------------------
#define HYPER_EPI_BIAS 0   // y = x W^T + bias
#define HYPER_EPI_GCN 1    // y = BN(leaky(A_hat (x W^T) + bias)) per sample of P rows
#define HYPER_EPI_HEAD 2   // y = min(clamp(sigmoid(x W^T + bias), 1e-4, 0.9999) * max_c, ...)
#define HYPER_EPI_GCN_TRAIN 3   // y = Dropout(BN_batch(leaky(A_hat (x W^T) + bias))) per sample,
                                //     saving M = A_hat (x W^T) + bias and the samples' BN statistics
#define HYPER_EPI_GCN_BWD 4     // y = gcn_bwd(x W^T): the GCN block backward (dadmm_hyper_train.hip's
                                //     gcn_bwd_kernel) in the epilogue of the input-gradient GEMM
struct HyperArgs {
    const float* x1;        // input columns [0, K1): row r at x1 + r * ld1
    const float* x2;        // input columns [K1, K): row r at x2 + r * ld2 (nullable if K1 == K)
    int ld1, ld2, K1;
    const float* W;         // [N][ldw] (nn.Linear.weight; ldw = K unless a column slice of it)
    int ldw;
    const float* bias;      // [N] (nullable for EPI_BIAS)
    float* y;               // [rows][ldy]
    int ldy;
    int rows, K, N;         // rows = B * P for EPI_GCN
    int B, P, S_t;          // GCN: samples, rows per sample, samples per tile (set by the launcher)
    const float* ahat;      // GCN: [B or 1][P][P] normalised adjacency
    int ahat_per_sample;
    const float* bn_mean;   // GCN: BatchNorm1d running statistics and affine parameters [N]
    const float* bn_var;
    const float* bn_w;
    const float* bn_b;
    float bn_eps, slope;    // GCN: BatchNorm eps, leaky_relu negative slope
    int H;                  // HEAD: hyper-parameter rows (P or 1); N = 4 H
    float maxv[4];          // HEAD: alpha_max, tau_max, rho_max, eta_max
    int splits;             // BIAS: split-K factor; split q writes y + q * split_stride (no bias)
    size_t split_stride;
    int gm, gn;             // tile grid (set by the launcher)
    // GCN_TRAIN: saved activations and the dropout stream
    float* save_m;          // [rows][N] M = A_hat (x W^T) + bias (pre-activation)
    float* save_mean;       // [B][N] per-sample BatchNorm batch mean over the P nodes
    float* save_var;        // [B][N] per-sample biased batch variance
    float drop_p;           // dropout probability (0: none)
    uint64_t seed;          // dropout stream: keep(site, row, col) = hash(seed, site, row, col) >= p
    int site;
    // GCN (inference) only: addend [rows][ld_add] added to the mix A_hat (x W^T) before the bias
    // (nullable); raw != 0: y = A_hat (x W^T) (+ addend), no bias / leaky_relu / BatchNorm
    const float* addend;
    int ld_add, raw;
    // GCN_BWD: save_m / save_mean / save_var are the block's saved activations (read), bn_w its
    // gamma; part [3][B][N] the per-sample dgamma / dbeta / dbias sums; bn_eval: running statistics
    float* part;
    int bn_eval;
    // GCN-class GEMMs (the GCN layers forward and backward, their input gradients): the launcher
    // may split a small grid's K loop over two wave sets of each workgroup (linear_kernel KS = 2;
    // hyper_kwave decides from the GEMM shape alone). 0 for the decoder's linears, whose chains
    // dadmm_hyper_tail.hip restates.
    int kwave;
};

// Counter-based dropout mask shared by the training forward and backward kernels (the backward
// regenerates it instead of storing it): keep element (row, col) of dropout site `site` iff
// hash(seed, site, row, col) >= p * 2^32; kept elements are scaled by 1 / (1 - p) (nn.Dropout).
__host__ __device__ inline uint32_t drop_hash(uint64_t seed, int site, uint32_t row, uint32_t col) {
    uint64_t z = seed ^ ((uint64_t)(uint32_t)site << 56) ^ ((uint64_t)row << 20) ^ (uint64_t)col;
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (uint32_t)(z >> 32);
}
__host__ __device__ inline uint32_t drop_threshold(float p) {
    const double t = (double)p * 4294967296.0;
    return t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t;
}
hipError_t launch_hyper(HyperArgs a, int epi, hipStream_t st);
// dadmm_hyper_linear_ex (no bias) as a GCN-class GEMM: a GCN layer's input gradient dX = dZ W on
// its B samples of P rows, which may take the K split like the fused dadmm_hyper_linear_gcn_bwd
// of the same shape (same bits either way); the C-ABI's linears never split (the decoder's)
int hyper_linear_gcn_dx(int32_t P, int32_t rows, int32_t K, int32_t N, const float* x, int32_t ldx, const float* W,
                        const float* addend, int32_t ld_add, float* y, int32_t ldy, void* stream);
int hyper_linear_splits(int rows, int K, int N);
struct RowNormArgs {
    const float* x;         // [nsum][rows][C] (row stride C, partial q at x + q * sum_stride)
    const float* weight;
    const float* bias;
    float* y;
    int rows, C, act;
    float eps, slope;
    int nsum;               // split-K partials summed (in order) before the LayerNorm
    size_t sum_stride;
    const float* pre_bias;  // nullable: the producing linear's bias, added after the sum
    // training: dropout on the LayerNorm input (decoder: Linear -> Dropout -> LayerNorm), and the
    // post-dropout LayerNorm input saved for the backward (xd, nullable)
    float drop_p;
    uint64_t seed;
    int site;
    float* xd;
};
// LayerNorm (+ LeakyReLU) backward of rownorm rows: dx (w.r.t. the pre-dropout input when
// drop_p > 0) and per-block partial sums of dweight / dbias ([nblk][2][C], nblk = ceil(rows / 64))
struct RowNormBwdArgs {
    const float* dy;        // [rows][C]
    const float* xd;        // [rows][C] LayerNorm input (post-dropout)
    const float* weight;
    const float* bias;
    float* dx;              // [rows][C]
    float* part;            // [nblk][2][C]
    int rows, C, act;
    float eps, slope, drop_p;
    uint64_t seed;
    int site;
};
hipError_t launch_rownorm_bwd(const RowNormBwdArgs& a, hipStream_t st);
constexpr int ROWNORM_BWD_ROWS = 8;    // rows per partial-sum block (2 per wave: B = 256 rows fill 32 workgroups)
// GCN layer (train mode) backward, everything but the two GEMMs: from dy (w.r.t. the layer's
// dropout output) to dZ (w.r.t. Z = x W^T), with per-sample partials of dgamma, dbeta, dbias
struct GcnBwdArgs {
    const float* dy;        // [B*P][N]
    const float* m;         // [B*P][N] saved M
    const float* mean;      // [B][N]
    const float* var;       // [B][N]
    const float* gamma;     // [N]
    const float* ahat;      // [B or 1][P][P]
    int ahat_per_sample;
    float* dz;              // [B*P][N]
    float* part;            // [3][B][N]: dgamma, dbeta, dbias per sample
    int B, P, N;
    float eps, slope, drop_p;
    uint64_t seed;
    int site;
    int bn_eval;            // BatchNorm on constant (running) statistics: no batch-statistics terms
};
hipError_t launch_gcn_bwd(const GcnBwdArgs& a, hipStream_t st);
// dadmm_hyper_gcn_train with a column slice of W (row stride ldw >= K) and an addend
// [B*P][ld_add] (nullable) added to the mix A_hat (x W^T) before the bias (dadmm_abi.cpp)
int gcn_train_impl(int32_t B, int32_t P, int32_t K, int32_t N, const float* x1, int32_t ld1, int32_t K1,
                   const float* x2, int32_t ld2, const float* W, int32_t ldw, const float* addend, int32_t ld_add,
                   const float* bias, const float* ahat, int32_t ahat_per_sample, const float* bn_weight,
                   const float* bn_bias, float bn_eps, float slope, float drop_p, uint64_t seed, int32_t site,
                   float* y, int32_t ldy, float* m_out, float* mean_out, float* var_out,
                   const float* bn_running_mean, const float* bn_running_var, void* stream);

// The decoder tail of the training hypernetwork, one launch each way (dadmm_hyper_tail.hip): decoder
// blocks 2 and 3 (index 1, 2), fc and the head; 16 samples per workgroup
struct TailArgs {
    int B, H;
    int D[3];                 // decoder widths (dec_width 0..2)
    const float* x0;          // fwd: dec_y[0] [B][D0]
    const float* W[3];        // fwd: dec_w[1] [D1][D0], dec_w[2] [D2][D1], fc_w [4H][D2]
    const float* bias[3];     // dec_b[1], dec_b[2], fc_b
    const float* lnw[2];      // ln_w[1], ln_w[2] (and ln_b)
    const float* lnb[2];
    float eps[2], slope[2], drop[2];
    uint64_t seed;
    int site0;                // the dropout site of block index 1 (block 2: site0 + 1)
    float* xd[2];             // dec_xd[1], dec_xd[2] (fwd: written; bwd: read)
    float* y[2];              // fwd: dec_y[1], dec_y[2]
    float* z;                 // fwd: [B][4H] logits
    float* hyp;               // fwd: [B][4H]
    float maxv[4];
    const float* dz;          // bwd: [B][4H] logit gradient
    const float* Wt[3];       // bwd: dec_wt[1] [D0][D1], dec_wt[2] [D1][D2], fc_wt [D2][4H]
    float* dv[2];             // bwd: the blocks' dZ [B][D1], [B][D2]
    float* part[2];           // bwd: their LayerNorm partials [ceil(B / 8)][2][D]
    float* dx0;               // bwd: [B][D0] gradient of dec_y[0]
};
size_t tail_lds_bytes(const TailArgs& a, bool bwd);
hipError_t launch_tail(const TailArgs& a, bool bwd, hipStream_t st);

// BatchNorm running statistics after T = iters * B sequential train-mode calls, closed form
// (dadmm_hyper_bn_running_update): up to BN_MAX_LAYERS layers in one pair of launches
constexpr int BN_MAX_LAYERS = 8;
struct BnRunArgs {
    int layers, iters, B, P;
    int width[BN_MAX_LAYERS];
    int col0[BN_MAX_LAYERS + 1];          // prefix sums of width (column offsets in the partials)
    float* rmean[BN_MAX_LAYERS];
    float* rvar[BN_MAX_LAYERS];
    int64_t* tracked[BN_MAX_LAYERS];      // num_batches_tracked (nullable)
    const float* mean[BN_MAX_LAYERS];     // [iters blocks][B][width] at block_stride floats
    const float* var[BN_MAX_LAYERS];
    int64_t block_stride;
    const double* w;                      // [T] momentum (1 - momentum)^(T - 1 - t)
    double decay;                         // (1 - momentum)^T
    double* part;                         // [splits][2][col0[layers]] float64 partial sums
    int splits;
};
hipError_t launch_bn_running(const BnRunArgs& a, hipStream_t st);
// hyper-parameter head: mode 0: hyp = head(z); mode 1: dz = dhyp * head'(z); z, hyp, dhyp [B][4H]
hipError_t launch_head_act(int mode, int B, int H, const float* z, const float* dhyp, const float* maxv4,
                           float* out, hipStream_t st);
hipError_t launch_rownorm(const RowNormArgs& a, hipStream_t st);

// ---- training-mode parameter gradients (dadmm_hyper_grad.hip) ----------------------------------
// g [N][K] (+)= dZ^T X over R rows; X = cat of two column segments (x1: columns < K1, x2: the
// rest); gbias [N] (+)= column sums of dZ (nullable); splits > 1: partial tiles in scratch
struct WgradArgs {
    const float* dz;        // [R][ldz]
    const float* x1;        // [R][ld1]
    const float* x2;        // [R][ld2] (K1 == K: unused)
    float* g;               // [N][K]
    float* gbias;           // [N] or nullptr
    float* scratch;         // [splits][N][K] when splits > 1
    float* scratch_bias;    // [splits][N] when splits > 1 and gbias
    int R, N, K, K1, ldz, ld1, ld2, splits, beta;
    // batches (deferred training gradients): nb blocks of R rows, block b at dz + b zs,
    // x1 + b s1, x2 + b s2 (floats); nb = 1 for one block
    int nb = 1;
    size_t zs = 0, s1 = 0, s2 = 0;
};
int wgrad_splits(int R, int N, int K);
hipError_t launch_wgrad(const WgradArgs& a, hipStream_t st);
// out [G][C] (+)= sum over r of part [G][R][C] (fixed order); bscratch [G][nb][C] floats: the
// two-stage form for nb > 1 batch blocks
hipError_t launch_colsum(const float* part, int G, int R, int C, float* out, int beta, hipStream_t st,
                         int nb = 1, size_t pstride = 0, float* bscratch = nullptr);
// out [cols][rows] = in [rows][cols]
hipError_t launch_transpose(const float* in, int rows, int cols, float* out, hipStream_t st);

// ---- device-side ER graph generation (dadmm_graphgen.hip) ---------------------------------------
struct GraphGenArgs {
    int B, P;
    float prob;
    uint64_t seed;
    int connect;            // apply the progressive driver's connectivity patch
    int64_t* nbr;           // [B][P] neighbour masks
    float* deg;             // [B][P]
    int32_t* order;         // [B][P] packed adjacency order (P <= 8) or nullptr
    int32_t* counts;        // scratch [B]: visit entries per sample, then their offsets
    int32_t* vptr;          // [B*P + 1]
    uint8_t* vq;            // visit lists (nullptr: offsets only)
};
hipError_t launch_graphgen(const GraphGenArgs& a, int pass, hipStream_t st);

// ---- forward prologue (dadmm_rng.hip) -----------------------------------------------------------
struct PrologueArgs {
    uint64_t seed, offset, offset_step;   // torch Philox state; per-tensor offset increment
    int64_t numel;                        // B*P*n per tensor (0: no draw)
    int64_t threads;                      // torch's 256 * grid virtual threads
    int64_t n, n_store;                   // row length drawn / stored
    float mean, stddev;
    float* y0;
    float* U0;
    float* d0;
    int32_t* zero;                        // words zeroed by the same launch
    int64_t nzero;
};
hipError_t launch_prologue(const PrologueArgs& a, hipStream_t stream);

// Operator preparation kernel launcher (dadmm_prepare.hip).
hipError_t launch_prepare(const float* A, float* Apad, float* Atpad, int P, int m, int n,
                          int n_pad, hipStream_t stream);

// ---- stepwise path (dadmm_stepwise.hip) --------------------------------------------------------
// flag words (int32, zeroed before every forward): barrier counter, barrier timeout, y0 guard,
// exit counter, then per iteration k: U_k non-finite, gradient NaN, y_next non-finite (U_K is index K).
#define SW_F_BARRIER 0
#define SW_F_TIMEOUT 1
#define SW_F_Y0 2
#define SW_F_EXIT 3    // persistent form: workgroups past their last write (the last one finishes)
#define SW_F_UBAD(k) (4 + 4 * (k))
#define SW_F_GBAD(k) (5 + 4 * (k))
#define SW_F_YNB(k) (6 + 4 * (k))
#define SW_FLAG_WORDS(K) (4 + 4 * ((K) + 1))

struct StepArgs {
    const float* A;         // prepared operator [P][m_pad][n_pad]
    const float* At;        // [P][n_pad][m_pad]
    const float* b;         // [B][P][m]
    const int32_t* vptr;    // visit lists: [G*P + 1] offsets into vq (G = 1 shared, B otherwise)
    const uint8_t* vq;      // neighbour ids in the reference's accumulation order
    const float* deg;       // [G][P]
    const float* hyp;       // [K][hyp_rows][4]
    const float* y0;        // [B][P][n]
    const float* U0;
    const float* d0;
    float* Y;               // [K][B][P][n]
    float* U;               // [B][P][n]: U_k (caller's U_out or scratch)
    float* D;               // [B][P][n]: delta_k (scratch)
    float* G;               // [B][P][n]: gradient of the current iteration (scratch)
    int32_t* flags;         // [SW_FLAG_WORDS(K)] (scratch)
    int32_t* status;        // [1]
    float* Grec;            // nullable [K][B][P][n]: pre-clamp gradient of iteration k
    float* Urec;            // nullable [K][B][P][n]: U_k entering iteration k
    int B, P, m, m_pad, n, n_pad, K, hyp_rows, variant, graph_shared;
};

size_t stepwise_flag_bytes(int K);
// gate = 1: one persistent launch that runs only if *status != 0 when it starts
hipError_t launch_stepwise(const StepArgs& a, int gate, bool flags_zeroed, hipStream_t stream);

inline int fused_nt(int n) {
    const int nt = (n + 63) / 64;
    return nt <= 1 ? 1 : (nt <= 2 ? 2 : (nt <= 4 ? 4 : nt));
}

}  // namespace dadmm
