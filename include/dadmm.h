/*
 * dadmm.h — C ABI of the MI355X (gfx950) unfolded D-ADMM forward path.
 *
 * This is the drop-in boundary below the Python modules that mirror the reference's
 * `unfolded_DLASSO.DLASSO_unfolded` (reference: unfolded_DLASSO.py:9-146). The reference has
 * no native code and no FFI of its own (SURVEY.md §2 "Native / kernel / collective inventory");
 * each entry point below replaces a group of torch eager ops / Python loops of the reference's
 * forward, cited per function. A ctypes binding (the reference is Python) is shown in
 * INTEGRATION.md.
 *
 * Conventions (all entry points):
 *   - every tensor pointer is a DEVICE pointer, fp32 row-major, caller-owned; nothing is
 *     allocated inside; work is enqueued asynchronously on `stream` (a hipStream_t, or NULL for
 *     the legacy default stream);
 *   - return 0 (DADMM_OK) on success, a negative DADMM_E* code otherwise; the message is
 *     available from dadmm_last_error() (thread-local); no C++ exception crosses the ABI;
 *   - no mutable global state: calls on different streams are independent and re-entrant.
 *
 * Layouts (B batch, P agents, m rows per agent, n signal dim, K unrolled iterations):
 *   A      [P][m][n]        per-agent sensing matrices (reference A[0], shape [1,P,m,n])
 *   b      [B][P][m]        measurements              (reference b,    shape [B,P,m,1])
 *   nbr    [B][P] uint64    bit q of nbr[s][p] set <=> q in graph_list[s].neighbors(p)  (P <= 64);
 *                           neighbours are visited in ascending order (networkx order for
 *                           erdos_renyi_graph); [P] when dims.graph_shared
 *   nbr_order [B][P] uint32 (nullable) graph.neighbors(p) in adjacency order, 4 bits per id,
 *                           first neighbour in the low nibble (P <= 8, per-sample graphs only);
 *                           NULL means ascending order
 *   deg    [B][P]           compute_sum_neighbors output (reference [B,P,1,1]); [P] when shared
 *   hyp    [K][H][4]        per-iteration (alpha, tau, rho, eta), H = P ('diff') or 1 ('same')
 *   y0,U0,d0 [B][P][n]      initial primal / dual / consensus states (reference draws them)
 *   Y      [K][B][P][n]     every iterate y_1..y_K     (reference Y, shape [K,B,P,n,1])
 *
 * Compiled configurations of dadmm_forward: P <= 6 (P <= 5 at n > 128), m <= 64, n <= 256,
 * n % 4 == 0 (callers zero-pad n otherwise: zero columns of A are inert), B*P*n*4 < 2^31.
 * Anything else returns DADMM_EUNSUPPORTED.
 */
#ifndef DADMM_H_
#define DADMM_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DADMM_ABI_VERSION 1

enum {
    DADMM_OK = 0,
    DADMM_EINVAL = -1,       /* bad dimensions / null pointer / misaligned pointer          */
    DADMM_EUNSUPPORTED = -2, /* shape outside every compiled kernel configuration            */
    DADMM_EHIP = -3          /* a HIP runtime call failed (message holds hipGetErrorString) */
};

enum {
    DADMM_VARIANT_UNFOLDED = 0, /* unfolded_DLASSO.py:79-99: k-dependent clamps, no delta clamp */
    DADMM_VARIANT_GNN = 1       /* gnn_dlasso_models_progressive.py:211-232: fixed clamps       */
};

/* Bits of the `status` word written by dadmm_forward (nullable). A set bit means a non-finite
 * value reached one of the reference's NaN/Inf guards (unfolded_DLASSO.py:55-61, 84-86,
 * 102-104). The fused kernel does not apply those batch-global resets; a caller that sees a
 * non-zero status re-runs the batch through dadmm_forward_guarded. */
enum {
    DADMM_STATUS_Y_NONFINITE = 1,    /* y_k had NaN/Inf at the top of an iteration   (:55)   */
    DADMM_STATUS_U_NONFINITE = 2,    /* U_k had NaN/Inf at the top of an iteration   (:59)   */
    DADMM_STATUS_GRAD_NAN = 4,       /* clamped gradient had NaN                     (:84)   */
    DADMM_STATUS_YNEXT_NAN = 8       /* clamped y_next had NaN                       (:102)  */
};

typedef struct dadmm_dims {
    int32_t B, P, m, n, K;
    int32_t variant;  /* DADMM_VARIANT_*                                  */
    int32_t hyp_rows; /* P for DADMM_mode 'diff', 1 for 'same'             */
    int32_t graph_shared; /* 1: every sample uses ONE graph; nbr and deg are then [P] arrays
                           *    (graph_list = [graph]*B, unfolded_train_new.py:67);
                           * 0: per-sample graphs, nbr and deg are [B][P]                   */
} dadmm_dims;

/* ABI version of the loaded library (== DADMM_ABI_VERSION of the header it was built from). */
int dadmm_abi_version(void);

/* Thread-local description of the last failure on this thread ("" if none). */
const char* dadmm_last_error(void);

/* Bytes of device workspace that hold the prepared (padded, transposed) operator for `d`. */
size_t dadmm_operator_bytes(const dadmm_dims* d);

/* Prepare the per-agent operator once per A.
 * Replaces: DLASSO_unfolded.__init__'s `self.AtA = self.compute_Atx(self.A)`
 *           (unfolded_DLASSO.py:16, :120-124). The Gram matrix is never formed: the kernels use
 *           the factored gradient A_p^T (A_p y - b_p); this call lays A out padded (rows to 64,
 *           columns to a multiple of 64) together with its transpose in `op`
 *           (dadmm_operator_bytes(d) bytes, 16-byte aligned). */
int dadmm_prepare_operator(const dadmm_dims* d, const float* A, void* op, void* stream);

/* The K-step unfolded D-ADMM forward, fused: one launch runs all K iterations.
 * Replaces: DLASSO_unfolded.forward's loop body (unfolded_DLASSO.py:45, 53-109):
 *           compute_Atx(b) (:45), the P per-agent AtA@y GEMVs (:69-71), the gradient assembly,
 *           clamps and primal update (:73-93), compute_delta (:95, :127-140), the dual update
 *           (:98-99) and torch.stack(Y) (:109). Inputs compute_sum_neighbors (:46 -> `deg`),
 *           the random inits (:49-51 -> y0/U0/d0) and seq_hyp(k) (:63 -> `hyp`) are produced by
 *           the caller.
 * `U_out` ([B][P][n], nullable) receives U_K. `status` (one int32, nullable) is OR-ed with
 * DADMM_STATUS_* bits; the caller zeroes it. */
int dadmm_forward(const dadmm_dims* d, const void* op, const float* b, const uint64_t* nbr,
                  const uint32_t* nbr_order, const float* deg, const float* hyp, const float* y0,
                  const float* U0, const float* d0, float* Y, float* U_out, int32_t* status,
                  void* stream);

#ifdef __cplusplus
}
#endif

#endif /* DADMM_H_ */
