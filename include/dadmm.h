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
 *   nbr    [B][P] uint64    bit q of nbr[s][p] set <=> q in graph_list[s].neighbors(p)  (P <= 64;
 *                           read only by the fused kernels: any valid pointer past 64 agents);
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
 *   visit_ptr [G*P+1] int32, visit_q [visit_ptr[G*P]] uint8 (stepwise path): for agent p of
 *                           graph g, the neighbour ids q in the order compute_delta
 *                           (unfolded_DLASSO.py:127-140) accumulates delta[p]: every p' < p
 *                           with p in neighbors(p'), then neighbors(p) in adjacency order, then
 *                           every p' > p with p in neighbors(p'); G = 1 when dims.graph_shared,
 *                           else B
 *
 * Compiled configurations of dadmm_forward (fused): P <= 6 (P <= 5 at n > 128), m <= 64,
 * n <= 256, n % 4 == 0 (callers zero-pad n otherwise: zero columns of A are inert),
 * B*P*n*4 < 2^31. Anything else returns DADMM_EUNSUPPORTED; dadmm_forward_tiled covers
 * P <= 255, m <= 128, and dadmm_forward_stepwise every P <= 140, m <= 1024, n % 4 == 0
 * (the reference's defaults m = 100, n = 500, configurations.py:6-9, run on the tiled path).
 * Agents are limited by the visit lists' uint8 ids (255) and by the kernels' per-wave LDS rows
 * (the stepwise update: 4 waves x P x 64 floats; longer visit lists than 4 KB per wave are walked
 * from global memory): a shape whose LDS would not fit returns an error instead of launching.
 */
#ifndef DADMM_H_
#define DADMM_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DADMM_ABI_VERSION 18

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

/* Bits of the `status` word. A set bit means a non-finite value reached one of the reference's
 * batch-global NaN/Inf guards (unfolded_DLASSO.py:55-61, 84-86, 102-104).
 *   dadmm_forward (fused) does NOT apply the guards: it ORs in the bits of every case where the
 *   reference would have fired one (bit 8 also for a non-finite hyper-parameter), and its Y is
 *   then not the reference's. dadmm_forward_stepwise with gate = 1, enqueued right after it on
 *   the same stream, recomputes exactly such batches on the device (no host round trip).
 *   dadmm_forward_stepwise applies the guards exactly and stores the bits of the guards that
 *   fired (the reference prints one warning per fired guard). */
enum {
    DADMM_STATUS_Y_NONFINITE = 1,    /* y_k had NaN/Inf at the top of an iteration   (:55)   */
    DADMM_STATUS_U_NONFINITE = 2,    /* U_k had NaN/Inf at the top of an iteration   (:59)   */
    DADMM_STATUS_GRAD_NAN = 4,       /* clamped gradient had NaN                     (:84)   */
    DADMM_STATUS_YNEXT_NAN = 8,      /* y_next had NaN/Inf                           (:102)  */
    DADMM_STATUS_RECOMPUTE = 16,     /* dadmm_forward only: the shared adjacency is not
                                      * symmetric, so the fused consensus cannot follow it;
                                      * dadmm_forward_split: a wait between slices timed out;
                                      * the gated stepwise run recomputes the batch (never set
                                      * after a gated run)                                    */
    DADMM_STATUS_BARRIER_TIMEOUT = 0x100 /* gated stepwise run could not synchronise its grid
                                          * (device shared with other work): Y is invalid    */
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
 *           the factored gradient A_p^T (A_p y - b_p); this call lays A out padded (rows to a
 *           multiple of 64, columns to a multiple of 64) together with its transpose in `op`
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

/* The same forward for SMALL batches, columns split over workgroups (csrc/dadmm_split.hip).
 * Replaces: the same reference lines as dadmm_forward (unfolded_DLASSO.py:45, 53-109).
 * dadmm_forward's 16-sample tiles fill ceil(B / 16) CUs; here each tile's n_pad columns are cut
 * into slices of 64, one workgroup each, with the operator slice resident in LDS and the GEMM1
 * partial sums A_p[:, slice] y_p[slice] exchanged between the slices every iteration. GEMM1 is
 * then R = ((c_0 + c_1) + c_2) + ... (slice 0's chain from -b, the others from +0), an order of
 * its own: bit-identical to the oracle's oracle_forward_f32_split(split_cols = 64), not to
 * dadmm_forward. Shapes: dadmm_forward's with n_pad = 128 or 256; applies when the batch fills at
 * most half of the device's CUs (ceil(B / 16) <= CUs / 2): dadmm_split_scratch_bytes is 0 otherwise.
 * `scratch`: dadmm_split_scratch_bytes(d) bytes (the partial sums), 16-byte aligned, any content;
 * `flags`: dadmm_split_flag_bytes(d) bytes (the epoch words), 16-byte aligned, ZERO at every call
 * (the prologue's `zero` words can clear them). A wait between slices is bounded: if the workgroups are not
 * co-resident (the device shared with other work) the launch sets DADMM_STATUS_RECOMPUTE and the
 * gated dadmm_forward_stepwise enqueued after it recomputes the batch exactly. Same outputs and
 * `status` contract as dadmm_forward (no recording). */
size_t dadmm_split_scratch_bytes(const dadmm_dims* d);
size_t dadmm_split_flag_bytes(const dadmm_dims* d);
int dadmm_forward_split(const dadmm_dims* d, const void* op, const float* b, const uint64_t* nbr,
                        const uint32_t* nbr_order, const float* deg, const float* hyp,
                        const float* y0, const float* U0, const float* d0, float* Y, float* U_out,
                        int32_t* status, void* flags, void* scratch, void* stream);

/* dadmm_forward that also records the trajectory the adjoint (dadmm_backward) consumes — the
 * training-mode forward (the drivers call loss.backward() through it: unfolded_train_new.py:74-80).
 *   Grec [K][B][P][n]: the gradient of iteration k BEFORE its clamp (unfolded_DLASSO.py:73-77)
 *   Urec [K][B][P][n]: U_k entering iteration k
 * Y is bit-identical to dadmm_forward's. Same shapes as dadmm_forward. */
int dadmm_forward_record(const dadmm_dims* d, const void* op, const float* b, const uint64_t* nbr,
                         const uint32_t* nbr_order, const float* deg, const float* hyp,
                         const float* y0, const float* U0, const float* d0, float* Y, float* Grec,
                         float* Urec, float* U_out, int32_t* status, void* stream);

/* Bits of the `gate` argument of dadmm_forward_stepwise. */
enum {
    DADMM_GATE_ON = 1,        /* run only if *status != 0 when the launch starts (see below)     */
    DADMM_FLAGS_ZEROED = 2    /* the scratch's flag words are already zero (dadmm_prologue)      */
};

/* Philox offset increment torch's normal_ consumes per tensor of `numel` float elements on the
 * current device (ATen/native/hip/DistributionTemplates.h calc_execution_policy). */
uint64_t dadmm_normal_offset_step(int64_t numel);

/* The forward's prologue, one launch:
 *   - when numel > 0, the reference's random inits (unfolded_DLASSO.py:49-51)
 *       y0, U0, d0 = torch.randn((B, P, n, 1)) * 1e-2, drawn in that order,
 *     bit-identical to three torch normal_(mean, stddev) calls on the generator state (seed,
 *     offset), the k-th at offset + k * dadmm_normal_offset_step(numel) (the caller advances its
 *     generator by 3 steps). numel = B*P*n; rows of n values are stored with stride n_store >= n
 *     (padding columns untouched);
 *   - zeroes `nzero` int32 words at `zero` (the status word / guard flags of the forward).
 * Replaces: the three torch.randn(...) * 1e-2 draws (6 eager kernels) and the status / flag fills. */
int dadmm_prologue(uint64_t seed, uint64_t offset, int64_t numel, int32_t n, int32_t n_store,
                   float mean, float stddev, float* y0, float* U0, float* d0, int32_t* zero,
                   int64_t nzero, void* stream);

/* Bytes of device scratch dadmm_forward_tiled needs for `d` (256-byte aligned pointer). */
size_t dadmm_tiled_scratch_bytes(const dadmm_dims* d);

/* The K-step forward for shapes the fused kernel cannot hold on chip (P > 6 or n > 256; e.g. P = 16,
 * n = 512), state in HBM. For P <= 16, m <= 64, n_pad >= 128 it is ONE launch (the streamed form,
 * dadmm_stream.hip: 16 samples x all agents per workgroup, y_k staged per 32-column block, R_k in
 * registers, the next iteration's GEMM1 fused into the update; environment DADMM_TILED_STREAM=0
 * selects the per-iteration launches below instead). Otherwise two launches per iteration: a consensus launch forms
 * delta_k for every agent of a sample from y_k (visit lists, the reference's order; scratch), then
 * each (32-sample tile, agent) workgroup applies the deferred dual update, the factored gradient
 * GEMM pair and the primal update; Y is bit-identical to dadmm_forward_stepwise's on guard-free
 * inputs. Scratch: the U_k ping-pong pair, delta_k and R_k (dadmm_tiled_scratch_bytes).
 * Environment DADMM_TILED_SPLIT=1 selects the column-split form instead (P <= 16): a GEMM1 launch
 * writes R_k = A_p y_k - b_p, then one launch per iteration takes a (32-sample, column block) x all
 * agents, forms delta_k in LDS and applies the updates; bit-identical, slower at configs[2].
 * Replaces: the same loop as dadmm_forward (unfolded_DLASSO.py:45, 53-109).
 * Like dadmm_forward it only FLAGS the reference's guards in `status` (OR-ed; caller zeroes it):
 * enqueue dadmm_forward_stepwise with DADMM_GATE_ON behind it for the exact guarded result.
 * Graph: visit_ptr / visit_q / deg as dadmm_forward_stepwise. P <= 64, m <= 128, n % 4 == 0. */
int dadmm_forward_tiled(const dadmm_dims* d, const void* op, const float* b,
                        const int32_t* visit_ptr, const uint8_t* visit_q, const float* deg,
                        const float* hyp, const float* y0, const float* U0, const float* d0,
                        float* Y, float* U_out, int32_t* status, void* scratch, void* stream);

/* dadmm_forward_tiled that also records the adjoint's trajectory, as dadmm_forward_record does for
 * the fused shapes: Grec [K][B][P][n] = the pre-clamp gradient of iteration k (unfolded_DLASSO.py:
 * 73-77) and Urec [K][B][P][n] = U_k entering iteration k; bit-identical to the stepwise recording
 * (dadmm_forward_stepwise with Grec / Urec) on guard-free inputs. Only the streamed single-launch
 * form records: P <= 16, m <= 64, n_pad >= 128 (DADMM_EUNSUPPORTED otherwise: record with
 * dadmm_forward_stepwise). Guards are flagged in `status` as by dadmm_forward_tiled; the gated
 * dadmm_forward_stepwise behind it (with the same Grec / Urec) re-records a flagged batch exactly.
 * Replaces: the forward half of loss.backward() through DLASSO_unfolded (unfolded_train_new.py:74-80). */
int dadmm_forward_tiled_record(const dadmm_dims* d, const void* op, const float* b,
                               const int32_t* visit_ptr, const uint8_t* visit_q, const float* deg,
                               const float* hyp, const float* y0, const float* U0, const float* d0,
                               float* Y, float* Grec, float* Urec, float* U_out, int32_t* status,
                               void* scratch, void* stream);

/* Bytes of device scratch dadmm_forward_stepwise needs for `d` (256-byte aligned pointer). */
size_t dadmm_stepwise_scratch_bytes(const dadmm_dims* d);

/* The K-step forward one iteration at a time, with the reference's batch-global NaN/Inf guards
 * applied exactly (unfolded_DLASSO.py:55-61, 84-86, 102-104) — same operation order as the fused
 * kernel, so on guard-free inputs its Y is bit-identical to dadmm_forward's.
 * Replaces: the same loop as dadmm_forward (unfolded_DLASSO.py:45, 53-109), for every shape.
 * Graph: visit_ptr / visit_q (layout above) and deg ([P] when graph_shared, else [B][P]).
 * gate bits DADMM_GATE_ON / DADMM_FLAGS_ZEROED (the latter skips the flag memset).
 * gate = 0: always runs (2K + 2 launches).
 * gate = 1: ONE persistent launch that returns at once unless *status != 0 when it starts: the
 *           exact recomputation of a batch the fused dadmm_forward flagged, enqueued right after it
 *           on the same stream. One workgroup per CU synchronised by an in-launch grid barrier;
 *           the device must not be shared with other work (DADMM_STATUS_BARRIER_TIMEOUT).
 * `status` (required for gate = 1) is overwritten with the DADMM_STATUS_* bits of the guards that
 * fired. `scratch`: dadmm_stepwise_scratch_bytes(d) bytes. Grec / Urec (nullable, both or neither):
 * the trajectory recording of dadmm_forward_record. */
int dadmm_forward_stepwise(const dadmm_dims* d, const void* op, const float* b,
                           const int32_t* visit_ptr, const uint8_t* visit_q, const float* deg,
                           const float* hyp, const float* y0, const float* U0, const float* d0,
                           float* Y, float* U_out, float* Grec, float* Urec, int32_t* status,
                           int32_t gate, void* scratch, void* stream);

/* Bytes of device scratch dadmm_backward needs for `d` (16-byte aligned pointer). */
size_t dadmm_backward_scratch_bytes(const dadmm_dims* d);

/* The adjoint of the K-step forward w.r.t. the hyper-parameter table: dhyp [K][H][4] (overwritten)
 * = d(sum_k <gY[k], Y[k]>)/d hyp along the trajectory (Y, Grec, Urec) that dadmm_forward_record
 * (or dadmm_forward_stepwise with recording) produced from the same operands; the derivative torch
 * autograd takes through the reference's forward (unfolded_DLASSO.py:53-107 with clamp / sign /
 * compute_delta backward rules), i.e. what loss.backward() delivers to the seq_hyp rows
 * (unfolded_train_new.py:78). Valid only when that forward's status was 0 (no guard fired).
 * Replaces: the autograd backward of the reference's eager forward graph.
 * Same shapes and graph operands as dadmm_forward; deterministic (fixed reduction order). */
int dadmm_backward(const dadmm_dims* d, const void* op, const uint64_t* nbr,
                   const uint32_t* nbr_order, const float* deg, const float* hyp, const float* y0,
                   const float* d0, const float* Y, const float* Grec, const float* Urec,
                   const float* gY, float* dhyp, void* scratch, void* stream);

/* Per-sample Erdos-Renyi agent graphs generated on the device, directly in the graph layouts
 * above: nbr [B][P], deg [B][P], order [B][P] (nullable; P <= 8), vptr [B*P+1], vq.
 * Replaces: the progressive driver's per-batch host loop (gnn_dlasso_progressive.py:181-191:
 *           nx.erdos_renyi_graph(P, prob) per sample, and with `connect` the edges that join its
 *           connected components in order) plus the ingestion of those graphs
 *           (unfolded_DLASSO.py:111-118, :127-140's graph walk).
 * Pair u < v of sample s is an edge iff a counter-based hash of (seed, s, u, v) maps below
 * `prob` (dadmm_graphgen.hip; reproducible, not networkx's RNG stream). Two calls: with
 * vq = NULL it writes nbr / deg / order / vptr (vptr[B*P] = the number of visit entries; the
 * caller reads it to size vq) and keeps per-sample offsets in `scratch` (B int32); the second
 * call, same arguments plus vq, writes the visit lists. */
int dadmm_graph_generate(int32_t B, int32_t P, float prob, uint64_t seed, int32_t connect,
                         int64_t* nbr, float* deg, int32_t* order, int32_t* vptr, uint8_t* vq,
                         int32_t* scratch, void* stream);

/* Bytes of device scratch dadmm_adjoint needs for `d` (256-byte aligned pointer). */
size_t dadmm_adjoint_scratch_bytes(const dadmm_dims* d);

/* The same adjoint as dadmm_backward for EVERY shape (P <= 255 within the LDS budget: 4, 2 or 1
 * waves per workgroup by agent count; m <= 1024, n % 4 == 0): the state
 * (dL/dy, dL/dU, the later iteration's gradient adjoint) lives in `scratch`, two launches per
 * reverse iteration (elementwise + consensus adjoint per (sample, 64 columns); the forward's
 * factored Gram pair for A^T A gr_bar). Takes the stepwise path's visit lists (the reference's
 * compute_delta order, unfolded_DLASSO.py:127-140) instead of the neighbour masks, so it also
 * covers the tiled / stepwise trajectories, e.g. the reference's defaults m = 100, n = 500
 * (configurations.py:6-9) under unfolded_train_new.py:74-80's loss.backward().
 * Replaces: the autograd backward of the reference's eager forward graph (as dadmm_backward).
 * Valid only when the recorded forward's status was 0; deterministic (fixed reduction order). */
int dadmm_adjoint(const dadmm_dims* d, const void* op, const int32_t* visit_ptr,
                  const uint8_t* visit_q, const float* deg, const float* hyp, const float* y0,
                  const float* d0, const float* Y, const float* Grec, const float* Urec,
                  const float* gY, float* dhyp, void* scratch, void* stream);

/* ---- GNN-hypernetwork model: per-iteration entry points --------------------------------------
 * DLASSO_GNNHyp3_Progressive.forward (gnn_dlasso_models_progressive.py:131-243) evaluates a GNN on
 * [A^T A y_k, A^T b] between iterations, so its loop runs one iteration per call, the caller
 * evaluating the hypernetwork in between:
 *   dadmm_gnn_begin                 once: zero the flags, k = 0 guards, Atb = A^T b
 *   for k in 0..K-1:
 *     dadmm_gnn_gram(k)             AtAy_k = A^T (A y_k)        (:158-162)
 *     [caller]                      hyp_k [B][4][H] from the hypernetwork (:165-196)
 *     dadmm_gnn_step(k)             gradient, clamps, y/delta/U updates, guards (:205-237)
 *   dadmm_gnn_finish                Y[K-1] guard fix-up, status bits
 * Y storage: `yptr` is a DEVICE array of K+1 float pointers: y0, then y_1 .. y_K, each [B][P][n]
 * (y_{k+1} = the reference's Y[k]; they may be the K slices of one [K][B][P][n] tensor). The
 * guards are the reference's batch-global NaN/Inf resets (:150-156, :216-218, :235-237), decided
 * on the device through `flags` (dadmm_gnn_flag_bytes(K) bytes): no host synchronisation.
 * Graph operands are the stepwise path's visit lists and degrees; H = dims.hyp_rows (P for
 * 'diff', 1 for 'same'); dims.variant selects the clamps (1 for this model). Shapes: P <= 255
 * (the step kernel stages P x 128 floats per workgroup), m <= 1024, n % 4 == 0. */
size_t dadmm_gnn_flag_bytes(int32_t K);
int dadmm_gnn_begin(const dadmm_dims* d, const void* op, const float* b, const float* y0,
                    const float* U0, float* Atb, int32_t* flags, void* stream);
/* out = A^T (A y_k) with y_k resolved through the guards (x == NULL), or out = A^T (A x) for an
 * explicit x [B][P][n] (the adjoint of AtAy; flags / yptr unused then). */
int dadmm_gnn_gram(const dadmm_dims* d, const void* op, int32_t k, float* const* yptr,
                   const int32_t* flags, const float* x, float* out, void* stream);
/* out += A^T (A x) (ABI 15): the GNN adjoint's y gradient picks up the gram of the AtAy gradient
 * in one launch instead of a gram and an add (bit-identical: out + the gram's value, one rounding).
 * ABI 17: then out += addend [B][P][n] (nullable; 16-byte aligned) in the same epilogue — the
 * loss's own gradient on y_k, (out + gram) + addend, the bits of a separate add after. */
int dadmm_gnn_gram_acc(const dadmm_dims* d, const void* op, const float* x, float* out, const float* addend,
                       void* stream);
/* One iteration: reads y_k (resolved), U_k (U, reset by the guard), delta_k (D), AtAy_k, Atb and
 * hyp_k [B][4][H]; writes y_{k+1} to yptr[k+1], U_{k+1} to U_next, delta_{k+1} to D_next.
 * G: [B][P][n] scratch. */
int dadmm_gnn_step(const dadmm_dims* d, int32_t k, const int32_t* visit_ptr, const uint8_t* visit_q,
                   const float* deg, const float* hyp_k, float* const* yptr, const float* AtAy,
                   const float* Atb, const float* U, const float* D, float* U_next, float* D_next,
                   float* G, int32_t* flags, void* stream);
int dadmm_gnn_finish(const dadmm_dims* d, float* const* yptr, int32_t* flags, int32_t* status,
                     void* stream);
/* The adjoint of one dadmm_gnn_step (no guard fired): from dL/d(y_{k+1}, U_{k+1}, delta_{k+1})
 * (nullable = zero) to dL/d(y_k, U_k, delta_k, AtAy_k) [B][P][n] and dL/dhyp_k [B][4][H]
 * (dL/dy_k excludes the path through AtAy_k: add dadmm_gnn_gram of dL/dAtAy_k). */
int dadmm_gnn_step_backward(const dadmm_dims* d, int32_t k, const int32_t* visit_ptr,
                            const uint8_t* visit_q, const float* deg, const float* hyp_k,
                            const float* y_k, const float* AtAy, const float* Atb, const float* U,
                            const float* D, const float* gy1, const float* gU1, const float* gd1,
                            float* gy, float* gU, float* gd, float* gAtAy, float* ghyp,
                            void* stream);
/* dadmm_gnn_step_backward_ex (ABI 17): dadmm_gnn_step_backward with the training backward's next
 * element-wise step in its epilogue (the add and the head's launch saved per iteration):
 *   head (nullable): dL/dhyp_k += head->ghyp_add (nullable), then the hyper-parameter head's
 *     backward (dadmm_hyper_head_act mode 1 on the logits head->z [B][4H], bit-identical) into
 *     head->dz [B][4H], the gradient dadmm_hyper_train_backward_deferred takes with flag bit 1.
 * Replaces the step's adjoint + the add + the head's derivative of
 * gnn_dlasso_models_progressive.py:165-237 under torch's backward. */
typedef struct dadmm_head_bwd {
    const float* z;         /* [B][4H] logits (dadmm_hyper_saved.z) */
    const float* ghyp_add;  /* nullable: added to dL/dhyp_k first */
    float maxv[4];          /* alpha_max, tau_max, rho_max, eta_max */
    float* dz;              /* [B][4H] out */
} dadmm_head_bwd;
int dadmm_gnn_step_backward_ex(const dadmm_dims* d, int32_t k, const int32_t* visit_ptr,
                               const uint8_t* visit_q, const float* deg, const float* hyp_k,
                               const float* y_k, const float* AtAy, const float* Atb, const float* U,
                               const float* D, const float* gy1, const float* gU1, const float* gd1,
                               float* gy, float* gU, float* gd, float* gAtAy, float* ghyp,
                               const dadmm_head_bwd* head, void* stream);

/* ---- the drivers' loss, fused ----------------------------------------------------------------
 * gnn_dlasso_utils.compute_loss (gnn_dlasso_utils.py:27-88) on the iterates Y [K][B*P][n_store]
 * (row stride n_store >= n; padding columns ignored) and label [B][n]:
 *   losses[k] = sum_{b,p,c} (Y[k,b,p,c] - label[b,c])^2 / (B P n),
 *   out = (mean_k losses + 1e-8, losses[K-1] + 1e-8), or (1, 1) when Y, the label or a loss is
 *   non-finite (flags[1] = 1 then). Deterministic (fixed-order sums). No host synchronisation.
 * Replaces: compute_loss's K*P F.mse_loss calls and its NaN/Inf checks. */
size_t dadmm_loss_scratch_bytes(int32_t K, int64_t rows, int32_t n);
int dadmm_loss(int32_t K, int32_t B, int32_t P, int32_t n, int32_t n_store, const float* Y,
               const float* label, float* losses, float* out, int32_t* flags, void* scratch,
               void* stream);
/* dL/dY of dadmm_loss for the upstream gradients gout = (dL/dloss_mean, dL/dloss_final) (device
 * [2]): dY[k] = (gout[0]/K + [k == K-1] gout[1]) * 2 (Y[k] - label) / (B P n), 0 in padding
 * columns and when the fallback fired (flags from dadmm_loss). dY: [K][B*P][n_store]. */
int dadmm_loss_grad(int32_t K, int32_t B, int32_t P, int32_t n, int32_t n_store, const float* Y,
                    const float* label, const int32_t* flags, const float* gout, float* dY,
                    void* stream);

/* ---- GNN hypernetwork, inference mode ---------------------------------------------------------
 * GNNHypernetwork3 + decoder + fc of DLASSO_GNNHyp3_Progressive (gnn_dlasso_models_progressive.py
 * :9-72, :93-123, :165-196) for model.eval() (Dropout = identity, BatchNorm on running
 * statistics), batched over all B samples: one launch per layer instead of the reference's
 * per-sample torch_geometric loop (:37-40). All operands are device fp32, row-major:
 *   x1 / x2: the input rows, columns [0, K1) from x1 (row stride ld1), [K1, K) from x2 (row stride
 *            ld2) — the cat(AtAy, Atb) of :165 without materialising it; K1 == K: x1 only;
 *   W [N][K], bias [N]: nn.Linear / GCNConv.lin parameters;  y: row stride ldy.
 * K, K1, ld1, ld2 multiples of 4 (K1 a multiple of 16 when K1 < K); x1, x2, W 16-byte aligned. f32 MFMA (exact f32 products and
 * sums, summed in a fixed order that differs from torch's GEMMs: results agree to f32 rounding).
 *
 * dadmm_hyper_gcn: GCNConv(K -> N) -> leaky_relu(slope) -> BatchNorm1d (eval) for B samples of P
 *   nodes (rows b*P + p): y = BN(leaky(A_hat[b] (x W^T) + bias)); ahat [B or 1][P][P] is
 *   D^-1/2 (Adj + I) D^-1/2 (ahat_per_sample = 0: one graph for every sample).
 *   Replaces: GCNConv + F.leaky_relu + self.bn_i of graph_conv (:52-68), per sample.
 * dadmm_hyper_linear: y = x W^T + bias (bias nullable). Replaces: the decoder's nn.Linear (:94-104).
 * dadmm_hyper_rownorm: y = LayerNorm(x) over C columns (biased variance), then LeakyReLU(slope)
 *   when act != 0. Replaces: self.norm (:69) and the decoder's LayerNorm + LeakyReLU pairs.
 *   C % 4 == 0, C <= 2048.
 * dadmm_hyper_head: hyp [B][4][H] = (sigmoid(x W^T + bias) clamped to [1e-4, 0.9999]) * max_c,
 *   then clamped to <= 0.9999 for c = tau, rho, eta; W [4H][K]. Replaces: fc, sigmoid, clamp and
 *   the alpha/tau/rho/eta scaling of :167-196 (hyp is the reference's h.view(B, 4, H)). */
int dadmm_hyper_gcn(int32_t B, int32_t P, int32_t K, int32_t N, const float* x1, int32_t ld1,
                    int32_t K1, const float* x2, int32_t ld2, const float* W, const float* bias,
                    const float* ahat, int32_t ahat_per_sample, const float* bn_mean,
                    const float* bn_var, const float* bn_weight, const float* bn_bias, float bn_eps,
                    float slope, float* y, int32_t ldy, void* stream);
/* dadmm_hyper_gcn_ex: the same GCN layer on x [B*P][K] (row stride ldx) with a column slice of
 *   the weight (W [N][ldw], ldw >= K: e.g. GCNConv.lin.weight + n for the Atb half of layer 1) and an
 *   optional addend [B*P][ld_add] added to the mix before the bias:
 *     raw == 0: y = BN(leaky(A_hat (x W^T) + addend + bias));   raw != 0: y = A_hat (x W^T) + addend
 *   (bias / BatchNorm pointers unused and nullable when raw). Layer 1's input cat(AtAy, Atb) then
 *   splits into a per-iteration GEMM over AtAy and a once-per-forward raw term over Atb, which
 *   does not change between iterations (gnn_dlasso_models_progressive.py:165: Atb is loop-invariant).
 *   Replaces: conv1 of graph_conv (:52-68) on cat(AtAy, Atb) (same value; f32 summation order differs). */
int dadmm_hyper_gcn_ex(int32_t B, int32_t P, int32_t K, int32_t N, const float* x, int32_t ldx,
                       const float* W, int32_t ldw, const float* addend, int32_t ld_add, const float* bias,
                       const float* ahat, int32_t ahat_per_sample, const float* bn_mean,
                       const float* bn_var, const float* bn_weight, const float* bn_bias, float bn_eps,
                       float slope, int32_t raw, float* y, int32_t ldy, void* stream);
int dadmm_hyper_linear(int32_t rows, int32_t K, int32_t N, const float* x1, int32_t ld1,
                       int32_t K1, const float* x2, int32_t ld2, const float* W, const float* bias,
                       float* y, int32_t ldy, void* stream);
/* dadmm_hyper_linear with y = addend + (x W^T + bias) in the epilogue (ABI 16; addend [rows][ld_add],
 * nullable, may alias y: each element is read before it is written by the same lane). */
int dadmm_hyper_linear_ex(int32_t rows, int32_t K, int32_t N, const float* x1, int32_t ld1, int32_t K1,
                          const float* x2, int32_t ld2, const float* W, const float* bias, const float* addend,
                          int32_t ld_add, float* y, int32_t ldy, void* stream);
int dadmm_hyper_rownorm(int32_t rows, int32_t C, const float* x, const float* weight,
                        const float* bias, float eps, int32_t act, float slope, float* y,
                        void* stream);
int dadmm_hyper_head(int32_t B, int32_t K, int32_t H, const float* x, int32_t ldx, const float* W,
                     const float* bias, float alpha_max, float tau_max, float rho_max,
                     float eta_max, float* hyp, void* stream);
/* dadmm_hyper_linear_ln: y [rows][N] = LeakyReLU?(LayerNorm(x W^T + bias)) — one decoder block
 *   (Linear -> Dropout(eval) -> LayerNorm -> LeakyReLU, :94-105) as a split-K GEMM whose partial
 *   sums (scratch: dadmm_hyper_linear_ln_scratch_bytes, 16-byte aligned) the LayerNorm launch adds
 *   in a fixed order (deterministic). N % 4 == 0, N <= 2048. */
size_t dadmm_hyper_linear_ln_scratch_bytes(int32_t rows, int32_t K, int32_t N);
int dadmm_hyper_linear_ln(int32_t rows, int32_t K, int32_t N, const float* x, int32_t ldx,
                          const float* W, const float* bias, const float* ln_weight,
                          const float* ln_bias, float eps, int32_t act, float slope, float* y,
                          void* scratch, void* stream);

/* dadmm_hyper_linear_gcn_bwd (ABI 17): dadmm_hyper_gcn_train_bwd(dy = x W^T) in ONE launch — the
 * input-gradient GEMM of GCN layer i + 1 (x = its dZ [B P][K], W = its weight transposed, [N][K])
 * with layer i's GCN block backward (leaky_relu, per-sample BatchNorm, Dropout, the A_hat mix) in
 * the epilogue: the GEMM's row tiles hold whole samples, so dy never goes to memory. dz, part and
 * every argument after W mean what they mean for dadmm_hyper_gcn_train_bwd; results are
 * bit-identical to dadmm_hyper_linear + dadmm_hyper_gcn_train_bwd. N % 4 == 0, dz 16-byte aligned.
 * Replaces the pair that follows each of gnn_dlasso_models_progressive.py:52-68's conv_{i+1}
 * blocks in torch's backward. */
int dadmm_hyper_linear_gcn_bwd(int32_t B, int32_t P, int32_t K, int32_t N, const float* x, int32_t ldx,
                               const float* W, const float* m, const float* mean, const float* var,
                               const float* bn_weight, float bn_eps, const float* ahat, int32_t ahat_per_sample,
                               float slope, float drop_p, uint64_t seed, int32_t site, float* dz, float* part,
                               int32_t bn_eval, void* stream);
/* dadmm_hyper_head_train (ABI 17): dadmm_hyper_head that also writes the logits z = x fc^T + f
 * [B][4H] (the training forward's saved activation for dadmm_hyper_head_act's backward) — the
 * training forward's fc and head activation in one launch; hyp bit-identical to
 * dadmm_hyper_linear + dadmm_hyper_head_act(mode 0). */
int dadmm_hyper_head_train(int32_t B, int32_t K, int32_t H, const float* x, int32_t ldx, const float* W,
                           const float* bias, float alpha_max, float tau_max, float rho_max, float eta_max,
                           float* z, float* hyp, void* stream);
/* ---- GNN hypernetwork, training mode ---------------------------------------------------------
 * The same hypernetwork with model.train() semantics (gnn_dlasso_models_progressive.py:52-72:
 * Dropout(0.1) active, BatchNorm1d on each sample's own batch statistics over its P nodes) and the
 * pieces of its backward (dW = dZ^T X on dadmm_hyper_wgrad, dX = dZ W on dadmm_hyper_linear with
 * the transposed weight; no hipBLASLt). Dropout masks come from a counter-based stream: element (row, col) of dropout site
 * `site` is kept iff hash(seed, site, row, col) >= drop_p * 2^32 (drop_hash in the sources); the
 * backward regenerates them. Results agree with torch's autograd of the same modules (given the
 * same masks) to f32 rounding; the reference's own dropout draws are not reproducible anywhere.
 *
 * dadmm_hyper_gcn_train: y = Dropout_p(BN_batch(leaky(A_hat (x W^T) + bias))) per sample; saves
 *   m_out [B*P][N] = A_hat (x W^T) + bias and the per-sample mean_out / var_out [B][N] (biased
 *   variance: the normalisation; the caller updates the running statistics). P >= 2, N % 4 == 0.
 *   Replaces: GCNConv + F.leaky_relu + bn_i (train) + self.dropout of graph_conv (:52-68).
 *   ABI 17: with bn_running_mean / bn_running_var (both non-NULL, [N]) the BatchNorm is the eval-mode
 *   one (running statistics; they are written to mean_out / var_out per sample for the backward):
 *   the layer of model.eval() with autograd (gnn_dlasso_models_progressive.py:52-68, eval).
 * dadmm_hyper_gcn_train_bwd: from dy [B*P][N] (gradient of that y) to dz [B*P][N] (gradient of
 *   x W^T), and part [3][B][N]: per-sample sums of dgamma, dbeta and d(GCNConv.bias). bn_eval:
 *   mean / var are constants (running statistics): dx = gamma rstd dy, no batch-statistics terms.
 * dadmm_hyper_linear_ln_train: one decoder block Linear -> Dropout_p -> LayerNorm -> LeakyReLU?
 *   (:94-105) in train mode; xd [rows][N] = the LayerNorm input (post-dropout), for the backward.
 * dadmm_hyper_rownorm_bwd: backward of LayerNorm (+ LeakyReLU when act) rows from their input xd:
 *   dx w.r.t. the pre-dropout values when drop_p > 0 (same seed / site as the forward), part =
 *   [ceil(rows / 8)][2][C] block partial sums of dweight, dbias (dadmm_hyper_rownorm_bwd_part_bytes).
 * dadmm_hyper_head_act: mode 0: hyp [B][4H] = head(z) for the fc logits z (sigmoid, clamp
 *   [1e-4, 0.9999], * max_c, clamp <= 0.9999 for tau / rho / eta: :167-196); mode 1: out = dz =
 *   dhyp * head'(z). */
int dadmm_hyper_gcn_train(int32_t B, int32_t P, int32_t K, int32_t N, const float* x1, int32_t ld1,
                          int32_t K1, const float* x2, int32_t ld2, const float* W, const float* bias,
                          const float* ahat, int32_t ahat_per_sample, const float* bn_weight,
                          const float* bn_bias, float bn_eps, float slope, float drop_p, uint64_t seed,
                          int32_t site, float* y, int32_t ldy, float* m_out, float* mean_out,
                          float* var_out, const float* bn_running_mean, const float* bn_running_var,
                          void* stream);
int dadmm_hyper_gcn_train_bwd(int32_t B, int32_t P, int32_t N, const float* dy, const float* m,
                              const float* mean, const float* var, const float* bn_weight,
                              float bn_eps, const float* ahat, int32_t ahat_per_sample, float slope,
                              float drop_p, uint64_t seed, int32_t site, float* dz, float* part,
                              int32_t bn_eval, void* stream);
int dadmm_hyper_linear_ln_train(int32_t rows, int32_t K, int32_t N, const float* x, int32_t ldx,
                                const float* W, const float* bias, const float* ln_weight,
                                const float* ln_bias, float eps, int32_t act, float slope, float drop_p,
                                uint64_t seed, int32_t site, float* y, float* xd, void* scratch,
                                void* stream);
size_t dadmm_hyper_rownorm_bwd_part_bytes(int32_t rows, int32_t C);
int dadmm_hyper_rownorm_bwd(int32_t rows, int32_t C, const float* dy, const float* xd,
                            const float* weight, const float* bias, float eps, int32_t act,
                            float slope, float drop_p, uint64_t seed, int32_t site, float* dx,
                            float* part, void* stream);
int dadmm_hyper_head_act(int32_t mode, int32_t B, int32_t H, const float* z, const float* dhyp,
                         float alpha_max, float tau_max, float rho_max, float eta_max, float* out,
                         void* stream);
/* dadmm_hyper_bn_running_update (ABI 17): the BatchNorm1d running statistics of `layers` (<= 8)
 * layers after T = iters * B sequential train-mode calls over P nodes each (the reference calls
 * bn_i once per sample, gnn_dlasso_models_progressive.py:52-68), in closed form and float64:
 *   r <- decay r + sum_t weights[t] s_t   (decay = (1 - m)^T, weights[t] = m (1 - m)^(T - 1 - t)),
 * s_t the sample's batch mean, resp. its biased variance times P / (P - 1); one pass of partial
 * sums and one finishing pass for every layer (it replaces ~16 torch launches per layer).
 * widths / running_mean / running_var / tracked / mean / var are HOST arrays of `layers` entries
 * (the latter five device pointers; tracked nullable: num_batches_tracked += T). mean[i] / var[i]:
 * [iters][B][widths[i]] with block_stride floats between iterations. scratch: at least
 * dadmm_hyper_bn_running_scratch_bytes bytes (8-byte aligned). */
size_t dadmm_hyper_bn_running_scratch_bytes(int32_t layers, const int32_t* widths, int32_t iters,
                                            int32_t B);
int dadmm_hyper_bn_running_update(int32_t layers, const int32_t* widths, float* const* running_mean,
                                  float* const* running_var, int64_t* const* tracked,
                                  const float* const* mean, const float* const* var,
                                  int64_t block_stride, int32_t iters, int32_t B, int32_t P,
                                  const double* weights, double decay, void* scratch, void* stream);

/* ---- GNN hypernetwork training: parameter gradients on hand-written kernels ------------------
 * Replace the weight / bias gradients torch's autograd computes through hipBLASLt and its sums
 * (gnn_dlasso_progressive.py:207-214 loss_final.backward() through the hypernetwork of
 * gnn_dlasso_models_progressive.py:9-72, :93-123), accumulated in place in a fixed order.
 * dadmm_hyper_wgrad: g [N][K] (+)= dZ^T X over R rows (f32 MFMA); X = cat of x1 (columns < K1,
 *   leading dimension ld1) and x2 (the other K - K1 columns, ld2); gbias [N] (+)= column sums of dZ
 *   (nullable); beta = 1 accumulates. scratch: dadmm_hyper_wgrad_scratch_bytes (0: none needed;
 *   16-byte aligned).
 * dadmm_hyper_colsum: out [G][C] (+)= sum_r part [G][R][C] (the per-block partials of
 *   dadmm_hyper_gcn_train_bwd / dadmm_hyper_rownorm_bwd), rows in order.
 * dadmm_hyper_transpose: out [cols][rows] = in [rows][cols] (the weights of the input-gradient
 *   GEMMs dX = dZ W, run as dadmm_hyper_linear with W^T). */
size_t dadmm_hyper_wgrad_scratch_bytes(int32_t R, int32_t N, int32_t K);
int dadmm_hyper_wgrad(int32_t R, int32_t N, int32_t K, const float* dz, int32_t ldz, const float* x1,
                      int32_t ld1, int32_t K1, const float* x2, int32_t ld2, float* g, float* gbias,
                      int32_t beta, void* scratch, void* stream);
int dadmm_hyper_colsum(const float* part, int32_t G, int32_t R, int32_t C, float* out, int32_t beta,
                       void* stream);
int dadmm_hyper_transpose(int32_t rows, int32_t cols, const float* in, float* out, void* stream);

/* ---- GNN hypernetwork training: one call per iteration (host orchestration in the library) ----
 * dadmm_hyper_train_forward runs the whole training-mode hypernetwork of one iteration
 * (gnn_dlasso_models_progressive.py:165-196 with :52-72 in train mode: 5 GCN blocks, LayerNorm,
 * 3 decoder blocks, fc, head) and stores its activations in `sv` (caller-allocated, 16-byte
 * aligned); dadmm_hyper_train_backward runs its backward from d hyp, ACCUMULATES (+=) every
 * parameter gradient into `g` (contiguous groups as the partial sums come: [bn.weight | bn.bias |
 * conv.bias], [LayerNorm weight | bias]) and writes the first n columns of d AtAy (row stride
 * net->ld). `work`: dadmm_hyper_train_work_bytes (16-byte aligned), shared by both and by one
 * stream at a time. The dropout
 * masks of both come from `seed` (the same value for an iteration's forward and backward).
 * Requires P >= 2, n % 16 == 0 and widths that are multiples of 4 (else DADMM_EINVAL /
 * DADMM_EUNSUPPORTED: the caller runs the per-kernel entry points above). */
typedef struct dadmm_hyper_net {
    int32_t P, n, ld;           /* agents; signal length; row stride of AtAy / Atb / dAtAy       */
    int32_t width[5];           /* GCNConv output widths (h, 2h, 4h, 4h, 4h)                     */
    int32_t dec_width[3];       /* decoder Linear output widths (4h, 2h, h)                      */
    int32_t H;                  /* P ('diff') or 1 ('same'): fc outputs 4H                       */
    const float* conv_w[5];     /* [width_i][width_{i-1}] (layer 1: [width_0][2n])               */
    const float* conv_b[5];
    const float* bn_w[5];
    const float* bn_b[5];
    float bn_eps[5];
    const float* norm_w;
    const float* norm_b;
    float norm_eps;
    const float* dec_w[3];
    const float* dec_b[3];
    const float* ln_w[3];
    const float* ln_b[3];
    float ln_eps[3], dec_slope[3], dec_drop[3];
    const float* fc_w;
    const float* fc_b;
    float drop_enc;             /* the encoder's Dropout p                                        */
    float maxv[4];              /* alpha_max, tau_max, rho_max, eta_max                           */
    /* ABI 17: bn_eval != 0 runs the same kernels with the module in eval mode (a backward of
     * model.eval() under autograd): every BatchNorm normalises with its running statistics
     * bn_rm / bn_rv [width_i] instead of the sample's batch statistics (which the saved
     * mean / var slices then hold, per sample), and the caller sets every dropout p to 0.     */
    const float* bn_rm[5];
    const float* bn_rv[5];
    int32_t bn_eval;
} dadmm_hyper_net;
typedef struct dadmm_hyper_saved {
    float* y[5];                /* [B*P][width_i] block outputs                                   */
    float* m[5];                /* [B*P][width_i] pre-activation mixes                            */
    float* mean[5];             /* [B][width_i] batch statistics                                  */
    float* var[5];
    float* e;                   /* [B*P][width_4] LayerNorm output = decoder input                */
    float* dec_y[3];            /* [B][dec_width_j] block outputs                                 */
    float* dec_xd[3];           /* [B][dec_width_j] LayerNorm inputs (after Dropout)              */
    float* z;                   /* [B][4H] fc logits                                              */
    float* hyp;                 /* [B][4][H] the iteration's (alpha, tau, rho, eta)               */
} dadmm_hyper_saved;
typedef struct dadmm_hyper_grads {
    float* conv_w[5];
    float* bn_wbc[5];           /* [3][width_i]: bn.weight, bn.bias, conv.bias                    */
    float* norm_wb;             /* [2][width_4]                                                   */
    float* dec_w[3];
    float* dec_b[3];
    float* ln_wb[3];            /* [2][dec_width_j]                                               */
    float* fc_w;
    float* fc_b;
    const float* conv_wt[5];    /* transposed weights (dadmm_hyper_transpose) for dX = dZ W       */
    const float* dec_wt[3];
    const float* fc_wt;
} dadmm_hyper_grads;
size_t dadmm_hyper_train_work_bytes(const dadmm_hyper_net* net, int32_t B);
int dadmm_hyper_train_forward(const dadmm_hyper_net* net, int32_t B, const float* AtAy, const float* Atb,
                              const float* ahat, int32_t ahat_per_sample, uint64_t seed,
                              const dadmm_hyper_saved* sv, void* work, void* stream);
/* ABI 17: layer 1's input is cat(AtAy_k, Atb) (:165) and Atb does not change between the
 * iterations of a forward, so its half of the GCNConv, A_hat (Atb W1[:, n:]^T) [B*P][width_0], is
 * formed once per forward (dadmm_hyper_train_atb_mix) and dadmm_hyper_train_forward_ex adds it to
 * layer 1's mix before the bias, running that GEMM over AtAy alone (half the depth). atb_mix NULL:
 * dadmm_hyper_train_forward. The backward and the weight gradients read AtAy and Atb as before. */
int dadmm_hyper_train_atb_mix(const dadmm_hyper_net* net, int32_t B, const float* Atb, const float* ahat,
                              int32_t ahat_per_sample, float* out, void* stream);
int dadmm_hyper_train_forward_ex(const dadmm_hyper_net* net, int32_t B, const float* AtAy, const float* Atb,
                                 const float* atb_mix, const float* ahat, int32_t ahat_per_sample, uint64_t seed,
                                 const dadmm_hyper_saved* sv, void* work, void* stream);
int dadmm_hyper_train_backward(const dadmm_hyper_net* net, int32_t B, const float* AtAy, const float* Atb,
                               const float* ahat, int32_t ahat_per_sample, uint64_t seed,
                               const dadmm_hyper_saved* sv, const float* dhyp, const dadmm_hyper_grads* g,
                               float* dAtAy, void* work, void* stream);
/* Deferred parameter gradients (round 4): dadmm_hyper_train_backward_deferred is the same backward
 * of one iteration, except that instead of accumulating the parameter gradients it writes their
 * operands (every layer's dZ and the normalisation partial sums) into `dsave`, one block of
 * dadmm_hyper_train_dsave_floats(net, B) floats per iteration (16-byte aligned); the input
 * gradients (dX, d AtAy) are computed as before. After the last (reverse) iteration,
 * dadmm_hyper_train_wgrad accumulates (+=) the parameter gradients of all `iters` iterations into
 * `g` at once — one batched weight-gradient GEMM per linear, one batched column sum per
 * normalisation — reading iteration k's activations at sv0 + k sv_stride floats (the saved
 * blocks of dadmm_hyper_train_forward, equally spaced), its gradient operands at
 * dsave + k dsave_stride and its AtAy at AtAy + k atay_stride (Atb shared). Replaces ~19
 * launches per iteration by ~19 in all (gnn_dlasso_progressive.py:207-214's backward at small
 * batches is bound by launches, not by work). */
/* accumulate, bit 0 (ABI 16): dAtAy += the input gradient (the adjoint's running AtAy gradient,
 * added in the last linear's epilogue: the same bits as writing it and adding after); clear:
 * dAtAy = it. Bit 1 (ABI 17): the head's logit gradient is already in the iteration's dsave block
 * (its first [B][4H] floats, written by dadmm_gnn_step_backward_ex's head epilogue): dhyp is not
 * read (may be NULL) and the head's backward launch is skipped. */
size_t dadmm_hyper_train_dsave_floats(const dadmm_hyper_net* net, int32_t B);
int dadmm_hyper_train_backward_deferred(const dadmm_hyper_net* net, int32_t B, const float* AtAy,
                                        const float* Atb, const float* ahat, int32_t ahat_per_sample,
                                        uint64_t seed, const dadmm_hyper_saved* sv, const float* dhyp,
                                        const dadmm_hyper_grads* g, float* dAtAy, void* work, float* dsave,
                                        int32_t accumulate, void* stream);
int dadmm_hyper_train_wgrad(const dadmm_hyper_net* net, int32_t B, int32_t iters, const float* AtAy,
                            int64_t atay_stride, const float* Atb, const dadmm_hyper_saved* sv0,
                            int64_t sv_stride, const float* dsave, int64_t dsave_stride,
                            const dadmm_hyper_grads* g, void* scratch, void* stream);
/* Row-split scratch of dadmm_hyper_train_wgrad (ABI 14): with `scratch` of at least this many bytes
 * (16-byte aligned) each weight gradient's rows spread over several workgroups per output tile and
 * the partials are added in a fixed order (deterministic); with scratch == NULL one workgroup walks
 * every row of its tile. The scratch also holds the normalisation-parameter sums' per-iteration
 * block sums (iters > 1), which are then added in iteration order: deterministic, but rounded in a
 * different order than with scratch == NULL (f32 rounding). */
size_t dadmm_hyper_train_wgrad_scratch_bytes(const dadmm_hyper_net* net, int32_t B, int32_t iters);

#ifdef __cplusplus
}
#endif

#endif /* DADMM_H_ */
