// dadmm_abi.cpp — the extern "C" boundary declared in include/dadmm.h.
//
// Validates arguments, picks the compiled kernel configuration and enqueues it. No allocation,
// no synchronisation, no global mutable state (the error message is thread-local), so every
// entry point can be captured into a hipGraph by the caller.

#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/dadmm.h"
#include "dadmm_internal.h"

namespace {

thread_local char g_err[512] = "";

int fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

int ok() {
    g_err[0] = '\0';
    return DADMM_OK;
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

int check_dims(const dadmm_dims* d) {
    if (d == nullptr) return fail(DADMM_EINVAL, "dims is NULL");
    if (d->B < 0 || d->P < 1 || d->m < 1 || d->n < 1 || d->K < 0)
        return fail(DADMM_EINVAL, "bad dims B=%d P=%d m=%d n=%d K=%d", d->B, d->P, d->m, d->n,
                    d->K);
    // visit lists carry uint8 agent ids; the uint64 neighbour masks (fused kernels, P <= 6) are
    // only read for the shapes the fused kernels serve
    if (d->P > 255) return fail(DADMM_EINVAL, "P=%d > 255 agents does not fit the uint8 visit-list ids", d->P);
    if (d->variant != DADMM_VARIANT_UNFOLDED && d->variant != DADMM_VARIANT_GNN)
        return fail(DADMM_EINVAL, "unknown variant %d", d->variant);
    if (d->hyp_rows != 1 && d->hyp_rows != d->P)
        return fail(DADMM_EINVAL, "hyp_rows=%d must be 1 ('same') or P=%d ('diff')", d->hyp_rows,
                    d->P);
    if (d->graph_shared != 0 && d->graph_shared != 1)
        return fail(DADMM_EINVAL, "graph_shared must be 0 or 1");
    return DADMM_OK;
}

int n_pad_of(const dadmm_dims* d) { return 64 * dadmm::fused_nt(d->n); }
int m_pad_of(const dadmm_dims* d) { return dadmm::m_pad_of(d->m); }

int check_m(const dadmm_dims* d) {
    if (d->m > dadmm::M_MAX)
        return fail(DADMM_EUNSUPPORTED, "m=%d > %d rows per agent", d->m, dadmm::M_MAX);
    return DADMM_OK;
}

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace

extern "C" {

int dadmm_abi_version(void) { return DADMM_ABI_VERSION; }

const char* dadmm_last_error(void) { return g_err; }

size_t dadmm_operator_bytes(const dadmm_dims* d) {
    if (check_dims(d) != DADMM_OK) return 0;
    if (check_m(d) != DADMM_OK) return 0;
    return 2 * sizeof(float) * (size_t)d->P * m_pad_of(d) * (size_t)n_pad_of(d);
}

int dadmm_prepare_operator(const dadmm_dims* d, const float* A, void* op, void* stream) {
    int rc = check_dims(d);
    if (rc) return rc;
    if (A == nullptr || op == nullptr) return fail(DADMM_EINVAL, "A/op is NULL");
    if (!aligned16(op)) return fail(DADMM_EINVAL, "op workspace must be 16-byte aligned");
    if ((rc = check_m(d)) != DADMM_OK) return rc;
    const int np = n_pad_of(d);
    float* Apad = (float*)op;
    float* Atpad = Apad + (size_t)d->P * m_pad_of(d) * np;
    hipError_t e = dadmm::launch_prepare(A, Apad, Atpad, d->P, d->m, d->n, np, (hipStream_t)stream);
    if (e != hipSuccess) return fail(DADMM_EHIP, "prepare launch: %s", hipGetErrorString(e));
    return ok();
}

}  // extern "C"

namespace {

// shape checks shared by the fused forward (plain / recording) and the fused adjoint; on success
// *graph and *nt select the compiled configuration
int check_fused_shape(const dadmm_dims* d, const uint32_t* nbr_order, int* graph, int* nt) {
    if (d->m > dadmm::M_PAD)   // the fused kernels hold one m-group of R on chip
        return fail(DADMM_EUNSUPPORTED, "m=%d > %d rows per agent: not a fused shape", d->m,
                    dadmm::M_PAD);
    if ((d->n & 3) != 0)
        return fail(DADMM_EUNSUPPORTED, "n=%d: the fused kernel needs n %% 4 == 0 (zero-pad n)", d->n);
    if ((size_t)d->B * d->P * d->n * 4 >= ((size_t)1 << 31))
        return fail(DADMM_EUNSUPPORTED, "B*P*n*4 >= 2^31 bytes per iterate (split the batch)");
    if (nbr_order != nullptr && d->graph_shared)
        return fail(DADMM_EINVAL, "nbr_order needs per-sample graphs (graph_shared = 0)");
    if (nbr_order != nullptr && d->P > 8)
        return fail(DADMM_EINVAL, "nbr_order packs 4-bit agent ids: P <= 8");
    *nt = dadmm::fused_nt(d->n);
    *graph = d->graph_shared ? dadmm::GRAPH_SHARED
                             : (nbr_order ? dadmm::GRAPH_ORDERED : dadmm::GRAPH_LANE);
    return DADMM_OK;
}

int forward_impl(const dadmm_dims* d, const void* op, const float* b, const uint64_t* nbr,
                 const uint32_t* nbr_order, const float* deg, const float* hyp, const float* y0,
                 const float* U0, const float* d0, float* Y, float* Grec, float* Urec,
                 float* U_out, int32_t* status, void* stream, bool rec) {
    int rc = check_dims(d);
    if (rc) return rc;
    if (d->B == 0 || d->K == 0) return ok();
    if (rec && (Grec == nullptr || Urec == nullptr || !aligned16(Grec) || !aligned16(Urec)))
        return fail(DADMM_EINVAL, "Grec and Urec must be non-NULL and 16-byte aligned");
    if (!op || !b || !nbr || !deg || !hyp || !y0 || !U0 || !d0 || !Y)
        return fail(DADMM_EINVAL, "a required pointer is NULL");
    if (!aligned16(op)) return fail(DADMM_EINVAL, "op workspace must be 16-byte aligned");
    if (!aligned16(Y) || !aligned16(y0) || !aligned16(U0) || !aligned16(d0) ||
        (U_out != nullptr && !aligned16(U_out)))
        return fail(DADMM_EINVAL, "Y, y0, U0, d0 and U_out must be 16-byte aligned");
    int graph = 0, nt = 0;
    if ((rc = check_fused_shape(d, nbr_order, &graph, &nt)) != DADMM_OK) return rc;
    dadmm::fused_fn_ptr fn = rec ? dadmm::find_fused_rec(d->P, nt, graph) : dadmm::find_fused(d->P, nt, graph);
    if (fn == nullptr)
        return fail(DADMM_EUNSUPPORTED, "no fused kernel for P=%d n=%d (n_pad=%d)", d->P, d->n,
                    64 * nt);
    const int np = 64 * nt;
    dadmm::FusedArgs a;
    a.A = (const float*)op;
    a.At = a.A + (size_t)d->P * m_pad_of(d) * np;
    a.b = b;
    a.nbr = nbr;
    a.nbr_order = nbr_order;
    a.deg = deg;
    a.hyp = hyp;
    a.y0 = y0;
    a.U0 = U0;
    a.d0 = d0;
    a.Y = Y;
    a.U_out = U_out;
    a.status = status;
    a.Grec = Grec;
    a.Urec = Urec;
    a.B = d->B;
    a.m = d->m;
    a.n = d->n;
    a.K = d->K;
    a.hyp_rows = d->hyp_rows;
    a.variant = d->variant;
    hipError_t e = fn(a, (hipStream_t)stream);
    if (e != hipSuccess) return fail(DADMM_EHIP, "fused launch: %s", hipGetErrorString(e));
    return ok();
}

}  // namespace

extern "C" {

int dadmm_forward(const dadmm_dims* d, const void* op, const float* b, const uint64_t* nbr,
                  const uint32_t* nbr_order, const float* deg, const float* hyp, const float* y0,
                  const float* U0, const float* d0, float* Y, float* U_out, int32_t* status,
                  void* stream) {
    return forward_impl(d, op, b, nbr, nbr_order, deg, hyp, y0, U0, d0, Y, nullptr, nullptr, U_out,
                        status, stream, false);
}

int dadmm_forward_record(const dadmm_dims* d, const void* op, const float* b, const uint64_t* nbr,
                         const uint32_t* nbr_order, const float* deg, const float* hyp,
                         const float* y0, const float* U0, const float* d0, float* Y, float* Grec,
                         float* Urec, float* U_out, int32_t* status, void* stream) {
    return forward_impl(d, op, b, nbr, nbr_order, deg, hyp, y0, U0, d0, Y, Grec, Urec, U_out,
                        status, stream, true);
}

// ---- the column-split forward (dadmm_split.hip) ----------------------------------------------
namespace {
int device_cus() {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
        cus = 256;
    return cus;
}
struct SplitPlan {
    int nt = 0, slices = 0, groups = 0, tiles = 0;
    size_t flag_bytes = 0, bytes = 0;
};
// groups = 0: the split path does not serve d (shape, or a batch that fills more than half the CUs)
SplitPlan split_plan(const dadmm_dims* d) {
    SplitPlan sp;
    if (d == nullptr || d->B <= 0 || d->K <= 0 || d->P < 1 || d->P > 6 || d->m < 1 ||
        d->m > dadmm::M_PAD || d->n < 1 || (d->n & 3) != 0 || d->hyp_rows < 1)
        return sp;
    if ((size_t)d->B * d->P * d->n * 4 >= ((size_t)1 << 31)) return sp;
    const int nt = dadmm::fused_nt(d->n);
    if (nt != 2 && nt != 4) return sp;
    const int cus = device_cus();
    const int tiles = (d->B + dadmm::BT - 1) / dadmm::BT;
    if (2 * tiles > cus) return sp;
    const int S = 64 * nt / dadmm::SPLIT_COLS;
    int groups = cus / S;
    groups = groups < tiles ? groups : tiles;
    if (groups < 1) return sp;
    sp.nt = nt;
    sp.slices = S;
    sp.groups = groups;
    sp.tiles = tiles;
    sp.flag_bytes = ((size_t)groups * d->P * 4 * S * 4 + 4 + 255) / 256 * 256;
    sp.bytes = (size_t)groups * 2 * d->P * 4 * S * 1024;
    return sp;
}
}  // namespace

size_t dadmm_split_scratch_bytes(const dadmm_dims* d) {
    if (d == nullptr || check_dims(d) != DADMM_OK) return 0;
    return split_plan(d).bytes;
}

size_t dadmm_split_flag_bytes(const dadmm_dims* d) {
    if (d == nullptr || check_dims(d) != DADMM_OK) return 0;
    return split_plan(d).flag_bytes;
}

int dadmm_forward_split(const dadmm_dims* d, const void* op, const float* b, const uint64_t* nbr,
                        const uint32_t* nbr_order, const float* deg, const float* hyp,
                        const float* y0, const float* U0, const float* d0, float* Y, float* U_out,
                        int32_t* status, void* flags, void* scratch, void* stream) {
    int rc = check_dims(d);
    if (rc) return rc;
    if (d->B == 0 || d->K == 0) return ok();
    if (!op || !b || !nbr || !deg || !hyp || !y0 || !U0 || !d0 || !Y || !flags || !scratch)
        return fail(DADMM_EINVAL, "a required pointer is NULL");
    if (!aligned16(op) || !aligned16(Y) || !aligned16(y0) || !aligned16(U0) || !aligned16(d0) ||
        !aligned16(flags) || !aligned16(scratch) || (U_out != nullptr && !aligned16(U_out)))
        return fail(DADMM_EINVAL, "op, Y, y0, U0, d0, U_out, flags and scratch must be 16-byte aligned");
    int graph = 0, nt = 0;
    if ((rc = check_fused_shape(d, nbr_order, &graph, &nt)) != DADMM_OK) return rc;
    const SplitPlan sp = split_plan(d);
    if (sp.groups == 0)
        return fail(DADMM_EUNSUPPORTED, "the column-split forward does not serve B=%d P=%d n=%d "
                    "(n_pad 128 or 256, P <= 6, ceil(B/16) <= CUs/2)", d->B, d->P, d->n);
    dadmm::split_fn_ptr fn = dadmm::find_split(d->P, nt, graph);
    if (fn == nullptr)
        return fail(DADMM_EUNSUPPORTED, "no split kernel for P=%d n_pad=%d", d->P, 64 * nt);
    const int np = 64 * nt;
    dadmm::SplitArgs sa;
    dadmm::FusedArgs& a = sa.f;
    a.A = (const float*)op;
    a.At = a.A + (size_t)d->P * m_pad_of(d) * np;
    a.b = b;
    a.nbr = nbr;
    a.nbr_order = nbr_order;
    a.deg = deg;
    a.hyp = hyp;
    a.y0 = y0;
    a.U0 = U0;
    a.d0 = d0;
    a.Y = Y;
    a.U_out = U_out;
    a.status = status;
    a.Grec = nullptr;
    a.Urec = nullptr;
    a.B = d->B;
    a.m = d->m;
    a.n = d->n;
    a.K = d->K;
    a.hyp_rows = d->hyp_rows;
    a.variant = d->variant;
    sa.xflag = (uint32_t*)flags;
    sa.xbuf = (float*)scratch;
    sa.groups = sp.groups;
    sa.tiles = sp.tiles;
    sa.spin_ticks = 20000000ull;   // 0.2 s at the 100 MHz s_memrealtime clock
    hipError_t e = fn(sa, (hipStream_t)stream);
    if (e != hipSuccess) return fail(DADMM_EHIP, "split launch: %s", hipGetErrorString(e));
    return ok();
}

size_t dadmm_backward_scratch_bytes(const dadmm_dims* d) {
    if (check_dims(d) != DADMM_OK) return 0;
    const size_t nwg = ((size_t)d->B + dadmm::BT - 1) / dadmm::BT;
    const size_t bytes = sizeof(float) * nwg * (size_t)d->K * d->P * 4;
    return bytes > 0 ? bytes : 16;
}

int dadmm_backward(const dadmm_dims* d, const void* op, const uint64_t* nbr,
                   const uint32_t* nbr_order, const float* deg, const float* hyp, const float* y0,
                   const float* d0, const float* Y, const float* Grec, const float* Urec,
                   const float* gY, float* dhyp, void* scratch, void* stream) {
    int rc = check_dims(d);
    if (rc) return rc;
    if (d->K == 0) return ok();
    if (!dhyp) return fail(DADMM_EINVAL, "dhyp is NULL");
    if (d->B == 0) {
        hipError_t e = hipMemsetAsync(dhyp, 0, sizeof(float) * (size_t)d->K * d->hyp_rows * 4,
                                      (hipStream_t)stream);
        if (e != hipSuccess) return fail(DADMM_EHIP, "memset: %s", hipGetErrorString(e));
        return ok();
    }
    if (!op || !nbr || !deg || !hyp || !y0 || !d0 || !Y || !Grec || !Urec || !gY || !scratch)
        return fail(DADMM_EINVAL, "a required pointer is NULL");
    if (!aligned16(op) || !aligned16(Y) || !aligned16(y0) || !aligned16(d0) || !aligned16(Grec) ||
        !aligned16(Urec) || !aligned16(gY) || !aligned16(scratch))
        return fail(DADMM_EINVAL, "op, Y, y0, d0, Grec, Urec, gY and scratch must be 16-byte aligned");
    int graph = 0, nt = 0;
    if ((rc = check_fused_shape(d, nbr_order, &graph, &nt)) != DADMM_OK) return rc;
    dadmm::backward_fn_ptr fn = dadmm::find_backward(d->P, nt, graph);
    if (fn == nullptr)
        return fail(DADMM_EUNSUPPORTED, "no adjoint kernel for P=%d n=%d (n_pad=%d)", d->P, d->n,
                    64 * nt);
    const int np = 64 * nt;
    dadmm::BackwardArgs a;
    a.A = (const float*)op;
    a.At = a.A + (size_t)d->P * m_pad_of(d) * np;
    a.nbr = nbr;
    a.nbr_order = nbr_order;
    a.deg = deg;
    a.hyp = hyp;
    a.y0 = y0;
    a.d0 = d0;
    a.Y = Y;
    a.Grec = Grec;
    a.Urec = Urec;
    a.gY = gY;
    a.partial = (float*)scratch;
    a.B = d->B;
    a.m = d->m;
    a.n = d->n;
    a.K = d->K;
    a.hyp_rows = d->hyp_rows;
    a.variant = d->variant;
    hipError_t e = fn(a, (hipStream_t)stream);
    if (e != hipSuccess) return fail(DADMM_EHIP, "adjoint launch: %s", hipGetErrorString(e));
    const int nwg = (d->B + dadmm::BT - 1) / dadmm::BT;
    e = dadmm::launch_backward_reduce(a.partial, dhyp, nwg, d->K, d->P, d->hyp_rows,
                                      (hipStream_t)stream);
    if (e != hipSuccess) return fail(DADMM_EHIP, "adjoint reduce launch: %s", hipGetErrorString(e));
    return ok();
}

size_t dadmm_adjoint_scratch_bytes(const dadmm_dims* d) {
    if (check_dims(d) != DADMM_OK) return 0;
    const size_t state = align256(sizeof(float) * (size_t)d->B * d->P * d->n);
    const size_t part = sizeof(float) * (size_t)dadmm::adjoint_workgroups(d->B, d->n, d->P) * d->K * d->P * 4;
    return 3 * state + align256(part > 0 ? part : 16);
}

int dadmm_adjoint(const dadmm_dims* d, const void* op, const int32_t* visit_ptr,
                  const uint8_t* visit_q, const float* deg, const float* hyp, const float* y0,
                  const float* d0, const float* Y, const float* Grec, const float* Urec,
                  const float* gY, float* dhyp, void* scratch, void* stream) {
    int rc = check_dims(d);
    if (rc) return rc;
    if (d->K == 0) return ok();
    if (!dhyp) return fail(DADMM_EINVAL, "dhyp is NULL");
    if (d->B == 0) {
        hipError_t e = hipMemsetAsync(dhyp, 0, sizeof(float) * (size_t)d->K * d->hyp_rows * 4,
                                      (hipStream_t)stream);
        if (e != hipSuccess) return fail(DADMM_EHIP, "memset: %s", hipGetErrorString(e));
        return ok();
    }
    if (!op || !visit_ptr || !visit_q || !deg || !hyp || !y0 || !d0 || !Y || !Grec || !Urec || !gY ||
        !scratch)
        return fail(DADMM_EINVAL, "a required pointer is NULL");
    if (!aligned16(op) || !aligned16(Y) || !aligned16(y0) || !aligned16(d0) || !aligned16(Grec) ||
        !aligned16(Urec) || !aligned16(gY))
        return fail(DADMM_EINVAL, "op, Y, y0, d0, Grec, Urec and gY must be 16-byte aligned");
    if (((uintptr_t)scratch & 255u) != 0) return fail(DADMM_EINVAL, "scratch must be 256-byte aligned");
    if ((rc = check_m(d)) != DADMM_OK) return rc;
    if ((d->n & 3) != 0) return fail(DADMM_EUNSUPPORTED, "n=%d: needs n %% 4 == 0 (zero-pad n)", d->n);
    if ((size_t)d->B * d->P * d->n * 4 >= ((size_t)1 << 31))   // 32-bit buffer offsets (gram)
        return fail(DADMM_EUNSUPPORTED, "B*P*n*4 >= 2^31 bytes per iterate (split the batch)");
    if (dadmm::adjoint_lds_bytes(d->P) > 160 * 1024 || dadmm::gnn_gram_lds(m_pad_of(d)) > 160 * 1024)
        return fail(DADMM_EUNSUPPORTED, "P=%d / m=%d: the adjoint's LDS tiles do not fit", d->P, d->m);
    const int np = n_pad_of(d);
    const size_t state = align256(sizeof(float) * (size_t)d->B * d->P * d->n);
    char* base = (char*)scratch;
    dadmm::AdjArgs a{};
    a.A = (const float*)op;
    a.At = a.A + (size_t)d->P * m_pad_of(d) * np;
    a.vptr = visit_ptr;
    a.vq = visit_q;
    a.deg = deg;
    a.hyp = hyp;
    a.y0 = y0;
    a.d0 = d0;
    a.Y = Y;
    a.Grec = Grec;
    a.Urec = Urec;
    a.gY = gY;
    a.yb = (float*)base;
    a.Ub = (float*)(base + state);
    a.Gb = (float*)(base + 2 * state);
    a.partial = (float*)(base + 3 * state);
    a.B = d->B;
    a.P = d->P;
    a.m = d->m;
    a.m_pad = m_pad_of(d);
    a.n = d->n;
    a.n_pad = np;
    a.K = d->K;
    a.hyp_rows = d->hyp_rows;
    a.variant = d->variant;
    a.graph_shared = d->graph_shared;
    hipError_t e = dadmm::launch_adjoint(a, dhyp, (hipStream_t)stream);
    if (e != hipSuccess) return fail(DADMM_EHIP, "adjoint launch: %s", hipGetErrorString(e));
    return ok();
}

namespace {

int gnn_common(const dadmm_dims* d, dadmm::GnnArgs* a) {
    int rc = check_dims(d);
    if (rc) return rc;
    if ((rc = check_m(d)) != DADMM_OK) return rc;
    if ((d->n & 3) != 0) return fail(DADMM_EUNSUPPORTED, "n=%d: needs n %% 4 == 0 (zero-pad n)", d->n);
    if ((size_t)d->B * d->P * d->n * 4 >= ((size_t)1 << 31))   // 32-bit buffer offsets (gram)
        return fail(DADMM_EUNSUPPORTED, "B*P*n*4 >= 2^31 bytes per iterate (split the batch)");
    *a = dadmm::GnnArgs{};
    a->B = d->B;
    a->P = d->P;
    a->m = d->m;
    a->m_pad = m_pad_of(d);
    a->n = d->n;
    a->n_pad = n_pad_of(d);
    a->K = d->K;
    a->hyp_rows = d->hyp_rows;
    a->variant = d->variant;
    a->graph_shared = d->graph_shared;
    return DADMM_OK;
}

void set_op(dadmm::GnnArgs* a, const void* op) {
    a->A = (const float*)op;
    a->At = a->A + (size_t)a->P * a->m_pad * a->n_pad;
}

int hip_rc(hipError_t e, const char* what) {
    if (e != hipSuccess) return fail(DADMM_EHIP, "%s: %s", what, hipGetErrorString(e));
    return ok();
}

}  // namespace

size_t dadmm_gnn_flag_bytes(int32_t K) {
    return K < 0 ? 0 : (size_t)GNN_FLAG_WORDS(K) * 4;
}

int dadmm_gnn_begin(const dadmm_dims* d, const void* op, const float* b, const float* y0,
                    const float* U0, float* Atb, int32_t* flags, void* stream) {
    dadmm::GnnArgs a;
    int rc = gnn_common(d, &a);
    if (rc) return rc;
    if (!flags) return fail(DADMM_EINVAL, "flags is NULL");
    if (d->B == 0) return hip_rc(dadmm::gnn_launch_zero(flags, GNN_FLAG_WORDS(d->K), (hipStream_t)stream), "zero launch");
    if (!op || !b || !y0 || !U0 || !Atb) return fail(DADMM_EINVAL, "a required pointer is NULL");
    if (!aligned16(op) || !aligned16(y0) || !aligned16(U0) || !aligned16(Atb))
        return fail(DADMM_EINVAL, "op, y0, U0 and Atb must be 16-byte aligned");
    set_op(&a, op);
    a.b = b;
    a.U = U0;
    a.flags = flags;
    hipError_t e = dadmm::gnn_launch_zero(flags, GNN_FLAG_WORDS(d->K), (hipStream_t)stream);
    if (e != hipSuccess) return hip_rc(e, "zero launch");
    e = dadmm::gnn_launch_check0(a, y0, (hipStream_t)stream);
    if (e != hipSuccess) return hip_rc(e, "check0 launch");
    return hip_rc(dadmm::gnn_launch_gram(a, 0, nullptr, Atb, 1, (hipStream_t)stream), "Atb launch");
}

int dadmm_gnn_gram(const dadmm_dims* d, const void* op, int32_t k, float* const* yptr,
                   const int32_t* flags, const float* x, float* out, void* stream) {
    dadmm::GnnArgs a;
    int rc = gnn_common(d, &a);
    if (rc) return rc;
    if (d->B == 0) return ok();
    if (!op || !out || (x == nullptr && (yptr == nullptr || flags == nullptr)))
        return fail(DADMM_EINVAL, "a required pointer is NULL");
    if (x == nullptr && (k < 0 || k >= d->K)) return fail(DADMM_EINVAL, "k=%d outside [0, K)", k);
    if (!aligned16(op) || !aligned16(out) || (x && !aligned16(x)))
        return fail(DADMM_EINVAL, "op, x and out must be 16-byte aligned");
    if (dadmm::gnn_gram_lds(a.m_pad) > 160 * 1024)
        return fail(DADMM_EUNSUPPORTED, "m=%d too large for the gram tile", d->m);
    set_op(&a, op);
    a.yptr = yptr;
    a.flags = const_cast<int32_t*>(flags);
    return hip_rc(dadmm::gnn_launch_gram(a, k, x, out, 0, (hipStream_t)stream), "gram launch");
}

int dadmm_gnn_gram_acc(const dadmm_dims* d, const void* op, const float* x, float* out, const float* addend,
                       void* stream) {
    dadmm::GnnArgs a;
    int rc = gnn_common(d, &a);
    if (rc) return rc;
    if (d->B == 0) return ok();
    if (!op || !out || !x) return fail(DADMM_EINVAL, "a required pointer is NULL");
    if (!aligned16(op) || !aligned16(out) || !aligned16(x))
        return fail(DADMM_EINVAL, "op, x and out must be 16-byte aligned");
    if (dadmm::gnn_gram_lds(a.m_pad) > 160 * 1024)
        return fail(DADMM_EUNSUPPORTED, "m=%d too large for the gram tile", d->m);
    if (addend && !aligned16(addend)) return fail(DADMM_EINVAL, "addend must be 16-byte aligned");
    set_op(&a, op);
    a.acc_add = addend;
    return hip_rc(dadmm::gnn_launch_gram(a, 0, x, out, 2, (hipStream_t)stream), "gram launch");
}

int dadmm_gnn_step(const dadmm_dims* d, int32_t k, const int32_t* visit_ptr, const uint8_t* visit_q,
                   const float* deg, const float* hyp_k, float* const* yptr, const float* AtAy,
                   const float* Atb, const float* U, const float* D, float* U_next, float* D_next,
                   float* G, int32_t* flags, void* stream) {
    dadmm::GnnArgs a;
    int rc = gnn_common(d, &a);
    if (rc) return rc;
    if (k < 0 || k >= d->K) return fail(DADMM_EINVAL, "k=%d outside [0, K)", k);
    if (d->B == 0) return ok();
    if (!visit_ptr || !visit_q || !deg || !hyp_k || !yptr || !AtAy || !Atb || !U || !D || !U_next ||
        !D_next || !G || !flags)
        return fail(DADMM_EINVAL, "a required pointer is NULL");
    if (!aligned16(AtAy) || !aligned16(Atb) || !aligned16(U) || !aligned16(D) || !aligned16(G) ||
        !aligned16(U_next) || !aligned16(D_next))
        return fail(DADMM_EINVAL, "AtAy, Atb, U, D, U_next, D_next and G must be 16-byte aligned");
    a.vptr = visit_ptr;
    a.vq = visit_q;
    a.deg = deg;
    a.hyp = hyp_k;
    a.yptr = yptr;
    a.AtAy = AtAy;
    a.Atb = Atb;
    a.U = U;
    a.D = D;
    a.U_next = U_next;
    a.D_next = D_next;
    a.G = G;
    a.flags = flags;
    return hip_rc(dadmm::gnn_launch_step(a, k, (hipStream_t)stream), "step launch");
}

int dadmm_gnn_finish(const dadmm_dims* d, float* const* yptr, int32_t* flags, int32_t* status,
                     void* stream) {
    dadmm::GnnArgs a;
    int rc = gnn_common(d, &a);
    if (rc) return rc;
    if (d->K == 0) return ok();
    if (!yptr || !flags) return fail(DADMM_EINVAL, "a required pointer is NULL");
    a.yptr = yptr;
    a.flags = flags;
    a.status = status;
    return hip_rc(dadmm::gnn_launch_finish(a, (hipStream_t)stream), "finish launch");
}

int dadmm_gnn_step_backward(const dadmm_dims* d, int32_t k, const int32_t* visit_ptr,
                            const uint8_t* visit_q, const float* deg, const float* hyp_k,
                            const float* y_k, const float* AtAy, const float* Atb, const float* U,
                            const float* D, const float* gy1, const float* gU1, const float* gd1,
                            float* gy, float* gU, float* gd, float* gAtAy, float* ghyp,
                            void* stream) {
    dadmm::GnnArgs a;
    int rc = gnn_common(d, &a);
    if (rc) return rc;
    if (k < 0 || k >= d->K) return fail(DADMM_EINVAL, "k=%d outside [0, K)", k);
    if (d->B == 0) return ok();
    if (!visit_ptr || !visit_q || !deg || !hyp_k || !y_k || !AtAy || !Atb || !U || !D || !gy ||
        !gU || !gd || !gAtAy || !ghyp)
        return fail(DADMM_EINVAL, "a required pointer is NULL");
    a.vptr = visit_ptr;
    a.vq = visit_q;
    a.deg = deg;
    a.hyp = hyp_k;
    a.yk = y_k;
    a.AtAy = AtAy;
    a.Atb = Atb;
    a.U = U;
    a.D = D;
    dadmm::GnnGrads g{gy1, gU1, gd1, gy, gU, gd, gAtAy, ghyp, nullptr, nullptr, nullptr, {}};
    return hip_rc(dadmm::gnn_launch_step_backward(a, k, g, (hipStream_t)stream), "step backward launch");
}

int dadmm_gnn_step_backward_ex(const dadmm_dims* d, int32_t k, const int32_t* visit_ptr,
                               const uint8_t* visit_q, const float* deg, const float* hyp_k,
                               const float* y_k, const float* AtAy, const float* Atb, const float* U,
                               const float* D, const float* gy1, const float* gU1, const float* gd1,
                               float* gy, float* gU, float* gd, float* gAtAy, float* ghyp,
                               const dadmm_head_bwd* head, void* stream) {
    dadmm::GnnArgs a;
    int rc = gnn_common(d, &a);
    if (rc) return rc;
    if (k < 0 || k >= d->K) return fail(DADMM_EINVAL, "k=%d outside [0, K)", k);
    if (d->B == 0) return ok();
    if (!visit_ptr || !visit_q || !deg || !hyp_k || !y_k || !AtAy || !Atb || !U || !D || !gy ||
        !gU || !gd || !gAtAy || !ghyp)
        return fail(DADMM_EINVAL, "a required pointer is NULL");
    if (head && (!head->z || !head->dz)) return fail(DADMM_EINVAL, "head: z and dz are required");
    a.vptr = visit_ptr;
    a.vq = visit_q;
    a.deg = deg;
    a.hyp = hyp_k;
    a.yk = y_k;
    a.AtAy = AtAy;
    a.Atb = Atb;
    a.U = U;
    a.D = D;
    dadmm::GnnGrads g{gy1, gU1, gd1, gy, gU, gd, gAtAy, ghyp, nullptr, nullptr, nullptr, {}};
    if (head) {
        g.ghyp_add = head->ghyp_add;
        g.hz = head->z;
        g.hdz = head->dz;
        for (int c = 0; c < 4; ++c) g.hmax[c] = head->maxv[c];
    }
    return hip_rc(dadmm::gnn_launch_step_backward(a, k, g, (hipStream_t)stream), "step backward launch");
}

namespace {
// torch's calc_execution_policy for its Philox distribution kernels on the current device
int normal_policy(int64_t numel, int64_t* threads, uint64_t* step) {
    int dev = 0, sms = 0, tpm = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&sms, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipDeviceGetAttribute(&tpm, hipDeviceAttributeMaxThreadsPerMultiProcessor, dev) != hipSuccess)
        return -1;
    const uint64_t block = 256, unroll = 4;
    uint64_t grid = ((uint64_t)numel + block - 1) / block;
    const uint64_t cap = (uint64_t)sms * ((uint64_t)tpm / block);
    if (grid > cap) grid = cap;
    if (grid < 1) grid = 1;
    *threads = (int64_t)(grid * block);
    *step = (((uint64_t)numel - 1) / (block * grid * unroll) + 1) * 4;   // already a multiple of 4
    return 0;
}
}  // namespace

uint64_t dadmm_normal_offset_step(int64_t numel) {
    int64_t threads = 0;
    uint64_t step = 0;
    if (numel <= 0 || normal_policy(numel, &threads, &step) != 0) return 0;
    return step;
}

int dadmm_prologue(uint64_t seed, uint64_t offset, int64_t numel, int32_t n, int32_t n_store,
                   float mean, float stddev, float* y0, float* U0, float* d0, int32_t* zero,
                   int64_t nzero, void* stream) {
    if (numel < 0 || nzero < 0) return fail(DADMM_EINVAL, "negative size");
    if (nzero > 0 && zero == nullptr) return fail(DADMM_EINVAL, "zero is NULL");
    dadmm::PrologueArgs a{};
    if (numel > 0) {
        if (!y0 || !U0 || !d0) return fail(DADMM_EINVAL, "y0/U0/d0 is NULL");
        if (n < 1 || n_store < n || numel % n != 0)
            return fail(DADMM_EINVAL, "bad row length n=%d n_store=%d for numel=%lld", n, n_store,
                        (long long)numel);
        if (normal_policy(numel, &a.threads, &a.offset_step) != 0)
            return fail(DADMM_EHIP, "device attribute query failed");
        if ((offset & 3u) != 0) return fail(DADMM_EINVAL, "Philox offset must be a multiple of 4");
    }
    a.seed = seed;
    a.offset = offset;
    a.numel = numel;
    a.n = n;
    a.n_store = n_store;
    a.mean = mean;
    a.stddev = stddev;
    a.y0 = y0;
    a.U0 = U0;
    a.d0 = d0;
    a.zero = zero;
    a.nzero = nzero;
    hipError_t e = dadmm::launch_prologue(a, (hipStream_t)stream);
    if (e != hipSuccess) return fail(DADMM_EHIP, "prologue launch: %s", hipGetErrorString(e));
    return ok();
}


int dadmm_graph_generate(int32_t B, int32_t P, float prob, uint64_t seed, int32_t connect,
                         int64_t* nbr, float* deg, int32_t* order, int32_t* vptr, uint8_t* vq,
                         int32_t* scratch, void* stream) {
    if (B < 0 || P < 1 || P > 64) return fail(DADMM_EINVAL, "bad graph dims B=%d P=%d (P <= 64)", B, P);
    if (!(prob >= 0.0f && prob <= 1.0f)) return fail(DADMM_EINVAL, "edge probability %g not in [0, 1]", prob);
    if (order != nullptr && P > 8) return fail(DADMM_EINVAL, "order packs 4-bit agent ids: P <= 8");
    if (B == 0) return ok();
    if (!nbr || !deg || !vptr || !scratch) return fail(DADMM_EINVAL, "a required pointer is NULL");
    if ((int64_t)B * 2 * P * (P - 1) >= ((int64_t)1 << 31))
        return fail(DADMM_EUNSUPPORTED, "visit lists past 2^31 entries (split the batch)");
    dadmm::GraphGenArgs a{B, P, prob, seed, connect ? 1 : 0, nbr, deg, order, scratch, vptr, vq};
    hipError_t e = dadmm::launch_graphgen(a, vq == nullptr ? 0 : 1, (hipStream_t)stream);
    if (e != hipSuccess) return fail(DADMM_EHIP, "graph generation launch: %s", hipGetErrorString(e));
    return ok();
}

size_t dadmm_tiled_scratch_bytes(const dadmm_dims* d) {
    if (check_dims(d) != DADMM_OK) return 0;
    // U ping-pong, delta; R_k of the column-split path
    return 3 * align256(sizeof(float) * (size_t)d->B * d->P * d->n) +
           align256(sizeof(float) * (size_t)d->B * d->P * m_pad_of(d));
}

static int forward_tiled_impl(const dadmm_dims* d, const void* op, const float* b,
                              const int32_t* visit_ptr, const uint8_t* visit_q, const float* deg,
                              const float* hyp, const float* y0, const float* U0, const float* d0,
                              float* Y, float* Grec, float* Urec, float* U_out, int32_t* status,
                              void* scratch, void* stream) {
    int rc = check_dims(d);
    if (rc) return rc;
    if (d->B == 0 || d->K == 0) return ok();
    if (!op || !b || !visit_ptr || !visit_q || !deg || !hyp || !y0 || !U0 || !d0 || !Y || !scratch)
        return fail(DADMM_EINVAL, "a required pointer is NULL");
    if (!aligned16(op) || !aligned16(Y) || !aligned16(y0) || !aligned16(U0) || !aligned16(d0) ||
        (U_out != nullptr && !aligned16(U_out)))
        return fail(DADMM_EINVAL, "op, Y, y0, U0, d0 and U_out must be 16-byte aligned");
    if (((uintptr_t)scratch & 255u) != 0) return fail(DADMM_EINVAL, "scratch must be 256-byte aligned");
    if (m_pad_of(d) > 2 * dadmm::M_PAD)   // iter_kernel<MB>: MB in {1, 2}
        return fail(DADMM_EUNSUPPORTED, "m=%d > %d rows per agent: not a tiled shape", d->m,
                    2 * dadmm::M_PAD);
    if ((d->n & 3) != 0) return fail(DADMM_EUNSUPPORTED, "n=%d: needs n %% 4 == 0 (zero-pad n)", d->n);
    if ((size_t)d->B * d->P * d->n * 4 >= ((size_t)1 << 31))
        return fail(DADMM_EUNSUPPORTED, "B*P*n*4 >= 2^31 bytes per iterate (split the batch)");
    const int np = n_pad_of(d);
    if (dadmm::tiled_lds_bytes(np, m_pad_of(d)) > 160 * 1024)
        return fail(DADMM_EUNSUPPORTED, "n=%d: the y tile does not fit the LDS", d->n);
    const size_t state = align256(sizeof(float) * (size_t)d->B * d->P * d->n);
    dadmm::TiledArgs a{};
    a.A = (const float*)op;
    a.At = a.A + (size_t)d->P * m_pad_of(d) * np;
    a.b = b;
    a.vptr = visit_ptr;
    a.vq = visit_q;
    a.deg = deg;
    a.hyp = hyp;
    a.y0 = y0;
    a.U0 = U0;
    a.d0 = d0;
    a.Y = Y;
    a.Ubuf[0] = (float*)scratch;
    a.Ubuf[1] = (float*)((char*)scratch + state);
    a.delta = (float*)((char*)scratch + 2 * state);
    a.R = (float*)((char*)scratch + 3 * state);
    a.U_out = U_out;
    a.status = status;
    a.B = d->B;
    a.P = d->P;
    a.m = d->m;
    a.m_pad = m_pad_of(d);
    a.n = d->n;
    a.n_pad = np;
    a.K = d->K;
    a.hyp_rows = d->hyp_rows;
    a.variant = d->variant;
    a.graph_shared = d->graph_shared;
    if (Grec != nullptr || Urec != nullptr) {   // recording: the streamed single-launch form only
        if (Grec == nullptr || Urec == nullptr || !aligned16(Grec) || !aligned16(Urec))
            return fail(DADMM_EINVAL, "Grec and Urec: both, 16-byte aligned");
        if ((size_t)d->K * d->B * d->P * d->n * 4 >= ((size_t)1 << 40))
            return fail(DADMM_EINVAL, "recording too large");
        a.Grec = Grec;
        a.Urec = Urec;
        if (!dadmm::stream_applies(a))
            return fail(DADMM_EUNSUPPORTED, "recording on the tiled path needs the streamed form (P <= 16, "
                                            "m <= 64, n_pad >= 128): use dadmm_forward_stepwise");
        hipError_t e = dadmm::launch_stream(a, (hipStream_t)stream);
        if (e != hipSuccess) return fail(DADMM_EHIP, "streamed recording launch: %s", hipGetErrorString(e));
        return ok();
    }
    hipError_t e = dadmm::launch_tiled(a, (hipStream_t)stream);
    if (e != hipSuccess) return fail(DADMM_EHIP, "tiled launch: %s", hipGetErrorString(e));
    return ok();
}

int dadmm_forward_tiled(const dadmm_dims* d, const void* op, const float* b,
                        const int32_t* visit_ptr, const uint8_t* visit_q, const float* deg,
                        const float* hyp, const float* y0, const float* U0, const float* d0,
                        float* Y, float* U_out, int32_t* status, void* scratch, void* stream) {
    return forward_tiled_impl(d, op, b, visit_ptr, visit_q, deg, hyp, y0, U0, d0, Y, nullptr, nullptr,
                              U_out, status, scratch, stream);
}

int dadmm_forward_tiled_record(const dadmm_dims* d, const void* op, const float* b,
                               const int32_t* visit_ptr, const uint8_t* visit_q, const float* deg,
                               const float* hyp, const float* y0, const float* U0, const float* d0,
                               float* Y, float* Grec, float* Urec, float* U_out, int32_t* status,
                               void* scratch, void* stream) {
    if (Grec == nullptr || Urec == nullptr) return fail(DADMM_EINVAL, "Grec and Urec are required");
    return forward_tiled_impl(d, op, b, visit_ptr, visit_q, deg, hyp, y0, U0, d0, Y, Grec, Urec, U_out,
                              status, scratch, stream);
}

size_t dadmm_loss_scratch_bytes(int32_t K, int64_t rows, int32_t n) {
    if (K < 1 || rows < 0 || n < 1) return 0;
    return 4 * dadmm::loss_scratch_floats(K, rows, n);
}

static int loss_args(int32_t K, int32_t B, int32_t P, int32_t n, int32_t n_store, const float* Y,
                     const float* label, dadmm::LossArgs* a) {
    if (K < 1 || B < 1 || P < 1 || n < 1 || n_store < n)
        return fail(DADMM_EINVAL, "bad loss dims K=%d B=%d P=%d n=%d n_store=%d", K, B, P, n, n_store);
    if (!Y || !label) return fail(DADMM_EINVAL, "Y/label is NULL");
    if ((int64_t)B * P * n_store >= ((int64_t)1 << 31))
        return fail(DADMM_EUNSUPPORTED, "B*P*n_store >= 2^31 values per layer");
    *a = dadmm::LossArgs{};
    a->Y = Y;
    a->label = label;
    a->K = K;
    a->P = P;
    a->n = n;
    a->n_store = n_store;
    a->rows = (int64_t)B * P;
    return DADMM_OK;
}

int dadmm_loss(int32_t K, int32_t B, int32_t P, int32_t n, int32_t n_store, const float* Y,
               const float* label, float* losses, float* out, int32_t* flags, void* scratch,
               void* stream) {
    dadmm::LossArgs a;
    int rc = loss_args(K, B, P, n, n_store, Y, label, &a);
    if (rc) return rc;
    if (!losses || !out || !flags || !scratch) return fail(DADMM_EINVAL, "a required pointer is NULL");
    a.partial = (float*)scratch;
    a.losses = losses;
    a.out = out;
    a.flags = flags;
    hipError_t e = dadmm::launch_loss(a, (hipStream_t)stream);
    if (e != hipSuccess) return fail(DADMM_EHIP, "loss launch: %s", hipGetErrorString(e));
    return ok();
}

int dadmm_loss_grad(int32_t K, int32_t B, int32_t P, int32_t n, int32_t n_store, const float* Y,
                    const float* label, const int32_t* flags, const float* gout, float* dY,
                    void* stream) {
    dadmm::LossArgs a;
    int rc = loss_args(K, B, P, n, n_store, Y, label, &a);
    if (rc) return rc;
    if (!flags || !gout || !dY) return fail(DADMM_EINVAL, "a required pointer is NULL");
    a.flags = const_cast<int32_t*>(flags);
    hipError_t e = dadmm::launch_loss_grad(a, gout, dY, (hipStream_t)stream);
    if (e != hipSuccess) return fail(DADMM_EHIP, "loss grad launch: %s", hipGetErrorString(e));
    return ok();
}

static int hyper_input(int32_t rows, int32_t K, int32_t N, const float* x1, int32_t ld1, int32_t K1,
                       const float* x2, int32_t ld2, const float* W, const float* y, int32_t ldy,
                       dadmm::HyperArgs* a) {
    if (rows < 0 || K < 1 || N < 1 || K1 < 1 || K1 > K)
        return fail(DADMM_EINVAL, "bad linear dims rows=%d K=%d N=%d K1=%d", rows, K, N, K1);
    if (!x1 || !W || !y || (K1 < K && !x2)) return fail(DADMM_EINVAL, "a required pointer is NULL");
    if ((K & 3) || (K1 & 3) || (ld1 & 3) || (K1 < K && (ld2 & 3)) || ld1 < K1 ||
        (K1 < K && ld2 < K - K1) || ldy < N)
        return fail(DADMM_EUNSUPPORTED, "K, K1 and the input row strides must be multiples of 4 "
                    "(K=%d K1=%d ld1=%d ld2=%d, ldy=%d >= N=%d)", K, K1, ld1, ld2, ldy, N);
    if (K1 < K && (K1 & 15))
        return fail(DADMM_EUNSUPPORTED, "a split input needs K1 %% 16 == 0 (K1=%d)", K1);
    if (!aligned16(x1) || (x2 && !aligned16(x2)) || !aligned16(W))
        return fail(DADMM_EINVAL, "x1, x2 and W must be 16-byte aligned");
    if ((int64_t)rows * (ld1 > ld2 ? ld1 : ld2) >= ((int64_t)1 << 31) ||
        (int64_t)rows * ldy >= ((int64_t)1 << 31))
        return fail(DADMM_EUNSUPPORTED, "operand larger than 2^31 floats");
    *a = dadmm::HyperArgs{};
    a->x1 = x1;
    a->x2 = x2;
    a->ld1 = ld1;
    a->ld2 = ld2;
    a->K1 = K1;
    a->W = W;
    a->ldw = K;
    a->y = const_cast<float*>(y);
    a->ldy = ldy;
    a->rows = rows;
    a->K = K;
    a->N = N;
    return DADMM_OK;
}

int dadmm_hyper_linear(int32_t rows, int32_t K, int32_t N, const float* x1, int32_t ld1,
                       int32_t K1, const float* x2, int32_t ld2, const float* W, const float* bias,
                       float* y, int32_t ldy, void* stream) {
    dadmm::HyperArgs a;
    int rc = hyper_input(rows, K, N, x1, ld1, K1, x2, ld2, W, y, ldy, &a);
    if (rc) return rc;
    a.bias = bias;
    a.P = 1;
    a.B = rows;
    a.splits = 1;
    hipError_t e = dadmm::launch_hyper(a, HYPER_EPI_BIAS, (hipStream_t)stream);
    if (e != hipSuccess) return fail(DADMM_EHIP, "linear launch: %s", hipGetErrorString(e));
    return ok();
}

static int hyper_linear_ex_kw(int32_t kwave, int32_t rows, int32_t K, int32_t N, const float* x1, int32_t ld1,
                              int32_t K1, const float* x2, int32_t ld2, const float* W, const float* bias,
                              const float* addend, int32_t ld_add, float* y, int32_t ldy, void* stream) {
    dadmm::HyperArgs a;
    int rc = hyper_input(rows, K, N, x1, ld1, K1, x2, ld2, W, y, ldy, &a);
    if (rc) return rc;
    if (addend && ld_add < N) return fail(DADMM_EINVAL, "ld_add=%d < N=%d", ld_add, N);
    a.bias = bias;
    a.addend = addend;
    a.ld_add = ld_add;
    a.P = 1;
    a.B = rows;
    a.splits = 1;
    a.kwave = kwave;
    hipError_t e = dadmm::launch_hyper(a, HYPER_EPI_BIAS, (hipStream_t)stream);
    if (e != hipSuccess) return fail(DADMM_EHIP, "linear launch: %s", hipGetErrorString(e));
    return ok();
}

int dadmm_hyper_linear_ex(int32_t rows, int32_t K, int32_t N, const float* x1, int32_t ld1, int32_t K1,
                          const float* x2, int32_t ld2, const float* W, const float* bias, const float* addend,
                          int32_t ld_add, float* y, int32_t ldy, void* stream) {
    return hyper_linear_ex_kw(0, rows, K, N, x1, ld1, K1, x2, ld2, W, bias, addend, ld_add, y, ldy, stream);
}

extern "C++" {
namespace dadmm {
int hyper_linear_gcn_dx(int32_t P, int32_t rows, int32_t K, int32_t N, const float* x, int32_t ldx, const float* W,
                        const float* addend, int32_t ld_add, float* y, int32_t ldy, void* stream) {
    return hyper_linear_ex_kw(P, rows, K, N, x, ldx, K, nullptr, 0, W, nullptr, addend, ld_add, y, ldy, stream);
}
}  // namespace dadmm
}

int dadmm_hyper_gcn(int32_t B, int32_t P, int32_t K, int32_t N, const float* x1, int32_t ld1,
                    int32_t K1, const float* x2, int32_t ld2, const float* W, const float* bias,
                    const float* ahat, int32_t ahat_per_sample, const float* bn_mean,
                    const float* bn_var, const float* bn_weight, const float* bn_bias, float bn_eps,
                    float slope, float* y, int32_t ldy, void* stream) {
    // the GCN epilogue's row tile holds whole samples: at most 160 rows
    if (B < 0 || P < 1 || P > 160) return fail(DADMM_EINVAL, "bad gcn dims B=%d P=%d (P <= 160)", B, P);
    dadmm::HyperArgs a;
    int rc = hyper_input(B * P, K, N, x1, ld1, K1, x2, ld2, W, y, ldy, &a);
    if (rc) return rc;
    if (!bias || !ahat || !bn_mean || !bn_var || !bn_weight || !bn_bias)
        return fail(DADMM_EINVAL, "a required pointer is NULL");
    a.bias = bias;
    a.B = B;
    a.P = P;
    a.kwave = P;   // GCN-class GEMM (the K split may apply, hyper_kwave)
    a.ahat = ahat;
    a.ahat_per_sample = ahat_per_sample ? 1 : 0;
    a.bn_mean = bn_mean;
    a.bn_var = bn_var;
    a.bn_w = bn_weight;
    a.bn_b = bn_bias;
    a.bn_eps = bn_eps;
    a.slope = slope;
    hipError_t e = dadmm::launch_hyper(a, HYPER_EPI_GCN, (hipStream_t)stream);
    if (e != hipSuccess) return fail(DADMM_EHIP, "gcn launch: %s", hipGetErrorString(e));
    return ok();
}

int dadmm_hyper_gcn_ex(int32_t B, int32_t P, int32_t K, int32_t N, const float* x, int32_t ldx,
                       const float* W, int32_t ldw, const float* addend, int32_t ld_add, const float* bias,
                       const float* ahat, int32_t ahat_per_sample, const float* bn_mean,
                       const float* bn_var, const float* bn_weight, const float* bn_bias, float bn_eps,
                       float slope, int32_t raw, float* y, int32_t ldy, void* stream) {
    if (B < 0 || P < 1 || P > 160) return fail(DADMM_EINVAL, "bad gcn dims B=%d P=%d (P <= 160)", B, P);
    dadmm::HyperArgs a;
    int rc = hyper_input(B * P, K, N, x, ldx, K, nullptr, 0, W, y, ldy, &a);
    if (rc) return rc;
    if (ldw < K || (ldw & 3)) return fail(DADMM_EUNSUPPORTED, "ldw=%d must be >= K=%d and a multiple of 4", ldw, K);
    if (!ahat || (!raw && (!bias || !bn_mean || !bn_var || !bn_weight || !bn_bias)))
        return fail(DADMM_EINVAL, "a required pointer is NULL");
    if (addend && (ld_add < N || (ld_add & 3) || !aligned16(addend)))
        return fail(DADMM_EUNSUPPORTED, "addend needs ld_add >= N, ld_add %% 4 == 0 and 16-byte alignment");
    a.ldw = ldw;
    a.addend = addend;
    a.ld_add = ld_add;
    a.raw = raw ? 1 : 0;
    a.bias = bias;
    a.B = B;
    a.P = P;
    a.kwave = P;   // GCN-class GEMM (the K split may apply, hyper_kwave)
    a.ahat = ahat;
    a.ahat_per_sample = ahat_per_sample ? 1 : 0;
    a.bn_mean = bn_mean;
    a.bn_var = bn_var;
    a.bn_w = bn_weight;
    a.bn_b = bn_bias;
    a.bn_eps = bn_eps;
    a.slope = slope;
    hipError_t e = dadmm::launch_hyper(a, HYPER_EPI_GCN, (hipStream_t)stream);
    if (e != hipSuccess) return fail(DADMM_EHIP, "gcn launch: %s", hipGetErrorString(e));
    return ok();
}

int dadmm_hyper_head(int32_t B, int32_t K, int32_t H, const float* x, int32_t ldx, const float* W,
                     const float* bias, float alpha_max, float tau_max, float rho_max,
                     float eta_max, float* hyp, void* stream) {
    if (H < 1) return fail(DADMM_EINVAL, "bad head rows H=%d", H);
    dadmm::HyperArgs a;
    int rc = hyper_input(B, K, 4 * H, x, ldx, K, nullptr, 0, W, hyp, 4 * H, &a);
    if (rc) return rc;
    if (!bias) return fail(DADMM_EINVAL, "bias is NULL");
    a.bias = bias;
    a.P = 1;
    a.B = B;
    a.H = H;
    a.maxv[0] = alpha_max;
    a.maxv[1] = tau_max;
    a.maxv[2] = rho_max;
    a.maxv[3] = eta_max;
    hipError_t e = dadmm::launch_hyper(a, HYPER_EPI_HEAD, (hipStream_t)stream);
    if (e != hipSuccess) return fail(DADMM_EHIP, "head launch: %s", hipGetErrorString(e));
    return ok();
}

int dadmm_hyper_head_train(int32_t B, int32_t K, int32_t H, const float* x, int32_t ldx, const float* W,
                           const float* bias, float alpha_max, float tau_max, float rho_max, float eta_max,
                           float* z, float* hyp, void* stream) {
    if (!z) return fail(DADMM_EINVAL, "z is NULL");
    if (H < 1) return fail(DADMM_EINVAL, "bad head rows H=%d", H);
    dadmm::HyperArgs a;
    int rc = hyper_input(B, K, 4 * H, x, ldx, K, nullptr, 0, W, hyp, 4 * H, &a);
    if (rc) return rc;
    if (!bias) return fail(DADMM_EINVAL, "bias is NULL");
    a.bias = bias;
    a.P = 1;
    a.B = B;
    a.H = H;
    a.maxv[0] = alpha_max;
    a.maxv[1] = tau_max;
    a.maxv[2] = rho_max;
    a.maxv[3] = eta_max;
    a.save_m = z;
    hipError_t e = dadmm::launch_hyper(a, HYPER_EPI_HEAD, (hipStream_t)stream);
    if (e != hipSuccess) return fail(DADMM_EHIP, "head launch: %s", hipGetErrorString(e));
    return ok();
}

int dadmm_hyper_rownorm(int32_t rows, int32_t C, const float* x, const float* weight,
                        const float* bias, float eps, int32_t act, float slope, float* y,
                        void* stream) {
    if (rows < 0 || C < 1) return fail(DADMM_EINVAL, "bad rownorm dims rows=%d C=%d", rows, C);
    if ((C & 3) || C > 2048) return fail(DADMM_EUNSUPPORTED, "rownorm needs C %% 4 == 0, C <= 2048 (C=%d)", C);
    if (!x || !weight || !bias || !y) return fail(DADMM_EINVAL, "a required pointer is NULL");
    if (!aligned16(x) || !aligned16(weight) || !aligned16(bias) || !aligned16(y))
        return fail(DADMM_EINVAL, "rownorm operands must be 16-byte aligned");
    dadmm::RowNormArgs a{x, weight, bias, y, rows, C, act ? 1 : 0, eps, slope, 1, 0, nullptr};
    hipError_t e = dadmm::launch_rownorm(a, (hipStream_t)stream);
    if (e != hipSuccess) return fail(DADMM_EHIP, "rownorm launch: %s", hipGetErrorString(e));
    return ok();
}

size_t dadmm_hyper_linear_ln_scratch_bytes(int32_t rows, int32_t K, int32_t N) {
    if (rows < 0 || K < 1 || N < 1) return 0;
    return 4 * (size_t)dadmm::hyper_linear_splits(rows, K, N) * rows * N;
}

int dadmm_hyper_linear_ln(int32_t rows, int32_t K, int32_t N, const float* x, int32_t ldx,
                          const float* W, const float* bias, const float* ln_weight,
                          const float* ln_bias, float eps, int32_t act, float slope, float* y,
                          void* scratch, void* stream) {
    dadmm::HyperArgs a;
    int rc = hyper_input(rows, K, N, x, ldx, K, nullptr, 0, W, y, N, &a);
    if (rc) return rc;
    if ((N & 3) || N > 2048) return fail(DADMM_EUNSUPPORTED, "LayerNorm width N=%d: N %% 4 == 0, N <= 2048", N);
    if (!bias || !ln_weight || !ln_bias || !scratch) return fail(DADMM_EINVAL, "a required pointer is NULL");
    if (!aligned16(scratch) || !aligned16(y) || !aligned16(bias) || !aligned16(ln_weight) ||
        !aligned16(ln_bias))
        return fail(DADMM_EINVAL, "y, scratch, bias and the LayerNorm parameters must be 16-byte aligned");
    if (rows == 0) return ok();
    a.splits = dadmm::hyper_linear_splits(rows, K, N);
    a.split_stride = (size_t)rows * N;
    a.y = (float*)scratch;
    a.ldy = N;
    a.P = 1;
    a.B = rows;
    hipError_t e = dadmm::launch_hyper(a, HYPER_EPI_BIAS, (hipStream_t)stream);
    if (e != hipSuccess) return fail(DADMM_EHIP, "linear launch: %s", hipGetErrorString(e));
    dadmm::RowNormArgs r{(const float*)scratch, ln_weight, ln_bias, y, rows, N, act ? 1 : 0, eps,
                         slope, a.splits, a.split_stride, bias};
    e = dadmm::launch_rownorm(r, (hipStream_t)stream);
    if (e != hipSuccess) return fail(DADMM_EHIP, "rownorm launch: %s", hipGetErrorString(e));
    return ok();
}

int dadmm_hyper_gcn_train(int32_t B, int32_t P, int32_t K, int32_t N, const float* x1, int32_t ld1,
                          int32_t K1, const float* x2, int32_t ld2, const float* W, const float* bias,
                          const float* ahat, int32_t ahat_per_sample, const float* bn_weight,
                          const float* bn_bias, float bn_eps, float slope, float drop_p, uint64_t seed,
                          int32_t site, float* y, int32_t ldy, float* m_out, float* mean_out,
                          float* var_out, const float* bn_running_mean, const float* bn_running_var,
                          void* stream) {
    return dadmm::gcn_train_impl(B, P, K, N, x1, ld1, K1, x2, ld2, W, K, nullptr, 0, bias, ahat, ahat_per_sample,
                                 bn_weight, bn_bias, bn_eps, slope, drop_p, seed, site, y, ldy, m_out, mean_out,
                                 var_out, bn_running_mean, bn_running_var, stream);
}

}  // extern "C"

// dadmm_hyper_gcn_train with a column slice of W (row stride ldw) and an addend [B*P][ld_add]
// added to the mix before the bias (layer 1's Atb half, formed once per forward)
int dadmm::gcn_train_impl(int32_t B, int32_t P, int32_t K, int32_t N, const float* x1, int32_t ld1, int32_t K1,
                          const float* x2, int32_t ld2, const float* W, int32_t ldw, const float* addend,
                          int32_t ld_add, const float* bias, const float* ahat, int32_t ahat_per_sample,
                          const float* bn_weight, const float* bn_bias, float bn_eps, float slope, float drop_p,
                          uint64_t seed, int32_t site, float* y, int32_t ldy, float* m_out, float* mean_out,
                          float* var_out, const float* bn_running_mean, const float* bn_running_var,
                          void* stream) {
    if ((bn_running_mean == nullptr) != (bn_running_var == nullptr))
        return fail(DADMM_EINVAL, "running mean and variance: both or neither");
    if (B < 0 || P < 2 || P > 160)
        return fail(DADMM_EINVAL, "bad gcn dims B=%d P=%d (training BatchNorm needs P >= 2; P <= 160)", B, P);
    if (!(drop_p >= 0.0f && drop_p < 1.0f)) return fail(DADMM_EINVAL, "dropout p=%g not in [0, 1)", drop_p);
    dadmm::HyperArgs a;
    int rc = hyper_input(B * P, K, N, x1, ld1, K1, x2, ld2, W, y, ldy, &a);
    if (rc) return rc;
    if (!bias || !ahat || !bn_weight || !bn_bias || !m_out || !mean_out || !var_out)
        return fail(DADMM_EINVAL, "a required pointer is NULL");
    if (!aligned16(m_out) || (N & 3) || (ldy & 3) || !aligned16(y))
        return fail(DADMM_EUNSUPPORTED, "training GCN needs N %% 4 == 0 and 16-byte aligned y / m_out");
    a.bias = bias;
    a.B = B;
    a.P = P;
    a.kwave = P;   // GCN-class GEMM (the K split may apply, hyper_kwave)
    a.ahat = ahat;
    a.ahat_per_sample = ahat_per_sample ? 1 : 0;
    a.bn_w = bn_weight;
    a.bn_b = bn_bias;
    a.bn_eps = bn_eps;
    a.slope = slope;
    a.save_m = m_out;
    a.save_mean = mean_out;
    a.save_var = var_out;
    // eval-mode BatchNorm (running statistics) inside the training epilogue, else batch statistics
    a.bn_mean = bn_running_mean;
    a.bn_var = bn_running_var;
    a.drop_p = drop_p;
    a.seed = seed;
    a.site = site;
    if (ldw < K || (ldw & 3)) return fail(DADMM_EINVAL, "ldw=%d < K=%d or not a multiple of 4", ldw, K);
    a.ldw = ldw;
    if (addend && (ld_add < N || (ld_add & 3) || !aligned16(addend)))
        return fail(DADMM_EINVAL, "addend: ld_add=%d < N=%d or misaligned", ld_add, N);
    a.addend = addend;
    a.ld_add = ld_add;
    hipError_t e = dadmm::launch_hyper(a, HYPER_EPI_GCN_TRAIN, (hipStream_t)stream);
    if (e != hipSuccess) return fail(DADMM_EHIP, "gcn train launch: %s", hipGetErrorString(e));
    return ok();
}

extern "C" {

static int bn_running_splits(int32_t iters, int32_t B) {
    // ~64 rows per split (16 per wave): enough blocks to spread the sums over the chip (256-row
    // splits measured 46 vs 30 us for the partial pass at B = 256, K = 25)
    const int64_t T = (int64_t)iters * B;
    const int64_t s = T / 64;
    return s < 1 ? 1 : (s > 256 ? 256 : (int)s);
}

size_t dadmm_hyper_bn_running_scratch_bytes(int32_t layers, const int32_t* widths, int32_t iters,
                                            int32_t B) {
    if (layers < 1 || layers > dadmm::BN_MAX_LAYERS || !widths || iters < 1 || B < 1) return 0;
    size_t total = 0;
    for (int i = 0; i < layers; ++i) total += widths[i] > 0 ? (size_t)widths[i] : 0;
    return 8 * 2 * total * (size_t)bn_running_splits(iters, B);
}

int dadmm_hyper_bn_running_update(int32_t layers, const int32_t* widths, float* const* running_mean,
                                  float* const* running_var, int64_t* const* tracked,
                                  const float* const* mean, const float* const* var,
                                  int64_t block_stride, int32_t iters, int32_t B, int32_t P,
                                  const double* weights, double decay, void* scratch, void* stream) {
    if (layers < 1 || layers > dadmm::BN_MAX_LAYERS || !widths || !running_mean || !running_var || !mean ||
        !var || !weights || !scratch || P < 2 || B < 0 || iters < 0)
        return fail(DADMM_EINVAL, "bad BatchNorm running-statistics arguments");
    if ((uintptr_t)scratch & 7) return fail(DADMM_EINVAL, "scratch must be 8-byte aligned");
    if (B == 0 || iters == 0) return ok();
    if ((int64_t)iters * B >= ((int64_t)1 << 31)) return fail(DADMM_EUNSUPPORTED, "too many rows");
    dadmm::BnRunArgs a{};
    a.layers = layers;
    a.iters = iters;
    a.B = B;
    a.P = P;
    a.col0[0] = 0;
    for (int i = 0; i < layers; ++i) {
        if (widths[i] < 1 || !running_mean[i] || !running_var[i] || !mean[i] || !var[i])
            return fail(DADMM_EINVAL, "layer %d: bad width or NULL pointer", i);
        if (block_stride < (int64_t)B * widths[i] && iters > 1)
            return fail(DADMM_EINVAL, "block_stride shorter than one iteration's [B][width] block");
        a.width[i] = widths[i];
        a.col0[i + 1] = a.col0[i] + widths[i];
        a.rmean[i] = running_mean[i];
        a.rvar[i] = running_var[i];
        a.tracked[i] = tracked ? tracked[i] : nullptr;
        a.mean[i] = mean[i];
        a.var[i] = var[i];
    }
    a.block_stride = block_stride;
    a.w = weights;
    a.decay = decay;
    a.part = (double*)scratch;
    a.splits = bn_running_splits(iters, B);
    hipError_t e = dadmm::launch_bn_running(a, (hipStream_t)stream);
    if (e != hipSuccess) return fail(DADMM_EHIP, "BatchNorm running-statistics launch: %s", hipGetErrorString(e));
    return ok();
}

int dadmm_hyper_gcn_train_bwd(int32_t B, int32_t P, int32_t N, const float* dy, const float* m,
                              const float* mean, const float* var, const float* bn_weight,
                              float bn_eps, const float* ahat, int32_t ahat_per_sample, float slope,
                              float drop_p, uint64_t seed, int32_t site, float* dz, float* part,
                              int32_t bn_eval, void* stream) {
    if (B < 0 || P < 2 || P > 64 || N < 1) return fail(DADMM_EINVAL, "bad gcn dims B=%d P=%d N=%d", B, P, N);
    if (!dy || !m || !mean || !var || !bn_weight || !ahat || !dz || !part)
        return fail(DADMM_EINVAL, "a required pointer is NULL");
    if ((int64_t)B * P * N >= ((int64_t)1 << 31)) return fail(DADMM_EUNSUPPORTED, "operand larger than 2^31 floats");
    dadmm::GcnBwdArgs a{dy, m, mean, var, bn_weight, ahat, ahat_per_sample ? 1 : 0, dz, part, B, P, N,
                        bn_eps, slope, drop_p, seed, site, bn_eval ? 1 : 0};
    hipError_t e = dadmm::launch_gcn_bwd(a, (hipStream_t)stream);
    if (e != hipSuccess) return fail(DADMM_EHIP, "gcn backward launch: %s", hipGetErrorString(e));
    return ok();
}

int dadmm_hyper_linear_gcn_bwd(int32_t B, int32_t P, int32_t K, int32_t N, const float* x, int32_t ldx,
                               const float* W, const float* m, const float* mean, const float* var,
                               const float* bn_weight, float bn_eps, const float* ahat, int32_t ahat_per_sample,
                               float slope, float drop_p, uint64_t seed, int32_t site, float* dz, float* part,
                               int32_t bn_eval, void* stream) {
    if (B < 0 || P < 2 || P > 64 || N < 1) return fail(DADMM_EINVAL, "bad gcn dims B=%d P=%d N=%d", B, P, N);
    dadmm::HyperArgs a;
    int rc = hyper_input(B * P, K, N, x, ldx, K, nullptr, 0, W, dz, N, &a);
    if (rc) return rc;
    if (!m || !mean || !var || !bn_weight || !ahat || !part) return fail(DADMM_EINVAL, "a required pointer is NULL");
    if ((N & 3) || !aligned16(dz)) return fail(DADMM_EUNSUPPORTED, "N %% 4 == 0 and a 16-byte aligned dz required");
    if (!(drop_p >= 0.0f && drop_p < 1.0f)) return fail(DADMM_EINVAL, "dropout p=%g not in [0, 1)", drop_p);
    if ((int64_t)B * P * (K > N ? K : N) >= ((int64_t)1 << 31))
        return fail(DADMM_EUNSUPPORTED, "operand larger than 2^31 floats");
    a.B = B;
    a.P = P;
    a.kwave = P;   // GCN-class GEMM (the K split may apply, hyper_kwave)
    a.splits = 1;
    a.ahat = ahat;
    a.ahat_per_sample = ahat_per_sample ? 1 : 0;
    a.save_m = const_cast<float*>(m);
    a.save_mean = const_cast<float*>(mean);
    a.save_var = const_cast<float*>(var);
    a.bn_w = bn_weight;
    a.bn_eps = bn_eps;
    a.slope = slope;
    a.drop_p = drop_p;
    a.seed = seed;
    a.site = site;
    a.part = part;
    a.bn_eval = bn_eval ? 1 : 0;
    hipError_t e = dadmm::launch_hyper(a, HYPER_EPI_GCN_BWD, (hipStream_t)stream);
    if (e != hipSuccess) return fail(DADMM_EHIP, "linear + gcn backward launch: %s", hipGetErrorString(e));
    return ok();
}

int dadmm_hyper_linear_ln_train(int32_t rows, int32_t K, int32_t N, const float* x, int32_t ldx,
                                const float* W, const float* bias, const float* ln_weight,
                                const float* ln_bias, float eps, int32_t act, float slope, float drop_p,
                                uint64_t seed, int32_t site, float* y, float* xd, void* scratch,
                                void* stream) {
    dadmm::HyperArgs a;
    int rc = hyper_input(rows, K, N, x, ldx, K, nullptr, 0, W, y, N, &a);
    if (rc) return rc;
    if ((N & 3) || N > 2048) return fail(DADMM_EUNSUPPORTED, "LayerNorm width N=%d: N %% 4 == 0, N <= 2048", N);
    if (!(drop_p >= 0.0f && drop_p < 1.0f)) return fail(DADMM_EINVAL, "dropout p=%g not in [0, 1)", drop_p);
    if (!bias || !ln_weight || !ln_bias || !scratch || !xd) return fail(DADMM_EINVAL, "a required pointer is NULL");
    if (!aligned16(scratch) || !aligned16(y) || !aligned16(xd) || !aligned16(bias) ||
        !aligned16(ln_weight) || !aligned16(ln_bias))
        return fail(DADMM_EINVAL, "y, xd, scratch, bias and the LayerNorm parameters must be 16-byte aligned");
    if (rows == 0) return ok();
    a.splits = dadmm::hyper_linear_splits(rows, K, N);
    a.split_stride = (size_t)rows * N;
    a.y = (float*)scratch;
    a.ldy = N;
    a.P = 1;
    a.B = rows;
    hipError_t e = dadmm::launch_hyper(a, HYPER_EPI_BIAS, (hipStream_t)stream);
    if (e != hipSuccess) return fail(DADMM_EHIP, "linear launch: %s", hipGetErrorString(e));
    dadmm::RowNormArgs r{(const float*)scratch, ln_weight, ln_bias, y, rows, N, act ? 1 : 0, eps,
                         slope, a.splits, a.split_stride, bias, drop_p, seed, site, xd};
    e = dadmm::launch_rownorm(r, (hipStream_t)stream);
    if (e != hipSuccess) return fail(DADMM_EHIP, "rownorm launch: %s", hipGetErrorString(e));
    return ok();
}

size_t dadmm_hyper_rownorm_bwd_part_bytes(int32_t rows, int32_t C) {
    if (rows < 0 || C < 1) return 0;
    return 4 * (size_t)((rows + dadmm::ROWNORM_BWD_ROWS - 1) / dadmm::ROWNORM_BWD_ROWS) * 2 * C;
}

int dadmm_hyper_rownorm_bwd(int32_t rows, int32_t C, const float* dy, const float* xd,
                            const float* weight, const float* bias, float eps, int32_t act,
                            float slope, float drop_p, uint64_t seed, int32_t site, float* dx,
                            float* part, void* stream) {
    if (rows < 0 || C < 1) return fail(DADMM_EINVAL, "bad rownorm dims rows=%d C=%d", rows, C);
    if ((C & 3) || C > 2048) return fail(DADMM_EUNSUPPORTED, "rownorm needs C %% 4 == 0, C <= 2048 (C=%d)", C);
    if (!dy || !xd || !weight || !bias || !dx || !part) return fail(DADMM_EINVAL, "a required pointer is NULL");
    if (!aligned16(dy) || !aligned16(xd) || !aligned16(weight) || !aligned16(bias) || !aligned16(dx))
        return fail(DADMM_EINVAL, "rownorm operands must be 16-byte aligned");
    dadmm::RowNormBwdArgs a{dy, xd, weight, bias, dx, part, rows, C, act ? 1 : 0, eps, slope, drop_p,
                            seed, site};
    hipError_t e = dadmm::launch_rownorm_bwd(a, (hipStream_t)stream);
    if (e != hipSuccess) return fail(DADMM_EHIP, "rownorm backward launch: %s", hipGetErrorString(e));
    return ok();
}

int dadmm_hyper_head_act(int32_t mode, int32_t B, int32_t H, const float* z, const float* dhyp,
                         float alpha_max, float tau_max, float rho_max, float eta_max, float* out,
                         void* stream) {
    if (B < 0 || H < 1 || (mode != 0 && mode != 1)) return fail(DADMM_EINVAL, "bad head dims/mode");
    if (!z || !out || (mode == 1 && !dhyp)) return fail(DADMM_EINVAL, "a required pointer is NULL");
    const float mx[4] = {alpha_max, tau_max, rho_max, eta_max};
    hipError_t e = dadmm::launch_head_act(mode, B, H, z, dhyp, mx, out, (hipStream_t)stream);
    if (e != hipSuccess) return fail(DADMM_EHIP, "head launch: %s", hipGetErrorString(e));
    return ok();
}

size_t dadmm_hyper_wgrad_scratch_bytes(int32_t R, int32_t N, int32_t K) {
    if (R < 0 || N < 1 || K < 1) return 0;
    const int s = dadmm::wgrad_splits(R, N, K);
    return s > 1 ? 4 * (size_t)s * N * (K + 1) : 0;
}

int dadmm_hyper_wgrad(int32_t R, int32_t N, int32_t K, const float* dz, int32_t ldz, const float* x1,
                      int32_t ld1, int32_t K1, const float* x2, int32_t ld2, float* g, float* gbias,
                      int32_t beta, void* scratch, void* stream) {
    if (R < 0 || N < 1 || K < 1 || K1 < 1 || K1 > K) return fail(DADMM_EINVAL, "bad wgrad dims R=%d N=%d K=%d K1=%d", R, N, K, K1);
    if (!dz || !x1 || !g || (K1 < K && !x2)) return fail(DADMM_EINVAL, "a required pointer is NULL");
    if (ldz < N || ld1 < K1 || (K1 < K && ld2 < K - K1)) return fail(DADMM_EINVAL, "leading dimension too small");
    if ((int64_t)R * (ldz > ld1 ? ldz : ld1) >= ((int64_t)1 << 31) || (int64_t)N * K >= ((int64_t)1 << 31))
        return fail(DADMM_EUNSUPPORTED, "operand larger than 2^31 floats");
    const int splits = dadmm::wgrad_splits(R, N, K);
    if (splits > 1 && (!scratch || !aligned16(scratch)))
        return fail(DADMM_EINVAL, "scratch (dadmm_hyper_wgrad_scratch_bytes) is NULL or not 16-byte aligned");
    if (R == 0) {
        if (beta) return ok();
        hipError_t e = hipMemsetAsync(g, 0, 4 * (size_t)N * K, (hipStream_t)stream);
        if (e == hipSuccess && gbias) e = hipMemsetAsync(gbias, 0, 4 * (size_t)N, (hipStream_t)stream);
        if (e != hipSuccess) return fail(DADMM_EHIP, "memset: %s", hipGetErrorString(e));
        return ok();
    }
    // scratch: [splits][N][K] partial tiles, [splits][N] partial bias sums
    float* part = splits > 1 ? (float*)scratch : nullptr;
    dadmm::WgradArgs a{dz, x1, K1 < K ? x2 : x1, g, gbias, part,
                       splits > 1 ? part + (size_t)splits * N * K : nullptr,
                       R, N, K, K1, ldz, ld1, K1 < K ? ld2 : ld1, splits, beta ? 1 : 0};
    hipError_t e = dadmm::launch_wgrad(a, (hipStream_t)stream);
    if (e != hipSuccess) return fail(DADMM_EHIP, "wgrad launch: %s", hipGetErrorString(e));
    return ok();
}

int dadmm_hyper_colsum(const float* part, int32_t G, int32_t R, int32_t C, float* out, int32_t beta,
                       void* stream) {
    if (G < 1 || R < 0 || C < 1) return fail(DADMM_EINVAL, "bad colsum dims G=%d R=%d C=%d", G, R, C);
    if (!out || (R > 0 && !part)) return fail(DADMM_EINVAL, "a required pointer is NULL");
    if ((int64_t)G * R * C >= ((int64_t)1 << 31)) return fail(DADMM_EUNSUPPORTED, "operand larger than 2^31 floats");
    hipError_t e = dadmm::launch_colsum(part, G, R, C, out, beta ? 1 : 0, (hipStream_t)stream);
    if (e != hipSuccess) return fail(DADMM_EHIP, "colsum launch: %s", hipGetErrorString(e));
    return ok();
}

int dadmm_hyper_transpose(int32_t rows, int32_t cols, const float* in, float* out, void* stream) {
    if (rows < 0 || cols < 0) return fail(DADMM_EINVAL, "bad transpose dims");
    if (rows == 0 || cols == 0) return ok();
    if (!in || !out) return fail(DADMM_EINVAL, "a required pointer is NULL");
    if ((int64_t)rows * cols >= ((int64_t)1 << 31)) return fail(DADMM_EUNSUPPORTED, "operand larger than 2^31 floats");
    hipError_t e = dadmm::launch_transpose(in, rows, cols, out, (hipStream_t)stream);
    if (e != hipSuccess) return fail(DADMM_EHIP, "transpose launch: %s", hipGetErrorString(e));
    return ok();
}

size_t dadmm_stepwise_scratch_bytes(const dadmm_dims* d) {
    if (check_dims(d) != DADMM_OK) return 0;
    const size_t state = align256(sizeof(float) * (size_t)d->B * d->P * d->n);
    return align256(dadmm::stepwise_flag_bytes(d->K)) + 3 * state;
}

int dadmm_forward_stepwise(const dadmm_dims* d, const void* op, const float* b,
                           const int32_t* visit_ptr, const uint8_t* visit_q, const float* deg,
                           const float* hyp, const float* y0, const float* U0, const float* d0,
                           float* Y, float* U_out, float* Grec, float* Urec, int32_t* status,
                           int32_t gate, void* scratch, void* stream) {
    int rc = check_dims(d);
    if (rc) return rc;
    if (gate & ~(DADMM_GATE_ON | DADMM_FLAGS_ZEROED)) return fail(DADMM_EINVAL, "unknown gate bits %d", gate);
    if ((gate & DADMM_GATE_ON) && status == nullptr)
        return fail(DADMM_EINVAL, "DADMM_GATE_ON needs the status word");
    if (d->B == 0 || d->K == 0) return ok();
    if (!op || !b || !visit_ptr || !visit_q || !deg || !hyp || !y0 || !U0 || !d0 || !Y || !scratch)
        return fail(DADMM_EINVAL, "a required pointer is NULL");
    if (!aligned16(op) || !aligned16(Y) || !aligned16(y0) || !aligned16(U0) || !aligned16(d0) ||
        (U_out != nullptr && !aligned16(U_out)))
        return fail(DADMM_EINVAL, "op, Y, y0, U0, d0 and U_out must be 16-byte aligned");
    if (((uintptr_t)scratch & 255u) != 0) return fail(DADMM_EINVAL, "scratch must be 256-byte aligned");
    if ((Grec == nullptr) != (Urec == nullptr))
        return fail(DADMM_EINVAL, "Grec and Urec: both or neither");
    if (Grec != nullptr && (!aligned16(Grec) || !aligned16(Urec)))
        return fail(DADMM_EINVAL, "Grec and Urec must be 16-byte aligned");
    if ((rc = check_m(d)) != DADMM_OK) return rc;
    if ((d->n & 3) != 0)
        return fail(DADMM_EUNSUPPORTED, "n=%d: needs n %% 4 == 0 (zero-pad n)", d->n);
    const size_t state = align256(sizeof(float) * (size_t)d->B * d->P * d->n);
    char* base = (char*)scratch + align256(dadmm::stepwise_flag_bytes(d->K));
    const int np = n_pad_of(d);
    dadmm::StepArgs a;
    a.A = (const float*)op;
    a.At = a.A + (size_t)d->P * m_pad_of(d) * np;
    a.b = b;
    a.vptr = visit_ptr;
    a.vq = visit_q;
    a.deg = deg;
    a.hyp = hyp;
    a.y0 = y0;
    a.U0 = U0;
    a.d0 = d0;
    a.Y = Y;
    a.D = (float*)base;
    a.G = (float*)(base + state);
    a.U = U_out != nullptr ? U_out : (float*)(base + 2 * state);
    a.flags = (int32_t*)scratch;
    a.status = status;
    a.Grec = Grec;
    a.Urec = Urec;
    a.B = d->B;
    a.P = d->P;
    a.m = d->m;
    a.m_pad = m_pad_of(d);
    a.n = d->n;
    a.n_pad = np;
    a.K = d->K;
    a.hyp_rows = d->hyp_rows;
    a.variant = d->variant;
    a.graph_shared = d->graph_shared;
    hipError_t e = dadmm::launch_stepwise(a, gate & DADMM_GATE_ON, (gate & DADMM_FLAGS_ZEROED) != 0,
                                          (hipStream_t)stream);
    if (e != hipSuccess) return fail(DADMM_EHIP, "stepwise launch: %s", hipGetErrorString(e));
    return ok();
}

}  // extern "C"
