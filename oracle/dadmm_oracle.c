/*
 * dadmm_oracle.c — CPU restatement of the reference's unfolded D-ADMM forward.
 *
 * TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may load this library, and only as the checker / the CPU baseline — never as the product path.
 *
 * Parity status: UNPINNED by reference outputs. The reference's own repository holds no test
 * vectors for this path and importing/running the reference was denied in
 * this environment. This restatement is written from the reference source text
 * and is pinned instead by known-answer tests derived from that text (tests/test_oracle.py) and
 * by the reference's shipped data fixtures (A.pt singular values, model.pt hyper-parameters).
 *
 * Two restatements of DLASSO_unfolded.forward (unfolded_DLASSO.py:34-140), both including the
 * reference's batch-global NaN/Inf guards (:55-61, :84-86, :102-104) and both variants:
 *   variant 0  unfolded_DLASSO.py:79-99            (k-dependent clamps, no delta clamp)
 *   variant 1  gnn_dlasso_models_progressive.py:205-237 (fixed clamps, delta clamped to +-20)
 *
 *  oracle_forward_f64  the reference's algorithm in double precision, in the reference's form:
 *                      AtA = A^T A precomputed (:16), Atb = A^T b (:45), grad uses AtA@y (:69-71).
 *  oracle_forward_f32  the same recurrence in float, evaluated in the EXACT operation order of the
 *                      HIP kernel: factored gradient A^T(A y - b) as single fma chains whose
 *                      reduction index visits 0,4,8,12,1,5,9,13,2,6,10,14,3,7,11,15 inside every
 *                      16-block (blocks ascending); GEMM1 chains start at -b, GEMM2 chains at +0;
 *                      every other operation rounds on its own, as the torch eager ops do.
 *  oracle_forward_f32_split  the same with GEMM1 in the order of the column-split forward
 *                      (dadmm_split.hip, small batches): the n columns cut into slices of
 *                      split_cols; slice s's chain (same visiting order) starts at -b for s = 0
 *                      and at +0 otherwise, and R = ((c_0 + c_1) + c_2) + ... left to right.
 *                      Built with -ffp-contract=off; fmaf is the C99 correctly rounded fma.
 *
 * compute_delta (:127-140) is restated literally for both: for p in 0..P-1, for q in
 * neighbors(p) (the order of the caller's adjacency lists): diff = y_p - y_q; delta[p] += diff;
 * delta[q] -= diff.
 *
 * hyp layouts: hyp_mode 0 -> [K][H][4] (seq_hyperparam table, H = P or 1);
 *              hyp_mode 1 -> [K][B][4][H] (GNN hypernetwork output per sample, view(B,4,H)).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

#define ORACLE_ABI_VERSION 1

int oracle_abi_version(void) { return ORACLE_ABI_VERSION; }

/* OpenMP team size of the restatements (the CPU-baseline legs time 1 thread and all host threads) */
int oracle_set_threads(int t) {
#ifdef _OPENMP
    if (t > 0) omp_set_num_threads(t);
    return omp_get_max_threads();
#else
    (void)t;
    return 1;
#endif
}

static int perm16(int idx) { return (idx & ~15) + 4 * (idx & 3) + ((idx & 15) >> 2); }

static void hyp_at(int hyp_mode, int H, int B, const float* hyp, int k, int s, int p, float out[4]) {
    const int hp = (H == 1) ? 0 : p;
    if (hyp_mode == 0) {
        const float* r = hyp + ((size_t)k * H + hp) * 4;
        out[0] = r[0]; out[1] = r[1]; out[2] = r[2]; out[3] = r[3];
    } else {
        const float* r = hyp + ((size_t)k * B + s) * 4 * H;
        for (int c = 0; c < 4; ++c) out[c] = r[c * H + hp];
    }
}

/* torch.clamp semantics: NaN propagates, +-inf saturate */
static float clampf_t(float x, float lo, float hi) {
    if (x != x) return x;
    return x < lo ? lo : (x > hi ? hi : x);
}
static double clampd_t(double x, double lo, double hi) {
    if (x != x) return x;
    return x < lo ? lo : (x > hi ? hi : x);
}
static float signf_t(float x) { return (float)((0.0f < x) - (x < 0.0f)); }
static double signd_t(double x) { return (double)((0.0 < x) - (x < 0.0)); }

/* ------------------------------------------------------------------------------------------ */
/* Grec / Urec (nullable, [K][B][P][n]): the trajectory the adjoint needs — the gradient of iteration
 * k BEFORE its clamp (unfolded_DLASSO.py:73-77) and U_k entering iteration k (after the :59 guard). */
static int forward_f32_impl(int B, int P, int m, int n, int K, int variant, int hyp_mode, int H,
                            const float* A, const float* b, const int32_t* nbr_ptr,
                            const int32_t* nbr_idx, const float* deg, const float* hyp,
                            const float* y0, const float* U0, const float* d0, float* Y,
                            float* U_out, int32_t* status, float* Grec, float* Urec,
                            int gram_mode, int split_cols) {
    if (B < 0 || P < 1 || m < 1 || n < 1 || K < 0 || (H != 1 && H != P)) return -1;
    const size_t S = (size_t)B * P * n;
    float* y = (float*)malloc(S * sizeof(float));
    float* U = (float*)malloc(S * sizeof(float));
    float* dl = (float*)malloc(S * sizeof(float));
    float* yn = (float*)malloc(S * sizeof(float));
    float* gr = (float*)malloc(S * sizeof(float));
    if (!y || !U || !dl || !yn || !gr) {
        free(y); free(U); free(dl); free(yn); free(gr);
        return -2;
    }
    memcpy(y, y0, S * sizeof(float));
    memcpy(U, U0, S * sizeof(float));
    memcpy(dl, d0, S * sizeof(float));
    int32_t st = 0;
    const int npad = (n + 15) & ~15, mpad = (m + 15) & ~15;

    for (int k = 0; k < K; ++k) {
        const float gclip = variant == 0 ? fmaxf(1.0f, 30.0f - (float)k) : 10.0f;
        const float vclip = variant == 0 ? fmaxf(10.0f, 200.0f - (float)(3 * k)) : 100.0f;
        /* :55-61 */
        int bad_y = 0, bad_u = 0;
        for (size_t i = 0; i < S; ++i) {
            bad_y |= !isfinite(y[i]);
            bad_u |= !isfinite(U[i]);
        }
        if (bad_y) { memset(y, 0, S * sizeof(float)); st |= 1; }
        if (bad_u) { memset(U, 0, S * sizeof(float)); st |= 2; }
        if (Urec) memcpy(Urec + (size_t)k * S, U, S * sizeof(float));

        int bad_g = 0;
#pragma omp parallel for schedule(static) reduction(| : bad_g)
        for (int s = 0; s < B; ++s) {
            float* R = (float*)malloc((size_t)m * sizeof(float));
            for (int p = 0; p < P; ++p) {
                float h4[4];
                hyp_at(hyp_mode, H, B, hyp, k, s, p, h4);
                const float* Ap = A + (size_t)p * m * n;
                const float* yp = y + ((size_t)s * P + p) * n;
                const float* bp = b + ((size_t)s * P + p) * m;
                /* GEMM1: R = A_p y_p - b_p, one fma chain per row from -b
                 * (gram_mode: R = A_p y_p from +0, b enters through Atb below) */
                for (int i = 0; i < m; ++i) {
                    float acc = gram_mode ? 0.0f : -bp[i];
                    if (split_cols > 0) {
                        /* column-split order: one chain per slice, slice 0's from -b, the others
                         * from +0, summed left to right */
                        float r = 0.0f;
                        for (int c0 = 0; c0 < npad; c0 += split_cols) {
                            float part = c0 == 0 ? acc : 0.0f;
                            for (int idx = c0; idx < c0 + split_cols && idx < npad; ++idx) {
                                const int c = perm16(idx);
                                if (c < n) part = fmaf(Ap[(size_t)i * n + c], yp[c], part);
                            }
                            r = c0 == 0 ? part : r + part;
                        }
                        R[i] = r;
                        continue;
                    }
                    for (int idx = 0; idx < npad; ++idx) {
                        const int c = perm16(idx);
                        if (c < n) acc = fmaf(Ap[(size_t)i * n + c], yp[c], acc);
                    }
                    R[i] = acc;
                }
                const float dg = deg[(size_t)s * P + p];
                for (int c = 0; c < n; ++c) {
                    /* GEMM2: A_p^T R, one fma chain per column from +0 */
                    float g = 0.0f;
                    for (int idx = 0; idx < mpad; ++idx) {
                        const int i = perm16(idx);
                        if (i < m) g = fmaf(Ap[(size_t)i * n + c], R[i], g);
                    }
                    const size_t e = ((size_t)s * P + p) * n + c;
                    if (gram_mode) {
                        /* GNN model (gnn_dlasso_models_progressive.py:205-209): AtAy - Atb with
                         * Atb = A_p^T b_p as its own chain from +0 */
                        float atb = 0.0f;
                        for (int idx = 0; idx < mpad; ++idx) {
                            const int i = perm16(idx);
                            if (i < m) atb = fmaf(Ap[(size_t)i * n + c], bp[i], atb);
                        }
                        g = g - atb;
                    }
                    /* :73-77 left to right */
                    float t = g + signf_t(y[e]) * h4[1];
                    t = t + U[e] * dg;
                    t = t + dl[e] * h4[2];
                    if (Grec) Grec[(size_t)k * S + e] = t;
                    t = clampf_t(t, -gclip, gclip); /* :80-81 */
                    bad_g |= (t != t);
                    gr[e] = t;
                }
            }
            free(R);
        }
        /* :84-86 (after the clamp only NaN can remain) */
        if (bad_g) { memset(gr, 0, S * sizeof(float)); st |= 4; }

        int bad_v = 0;
        for (int s = 0; s < B; ++s)
            for (int p = 0; p < P; ++p) {
                float h4[4];
                hyp_at(hyp_mode, H, B, hyp, k, s, p, h4);
                for (int c = 0; c < n; ++c) {
                    const size_t e = ((size_t)s * P + p) * n + c;
                    float v = y[e] - h4[0] * gr[e];     /* :89 */
                    v = clampf_t(v, -vclip, vclip);     /* :92-93 */
                    bad_v |= (v != v);
                    yn[e] = v;
                }
            }
        /* compute_delta(y_next) :95, :127-140 */
        memset(dl, 0, S * sizeof(float));
        for (int s = 0; s < B; ++s)
            for (int p = 0; p < P; ++p)
                for (int t = nbr_ptr[(size_t)s * P + p]; t < nbr_ptr[(size_t)s * P + p + 1]; ++t) {
                    const int q = nbr_idx[t];
                    float* dp = dl + ((size_t)s * P + p) * n;
                    float* dq = dl + ((size_t)s * P + q) * n;
                    const float* yp = yn + ((size_t)s * P + p) * n;
                    const float* yq = yn + ((size_t)s * P + q) * n;
                    for (int c = 0; c < n; ++c) {
                        const float diff = yp[c] - yq[c];
                        dp[c] = dp[c] + diff;
                        dq[c] = dq[c] - diff;
                    }
                }
        if (variant != 0)
            for (size_t i = 0; i < S; ++i) dl[i] = clampf_t(dl[i], -20.0f, 20.0f); /* GNN :229 */
        /* :98-99 */
        for (int s = 0; s < B; ++s)
            for (int p = 0; p < P; ++p) {
                float h4[4];
                hyp_at(hyp_mode, H, B, hyp, k, s, p, h4);
                for (int c = 0; c < n; ++c) {
                    const size_t e = ((size_t)s * P + p) * n + c;
                    U[e] = clampf_t(U[e] + dl[e] * h4[3], -vclip, vclip);
                }
            }
        /* :102-104 */
        if (bad_v) st |= 8;
        else memcpy(y, yn, S * sizeof(float));
        memcpy(Y + (size_t)k * S, y, S * sizeof(float));
    }
    if (U_out) memcpy(U_out, U, S * sizeof(float));
    if (status) *status = st;
    free(y); free(U); free(dl); free(yn); free(gr);
    return 0;
}

int oracle_forward_f32(int B, int P, int m, int n, int K, int variant, int hyp_mode, int H,
                       const float* A, const float* b, const int32_t* nbr_ptr,
                       const int32_t* nbr_idx, const float* deg, const float* hyp,
                       const float* y0, const float* U0, const float* d0, float* Y, float* U_out,
                       int32_t* status) {
    return forward_f32_impl(B, P, m, n, K, variant, hyp_mode, H, A, b, nbr_ptr, nbr_idx, deg, hyp,
                            y0, U0, d0, Y, U_out, status, NULL, NULL, 0, 0);
}

/* oracle_forward_f32 with GEMM1 in the column-split order (split_cols: a multiple of 16). */
int oracle_forward_f32_split(int B, int P, int m, int n, int K, int variant, int hyp_mode, int H,
                             const float* A, const float* b, const int32_t* nbr_ptr,
                             const int32_t* nbr_idx, const float* deg, const float* hyp,
                             const float* y0, const float* U0, const float* d0, float* Y,
                             float* U_out, int32_t* status, int split_cols) {
    if (split_cols < 0 || (split_cols & 15)) return -1;
    return forward_f32_impl(B, P, m, n, K, variant, hyp_mode, H, A, b, nbr_ptr, nbr_idx, deg, hyp,
                            y0, U0, d0, Y, U_out, status, NULL, NULL, 0, split_cols);
}

/* oracle_forward_f32 that also records the adjoint's trajectory (Grec, Urec: [K][B][P][n]). */
int oracle_forward_f32_rec(int B, int P, int m, int n, int K, int variant, int hyp_mode, int H,
                           const float* A, const float* b, const int32_t* nbr_ptr,
                           const int32_t* nbr_idx, const float* deg, const float* hyp,
                           const float* y0, const float* U0, const float* d0, float* Y,
                           float* U_out, int32_t* status, float* Grec, float* Urec) {
    return forward_f32_impl(B, P, m, n, K, variant, hyp_mode, H, A, b, nbr_ptr, nbr_idx, deg, hyp,
                            y0, U0, d0, Y, U_out, status, Grec, Urec, 0, 0);
}

/* The GNN model's recurrence in the order of the per-iteration HIP path (dadmm_gnn.hip): gradient
 * ((((AtAy - Atb) + sign*tau) + U*deg) + delta*rho) with AtAy = A^T (A y) and Atb = A^T b as
 * separate fma chains. Usually hyp_mode 1 (the hypernetwork's per-sample [K][B][4][H]). */
int oracle_forward_f32_gram(int B, int P, int m, int n, int K, int variant, int hyp_mode, int H,
                            const float* A, const float* b, const int32_t* nbr_ptr,
                            const int32_t* nbr_idx, const float* deg, const float* hyp,
                            const float* y0, const float* U0, const float* d0, float* Y,
                            float* U_out, int32_t* status) {
    return forward_f32_impl(B, P, m, n, K, variant, hyp_mode, H, A, b, nbr_ptr, nbr_idx, deg, hyp,
                            y0, U0, d0, Y, U_out, status, NULL, NULL, 1, 0);
}

/* ------------------------------------------------------------------------------------------ */
int oracle_forward_f64(int B, int P, int m, int n, int K, int variant, int hyp_mode, int H,
                       const float* A, const float* b, const int32_t* nbr_ptr,
                       const int32_t* nbr_idx, const float* deg, const float* hyp,
                       const float* y0, const float* U0, const float* d0, double* Y,
                       double* U_out, int32_t* status) {
    if (B < 0 || P < 1 || m < 1 || n < 1 || K < 0 || (H != 1 && H != P)) return -1;
    const size_t S = (size_t)B * P * n;
    double* AtA = (double*)calloc((size_t)P * n * n, sizeof(double));
    double* Atb = (double*)calloc(S, sizeof(double));
    double* y = (double*)malloc(S * sizeof(double));
    double* U = (double*)malloc(S * sizeof(double));
    double* dl = (double*)malloc(S * sizeof(double));
    double* yn = (double*)malloc(S * sizeof(double));
    double* gr = (double*)malloc(S * sizeof(double));
    if (!AtA || !Atb || !y || !U || !dl || !yn || !gr) {
        free(AtA); free(Atb); free(y); free(U); free(dl); free(yn); free(gr);
        return -2;
    }
    /* self.AtA = compute_Atx(self.A) (:16, :120-124) */
#pragma omp parallel for schedule(static)
    for (int p = 0; p < P; ++p)
        for (int i = 0; i < n; ++i)
            for (int j = 0; j < n; ++j) {
                double acc = 0.0;
                for (int r = 0; r < m; ++r)
                    acc += (double)A[((size_t)p * m + r) * n + i] * (double)A[((size_t)p * m + r) * n + j];
                AtA[((size_t)p * n + i) * n + j] = acc;
            }
    /* Atb = compute_Atx(b) (:45) */
#pragma omp parallel for schedule(static)
    for (int s = 0; s < B; ++s)
        for (int p = 0; p < P; ++p)
            for (int i = 0; i < n; ++i) {
                double acc = 0.0;
                for (int r = 0; r < m; ++r)
                    acc += (double)A[((size_t)p * m + r) * n + i] * (double)b[((size_t)s * P + p) * m + r];
                Atb[((size_t)s * P + p) * n + i] = acc;
            }
    for (size_t i = 0; i < S; ++i) {
        y[i] = y0[i];
        U[i] = U0[i];
        dl[i] = d0[i];
    }
    int32_t st = 0;
    for (int k = 0; k < K; ++k) {
        const double gclip = variant == 0 ? fmax(1.0, 30.0 - k) : 10.0;
        const double vclip = variant == 0 ? fmax(10.0, 200.0 - 3.0 * k) : 100.0;
        int bad_y = 0, bad_u = 0;
        for (size_t i = 0; i < S; ++i) {
            bad_y |= !isfinite(y[i]);
            bad_u |= !isfinite(U[i]);
        }
        if (bad_y) { for (size_t i = 0; i < S; ++i) y[i] = 0.0; st |= 1; }
        if (bad_u) { for (size_t i = 0; i < S; ++i) U[i] = 0.0; st |= 2; }
        int bad_g = 0;
#pragma omp parallel for schedule(static) reduction(| : bad_g)
        for (int s = 0; s < B; ++s)
            for (int p = 0; p < P; ++p) {
                float h4[4];
                hyp_at(hyp_mode, H, B, hyp, k, s, p, h4);
                const double dg = deg[(size_t)s * P + p];
                const double* yp = y + ((size_t)s * P + p) * n;
                for (int i = 0; i < n; ++i) {
                    double acc = 0.0; /* AtAy[:, p] = AtA[0,p] @ y[:, p] (:69-71) */
                    const double* row = AtA + ((size_t)p * n + i) * n;
                    for (int j = 0; j < n; ++j) acc += row[j] * yp[j];
                    const size_t e = ((size_t)s * P + p) * n + i;
                    double t = acc - Atb[e];
                    t = t + signd_t(y[e]) * (double)h4[1];
                    t = t + U[e] * dg;
                    t = t + dl[e] * (double)h4[2];
                    t = clampd_t(t, -gclip, gclip);
                    bad_g |= (t != t);
                    gr[e] = t;
                }
            }
        if (bad_g) { for (size_t i = 0; i < S; ++i) gr[i] = 0.0; st |= 4; }
        int bad_v = 0;
        for (int s = 0; s < B; ++s)
            for (int p = 0; p < P; ++p) {
                float h4[4];
                hyp_at(hyp_mode, H, B, hyp, k, s, p, h4);
                for (int c = 0; c < n; ++c) {
                    const size_t e = ((size_t)s * P + p) * n + c;
                    double v = clampd_t(y[e] - (double)h4[0] * gr[e], -vclip, vclip);
                    bad_v |= (v != v);
                    yn[e] = v;
                }
            }
        for (size_t i = 0; i < S; ++i) dl[i] = 0.0;
        for (int s = 0; s < B; ++s)
            for (int p = 0; p < P; ++p)
                for (int t = nbr_ptr[(size_t)s * P + p]; t < nbr_ptr[(size_t)s * P + p + 1]; ++t) {
                    const int q = nbr_idx[t];
                    for (int c = 0; c < n; ++c) {
                        const double diff = yn[((size_t)s * P + p) * n + c] - yn[((size_t)s * P + q) * n + c];
                        dl[((size_t)s * P + p) * n + c] += diff;
                        dl[((size_t)s * P + q) * n + c] -= diff;
                    }
                }
        if (variant != 0)
            for (size_t i = 0; i < S; ++i) dl[i] = clampd_t(dl[i], -20.0, 20.0);
        for (int s = 0; s < B; ++s)
            for (int p = 0; p < P; ++p) {
                float h4[4];
                hyp_at(hyp_mode, H, B, hyp, k, s, p, h4);
                for (int c = 0; c < n; ++c) {
                    const size_t e = ((size_t)s * P + p) * n + c;
                    U[e] = clampd_t(U[e] + dl[e] * (double)h4[3], -vclip, vclip);
                }
            }
        if (bad_v) st |= 8;
        else memcpy(y, yn, S * sizeof(double));
        memcpy(Y + (size_t)k * S, y, S * sizeof(double));
    }
    if (U_out) memcpy(U_out, U, S * sizeof(double));
    if (status) *status = st;
    free(AtA); free(Atb); free(y); free(U); free(dl); free(yn); free(gr);
    return 0;
}
