// dadmm_hyper_train.hip — training-mode backward of the GNN hypernetwork of
// DLASSO_GNNHyp3_Progressive (gnn_dlasso_models_progressive.py:9-72 GNNHypernetwork3, :93-123
// decoder / fc, :165-196 head), everything but the plain GEMMs:
//   gcn_bwd_kernel    : one GCN block  Dropout(BN_batch(leaky(A_hat Z + bias)))  from dy to dZ,
//                       with per-sample partial sums of dgamma, dbeta, dbias;
//   rownorm_bwd_kernel: LayerNorm (+ LeakyReLU) rows from dy to dx (through the decoder's
//                       Dropout when it has one), with per-block partial sums of dweight, dbias;
//   head_act_kernel   : the hyper-parameter head (sigmoid, clamps, maxima) forward and backward.
// The forward kernels are the train epilogues of dadmm_hyper.hip (HYPER_EPI_GCN_TRAIN and the
// rownorm dropout); the dropout masks are regenerated here from the same counter-based stream
// (drop_hash), never stored. The weight / input gradients of the linears (dW = dZ^T X,
// dX = dZ W) are plain GEMMs: dadmm_hyper_grad.hip (wgrad_kernel) and dadmm_hyper.hip's linear
// with the transposed weight.
//
// Every formula is the derivative torch's autograd applies to the reference's modules:
//   Dropout: dx = dy * keep / (1 - p);   leaky_relu: dx = dy * (x > 0 ? 1 : slope);
//   BatchNorm (batch statistics of the P nodes of a sample, biased variance):
//     dx = gamma rstd (dxn - mean(dxn) - xhat mean(dxn xhat)),  dgamma = sum dxn xhat, dbeta = sum dxn;
//   BatchNorm in eval mode (running statistics: constants): dx = gamma rstd dxn, same dgamma / dbeta;
//   LayerNorm over C columns: the same with the row's statistics and per-column affine;
//   clamp(x, lo, hi): dx = dy * (lo <= x <= hi);  sigmoid: dx = dy * s (1 - s).
// Sums run in fixed orders (deterministic); results agree with torch to f32 rounding.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dadmm_internal.h"

namespace dadmm {
namespace hyper_train {

typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int THREADS = 256;
constexpr int CB = 64;   // columns per gcn_bwd workgroup
// gcn_bwd workgroup size NT: its passes 1-2 use one lane per column (64), so at 256 threads three
// waves idle until the mix. When the grid fills the chip (>= GCNBWD_WIDE_MIN workgroups) the
// one-wave form wins on throughput (B = 4096 train step 61.2 -> 56.6 ms); on small grids the
// 4-wave mix's shorter per-lane chain wins (B = 256: 10.3 vs 10.8-11.6 ms). Same sums either way.
constexpr int GCNBWD_WIDE_MIN = 2048;
// PR: at P <= PR agents a lane's rows are loaded at once into registers (0: the per-row loop)
constexpr int GCNBWD_PR = 8;

// One workgroup per (sample, 64 columns). LDS: M, then dM [P][CB]; A_hat block [P][P].
template <int NT, int PR>
__global__ __launch_bounds__(NT) void gcn_bwd_kernel(GcnBwdArgs a) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int P = a.P, N = a.N;
    const int ncb = (N + CB - 1) / CB;
    const int s = blockIdx.x / ncb, c0 = (blockIdx.x % ncb) * CB;
    float* dm = lds;                 // [P][CB]
    float* ah = dm + P * CB;         // [P][P]
    const float* ahg = a.ahat + (a.ahat_per_sample ? (size_t)s * P * P : 0);
    for (int i = threadIdx.x; i < P * P; i += NT) ah[i] = ahg[i];
    const size_t row0 = (size_t)s * P;
    const uint32_t thr = drop_threshold(a.drop_p);
    const float scale = a.drop_p > 0.0f ? 1.0f / (1.0f - a.drop_p) : 1.0f;
    if (threadIdx.x < CB && c0 + (int)threadIdx.x < N) {
        const int c = c0 + threadIdx.x;
        const float mean = a.mean[(size_t)s * N + c];
        const float rstd = 1.0f / sqrtf(a.var[(size_t)s * N + c] + a.eps);
        const float gam = a.gamma[c];
        float sb = 0.0f, sg = 0.0f, sbias = 0.0f;
        if constexpr (PR > 0) {
            // P <= PR: every row's M and dY loaded at once (rows past P re-read row P - 1, unused),
            // so the lane waits for memory once instead of once per row; same sums, same order
            float mr[PR], gr[PR], xr[PR];
#pragma unroll
            for (int p = 0; p < PR; ++p) {
                const size_t o = (row0 + (p < P ? p : P - 1)) * N + c;
                mr[p] = a.m[o];
                gr[p] = a.dy[o];
            }
#pragma unroll
            for (int p = 0; p < PR; ++p) {
                if (p >= P) break;
                const float mv = mr[p];
                const float t = mv > 0.0f ? mv : mv * a.slope;
                xr[p] = (t - mean) * rstd;
                float g = gr[p];
                if (a.drop_p > 0.0f)
                    g = drop_hash(a.seed, a.site, (uint32_t)(row0 + p), (uint32_t)c) >= thr ? g * scale : 0.0f;
                sb += g;
                sg += g * xr[p];
                gr[p] = g;
            }
            // eval-mode BatchNorm (running statistics): the mean / var are constants, dt = gamma rstd dy
            const float inv = a.bn_eval ? 0.0f : 1.0f / (float)P;
#pragma unroll
            for (int p = 0; p < PR; ++p) {
                if (p >= P) break;
                const float dt = a.bn_eval ? gam * rstd * gr[p] : gam * rstd * (gr[p] - sb * inv - xr[p] * (sg * inv));
                const float d = mr[p] > 0.0f ? dt : dt * a.slope;
                sbias += d;
                dm[p * CB + threadIdx.x] = d;
            }
        } else {
            // pass 1: dxn = dropout'(dy), the two BatchNorm sums
            for (int p = 0; p < P; ++p) {
                const size_t o = (row0 + p) * N + c;
                const float mv = a.m[o];
                const float t = mv > 0.0f ? mv : mv * a.slope;
                const float xh = (t - mean) * rstd;
                float g = a.dy[o];
                if (a.drop_p > 0.0f)
                    g = drop_hash(a.seed, a.site, (uint32_t)(row0 + p), (uint32_t)c) >= thr ? g * scale : 0.0f;
                sb += g;
                sg += g * xh;
                dm[p * CB + threadIdx.x] = g;
            }
            // pass 2: BatchNorm and leaky_relu backward -> dM
            const float inv = 1.0f / (float)P;
            for (int p = 0; p < P; ++p) {
                const size_t o = (row0 + p) * N + c;
                const float mv = a.m[o];
                const float t = mv > 0.0f ? mv : mv * a.slope;
                const float xh = (t - mean) * rstd;
                const float g = dm[p * CB + threadIdx.x];
                const float dt = a.bn_eval ? gam * rstd * g : gam * rstd * (g - sb * inv - xh * (sg * inv));
                const float d = mv > 0.0f ? dt : dt * a.slope;
                sbias += d;
                dm[p * CB + threadIdx.x] = d;
            }
        }
        a.part[(size_t)s * N + c] = sg;                          // dgamma
        a.part[((size_t)a.B + s) * N + c] = sb;                  // dbeta
        a.part[((size_t)2 * a.B + s) * N + c] = sbias;           // dbias (GCNConv.bias)
    }
    __syncthreads();
    // dZ[q] = sum_p A_hat[p][q] dM[p]  (the mix M = A_hat Z, transposed)
    const int cols = N - c0 < CB ? N - c0 : CB;
    for (int task = threadIdx.x; task < P * CB; task += NT) {
        const int q = task / CB, c = task - q * CB;
        if (c >= cols) continue;
        float acc = 0.0f;
        for (int p = 0; p < P; ++p) acc += ah[p * P + q] * dm[p * CB + c];
        a.dz[(row0 + q) * N + c0 + c] = acc;
    }
}

// One wave per row, ROWNORM_BWD_ROWS rows per workgroup (2 per wave); per-lane column partials
// of dweight / dbias are combined across the 4 waves in LDS in wave order (deterministic).
// CH: 256-column chunks per lane (C <= 256 CH; the launcher picks the smallest). Round 4: the
// wave's rows, dy rows and the affine parameters are loaded up front and unconditionally (columns
// past C read column C - 1, a row past the last reads the last row; their terms are selected
// away), so the wave waits for memory once instead of twice per row — the per-row load / reduce /
// load chain at small batches was latency-bound (7.9 us per call at B = 256). Same operations in
// the same order as before: bit-identical.
template <int CH>
__global__ __launch_bounds__(THREADS) void rownorm_bwd_kernel(RowNormBwdArgs a) {
    __shared__ __attribute__((aligned(16))) float red[4][2][2048];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int C = a.C, C4 = C / 4;
    constexpr int RPW = ROWNORM_BWD_ROWS / 4;
    const f32x4 z4 = {0.0f, 0.0f, 0.0f, 0.0f};
    f32x4 pw[CH], pb[CH];
#pragma unroll
    for (int u = 0; u < CH; ++u) pw[u] = pb[u] = z4;
    const uint32_t thr = drop_threshold(a.drop_p);
    const float scale = a.drop_p > 0.0f ? 1.0f / (1.0f - a.drop_p) : 1.0f;
    const float invC = 1.0f / (float)C;
    bool cok[CH];
    int cc[CH];
    f32x4 wv[CH], bv[CH];
#pragma unroll
    for (int u = 0; u < CH; ++u) {
        const int c4 = lane + 64 * u;
        cok[u] = c4 < C4;
        cc[u] = cok[u] ? c4 : C4 - 1;
        wv[u] = *(const f32x4*)(a.weight + 4 * cc[u]);
        bv[u] = *(const f32x4*)(a.bias + 4 * cc[u]);
    }
    f32x4 xr[RPW][CH], dr[RPW][CH];
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
        const int row = blockIdx.x * ROWNORM_BWD_ROWS + w * RPW + i;
        const int rc = row < a.rows ? row : a.rows - 1;
#pragma unroll
        for (int u = 0; u < CH; ++u) {
            xr[i][u] = *(const f32x4*)(a.xd + (size_t)rc * C + 4 * cc[u]);
            dr[i][u] = *(const f32x4*)(a.dy + (size_t)rc * C + 4 * cc[u]);
        }
    }
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
        const int row = blockIdx.x * ROWNORM_BWD_ROWS + w * RPW + i;
        if (row >= a.rows) break;
        f32x4 v[CH], g[CH];
        float s = 0.0f;
#pragma unroll
        for (int u = 0; u < CH; ++u) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[u][e] = cok[u] ? xr[i][u][e] : 0.0f;
            s += (v[u][0] + v[u][1]) + (v[u][2] + v[u][3]);
        }
        s = ln_row_sum(s);
        const float mean = s * invC;
        float q = 0.0f;
#pragma unroll
        for (int u = 0; u < CH; ++u) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float d = v[u][e] - mean;
                const float dd = d * d;
                q = cok[u] ? q + dd : q;
            }
        }
        q = ln_row_sum(q);
        const float rstd = 1.0f / sqrtf(q * invC + a.eps);
        // xhat, dt (through the LeakyReLU), the affine partials, dxhat and its two row sums
        float s1 = 0.0f, s2 = 0.0f;
#pragma unroll
        for (int u = 0; u < CH; ++u) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float xh = (v[u][e] - mean) * rstd;
                float dt = dr[i][u][e];
                if (a.act) {
                    const float t = xh * wv[u][e] + bv[u][e];
                    dt = t > 0.0f ? dt : dt * a.slope;
                }
                const float dxh = dt * wv[u][e];
                if (cok[u]) {
                    pw[u][e] += dt * xh;
                    pb[u][e] += dt;
                    s1 += dxh;
                    s2 += dxh * xh;
                }
                v[u][e] = xh;
                g[u][e] = dxh;
            }
        }
        s1 = ln_row_sum(s1);
        s2 = ln_row_sum(s2);
        const float m1 = s1 * invC, m2 = s2 * invC;
        float* dx = a.dx + (size_t)row * C;
#pragma unroll
        for (int u = 0; u < CH; ++u) {
            const int c4 = lane + 64 * u;
            if (!cok[u]) continue;
            f32x4 o;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float d = rstd * (g[u][e] - m1 - v[u][e] * m2);
                if (a.drop_p > 0.0f)
                    d = drop_hash(a.seed, a.site, (uint32_t)row, (uint32_t)(4 * c4 + e)) >= thr ? d * scale : 0.0f;
                o[e] = d;
            }
            *(f32x4*)(dx + 4 * c4) = o;
        }
    }
#pragma unroll
    for (int u = 0; u < CH; ++u) {
        const int c4 = lane + 64 * u;
        if (c4 < C4) {
            *(f32x4*)(&red[w][0][4 * c4]) = pw[u];
            *(f32x4*)(&red[w][1][4 * c4]) = pb[u];
        }
    }
    __syncthreads();
    float* part = a.part + (size_t)blockIdx.x * 2 * C;
    for (int i = threadIdx.x; i < 2 * C; i += THREADS) {
        const int k = i / C, c = i - k * C;
        part[i] = ((red[0][k][c] + red[1][k][c]) + red[2][k][c]) + red[3][k][c];
    }
}

// mode 0: out = hyp = head(z); mode 1: out = dz = dhyp * head'(z). Element (b, i) of [B][4H],
// channel c = i / H (the reference's h.view(B, 4, H)):
//   s = sigmoid(z); u = clamp(s, 1e-4, 0.9999); v = u * max_c; hyp = c > 0 ? min(v, 0.9999) : v
__global__ __launch_bounds__(THREADS) void head_act_kernel(int mode, int B, int H, const float* z,
                                                           const float* dhyp, float m0, float m1,
                                                           float m2, float m3, float* out) {
    const int idx = blockIdx.x * THREADS + threadIdx.x;
    if (idx >= B * 4 * H) return;
    const int c = (idx % (4 * H)) / H;
    const float mx = c == 0 ? m0 : (c == 1 ? m1 : (c == 2 ? m2 : m3));
    const float s = 1.0f / (1.0f + expf(-z[idx]));
    const float u = fminf(fmaxf(s, 1e-4f), 0.9999f);
    const float v = u * mx;
    if (mode == 0) {
        out[idx] = c > 0 ? fminf(v, 0.9999f) : v;
        return;
    }
    float g = dhyp[idx];
    if (c > 0 && !(v <= 0.9999f)) g = 0.0f;           // clamp(max=0.9999)
    g = g * mx;
    if (!(s >= 1e-4f && s <= 0.9999f)) g = 0.0f;      // clamp(1e-4, 0.9999)
    out[idx] = g * ((1.0f - s) * s);                   // sigmoid
}

// BatchNorm running statistics in closed form (dadmm_hyper_bn_running_update). Pass 1: workgroup
// (64-column block of the concatenated layers, split s) — lane = column, wave = a quarter of the
// split's rows — sums w[t] mean[t][c] and w[t] var[t][c] P / (P - 1) over its rows in float64
// (coalesced along the columns); the 4 waves add in wave order (LDS). Pass 2: per column, the
// splits in order, plus decay * the old value. Deterministic.
// the layer of column block cb (64 columns; blocks never straddle layers) and its pointers,
// selected with uniform branches (no dynamic indexing of the kernel-argument arrays)
__device__ inline int bn_layer_of_block(const BnRunArgs& a, int cb, int* c0) {
    int L = 0, first = 0;
#pragma unroll
    for (int i = 0; i < BN_MAX_LAYERS; ++i) {
        if (i >= a.layers) break;
        const int nb = (a.width[i] + 63) / 64;
        if (cb < first + nb) {
            L = i;
            break;
        }
        first += nb;
    }
    *c0 = (cb - first) * 64;
    return L;
}

template <class T, int S>
__device__ inline T bn_pick(const T (&arr)[S], int L) {
    T r = arr[0];
#pragma unroll
    for (int i = 1; i < S; ++i)
        if (L == i) r = arr[i];
    return r;
}

// partial weighted sums: block (cb, sp) covers 64 columns of one layer and rows t of split sp;
// the 4 waves take interleaved quarters of the split and reduce through LDS (fixed order)
__global__ __launch_bounds__(256) void bn_running_part_kernel(BnRunArgs a) {
    __shared__ double red[4][2][64];
    const int total = a.col0[a.layers];
    const int sp = blockIdx.y;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int c0;
    const int L = bn_layer_of_block(a, blockIdx.x, &c0);
    const int N = bn_pick(a.width, L);
    const float* __restrict__ mean = bn_pick(a.mean, L);
    const float* __restrict__ var = bn_pick(a.var, L);
    const int cc = c0 + lane;
    const int T = a.iters * a.B;
    const int per = (T + a.splits - 1) / a.splits;
    const int t0 = sp * per, t1 = t0 + per < T ? t0 + per : T;
    const double uf = (double)a.P / (double)(a.P - 1);
    double sm = 0.0, sv = 0.0;
    if (cc < N) {
        // the wave's rows t0 + wv, + 4, ...: their offsets first, then the loads in groups of 8 in
        // flight, then the sums in row order (the same order as one row at a time)
        int k = t0 / a.B, b = t0 - k * a.B + wv;
        while (b >= a.B) { b -= a.B; ++k; }
        for (int t = t0 + wv; t < t1; t += 32) {
            float mv[8], vv[8];
            double wt[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const bool in = t + 4 * u < t1;
                const size_t o = (size_t)k * a.block_stride + (size_t)b * N + cc;
                mv[u] = in ? mean[o] : 0.0f;
                vv[u] = in ? var[o] : 0.0f;
                wt[u] = in ? a.w[t + 4 * u] : 0.0;
                b += 4;
                while (b >= a.B) { b -= a.B; ++k; }
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                if (t + 4 * u < t1) {
                    sm += wt[u] * (double)mv[u];
                    sv += wt[u] * ((double)vv[u] * uf);
                }
            }
        }
    }
    red[wv][0][lane] = sm;
    red[wv][1][lane] = sv;
    __syncthreads();
    if (wv == 0 && cc < N) {
        double m = red[0][0][lane], v = red[0][1][lane];
        for (int q = 1; q < 4; ++q) {
            m += red[q][0][lane];
            v += red[q][1][lane];
        }
        const int c = bn_pick(a.col0, L) + cc;
        a.part[((size_t)sp * 2) * total + c] = m;
        a.part[((size_t)sp * 2 + 1) * total + c] = v;
    }
}

__global__ __launch_bounds__(256) void bn_running_finish_kernel(BnRunArgs a) {
    const int total = a.col0[a.layers];
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= total) return;
    int L = 0;
#pragma unroll
    for (int i = 1; i < BN_MAX_LAYERS; ++i)
        if (i < a.layers && c >= a.col0[i]) L = i;
    const int cc = c - bn_pick(a.col0, L);
    double m = 0.0, v = 0.0;
    for (int sp0 = 0; sp0 < a.splits; sp0 += 8) {   // 8 splits' loads in flight, added in order
        double pm[8], pv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int sp = sp0 + u < a.splits ? sp0 + u : a.splits - 1;
            pm[u] = a.part[((size_t)sp * 2) * total + c];
            pv[u] = a.part[((size_t)sp * 2 + 1) * total + c];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (sp0 + u < a.splits) {
                m += pm[u];
                v += pv[u];
            }
    }
    float* rm = bn_pick(a.rmean, L);
    float* rv = bn_pick(a.rvar, L);
    rm[cc] = (float)(a.decay * (double)rm[cc] + m);
    rv[cc] = (float)(a.decay * (double)rv[cc] + v);
    int64_t* tr = bn_pick(a.tracked, L);
    if (cc == 0 && tr != nullptr) tr[0] += (int64_t)a.iters * a.B;
}

}  // namespace hyper_train

hipError_t launch_bn_running(const BnRunArgs& a, hipStream_t st) {
    const int total = a.col0[a.layers];
    if (total == 0) return hipSuccess;
    int blocks = 0;
    for (int i = 0; i < a.layers; ++i) blocks += (a.width[i] + 63) / 64;
    hipLaunchKernelGGL(hyper_train::bn_running_part_kernel, dim3(blocks, a.splits), dim3(256), 0, st, a);
    hipLaunchKernelGGL(hyper_train::bn_running_finish_kernel, dim3((total + 255) / 256), dim3(256), 0, st, a);
    return hipGetLastError();
}

template <int NT, int PR>
static hipError_t launch_gcn_bwd_nt(const GcnBwdArgs& a, int grid, size_t lds, hipStream_t st) {
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute((const void*)hyper_train::gcn_bwd_kernel<NT, PR>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL((hyper_train::gcn_bwd_kernel<NT, PR>), dim3(grid), dim3(NT), lds, st, a);
    return hipGetLastError();
}

hipError_t launch_gcn_bwd(const GcnBwdArgs& a, hipStream_t st) {
    if (a.B <= 0 || a.N <= 0) return hipSuccess;
    const size_t lds = 4 * ((size_t)a.P * hyper_train::CB + (size_t)a.P * a.P);
    const int ncb = (a.N + hyper_train::CB - 1) / hyper_train::CB;
    const int grid = a.B * ncb;
    constexpr int T4 = hyper_train::THREADS;
    if (a.P <= hyper_train::GCNBWD_PR)
        return grid >= hyper_train::GCNBWD_WIDE_MIN ? launch_gcn_bwd_nt<64, hyper_train::GCNBWD_PR>(a, grid, lds, st)
                                             : launch_gcn_bwd_nt<T4, hyper_train::GCNBWD_PR>(a, grid, lds, st);
    return grid >= hyper_train::GCNBWD_WIDE_MIN ? launch_gcn_bwd_nt<64, 0>(a, grid, lds, st)
                                         : launch_gcn_bwd_nt<T4, 0>(a, grid, lds, st);
}

hipError_t launch_rownorm_bwd(const RowNormBwdArgs& a, hipStream_t st) {
    if (a.rows <= 0) return hipSuccess;
    const int nblk = (a.rows + ROWNORM_BWD_ROWS - 1) / ROWNORM_BWD_ROWS;
    if (a.C > 2048) return hipErrorInvalidValue;
    const dim3 g(nblk), b(hyper_train::THREADS);
    if (a.C <= 256) hipLaunchKernelGGL(hyper_train::rownorm_bwd_kernel<1>, g, b, 0, st, a);
    else if (a.C <= 512) hipLaunchKernelGGL(hyper_train::rownorm_bwd_kernel<2>, g, b, 0, st, a);
    else if (a.C <= 1024) hipLaunchKernelGGL(hyper_train::rownorm_bwd_kernel<4>, g, b, 0, st, a);
    else hipLaunchKernelGGL(hyper_train::rownorm_bwd_kernel<8>, g, b, 0, st, a);
    return hipGetLastError();
}

hipError_t launch_head_act(int mode, int B, int H, const float* z, const float* dhyp, const float* maxv4,
                           float* out, hipStream_t st) {
    const int n = B * 4 * H;
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(hyper_train::head_act_kernel, dim3((n + hyper_train::THREADS - 1) / hyper_train::THREADS),
                       dim3(hyper_train::THREADS), 0, st, mode, B, H, z, dhyp, maxv4[0], maxv4[1],
                       maxv4[2], maxv4[3], out);
    return hipGetLastError();
}

}  // namespace dadmm
