// dadmm_hyper_net.cpp — host orchestration of one training-mode hypernetwork call of
// DLASSO_GNNHyp3_Progressive (gnn_dlasso_models_progressive.py:165-196 with :52-72 in train mode)
// and of its backward, as ONE C-ABI call each: the 13 forward launches and ~35 backward launches
// of an iteration are issued from here instead of one Python / ctypes round trip each
// (dadmm_hip.hyper_ops, VERDICT r2 weak #6: the train step was host-bound on ~2,700 launches).
//
// Forward, per iteration (B samples of P nodes, rows = B P):
//   x_i = Dropout(BN_batch(leaky(A_hat (x_{i-1} W_i^T) + b_i)))   5 x dadmm_hyper_gcn_train
//   e   = LayerNorm(x_5)                                          dadmm_hyper_rownorm
//   d_j = LReLU(LN(Dropout(d_{j-1} D_j^T + c_j)))                 3 x dadmm_hyper_linear_ln_train
//   z   = d_3 fc^T + f; hyp = head(z)                             dadmm_hyper_linear, _head_act
// Backward: the same stages reversed; the parameter gradients are accumulated IN PLACE into the
// caller's buffers (dadmm_hyper_wgrad / dadmm_hyper_colsum: G += ...), the input gradients run as
// dadmm_hyper_linear with the caller's transposed weights. Everything is enqueued on `stream`;
// nothing here allocates or synchronises.

#include <stdint.h>
#include <string.h>

#include "../../include/dadmm.h"
#include "dadmm_internal.h"

namespace {

constexpr float LEAKY = 0.01f;   // F.leaky_relu's default slope (reference :52-68)

inline size_t up16(size_t b) { return (b + 15) & ~(size_t)15; }

struct Work {   // carve of the caller's work buffer (dadmm_hyper_train_work_bytes)
    float* dz;      // [B][4H]
    float* dx[2];   // [rows][max width] ping-pong
    float* dv;      // [B][max decoder width]
    float* part;    // max(3 B N, rownorm partials)
    float* wscr;    // dadmm_hyper_wgrad split partials
    float* lscr;    // dadmm_hyper_linear_ln_train split-K partials
};

int max_width(const dadmm_hyper_net* net) {
    int w = 2 * net->n;
    for (int i = 0; i < 5; ++i) w = w > net->width[i] ? w : net->width[i];
    return w;
}

size_t layout(const dadmm_hyper_net* net, int B, Work* w, char* base) {
    const int P = net->P, rows = B * P;
    const int mw = max_width(net);
    int md = net->dec_width[0];
    for (int j = 1; j < 3; ++j) md = md > net->dec_width[j] ? md : net->dec_width[j];
    size_t part = (size_t)3 * B * (mw > md ? mw : md);
    const size_t rn1 = dadmm_hyper_rownorm_bwd_part_bytes(rows, net->width[4]) / 4;
    part = part > rn1 ? part : rn1;
    for (int j = 0; j < 3; ++j) {
        const size_t r = dadmm_hyper_rownorm_bwd_part_bytes(B, net->dec_width[j]) / 4;
        part = part > r ? part : r;
    }
    // scratch: the largest split partials of any weight gradient; of any decoder linear
    size_t scr = 0, lscr = 0;
    int kin = 2 * net->n;
    for (int i = 0; i < 5; ++i) {
        const size_t s = dadmm_hyper_wgrad_scratch_bytes(rows, net->width[i], kin);
        scr = scr > s ? scr : s;
        kin = net->width[i];
    }
    int din = P * net->width[4];
    for (int j = 0; j < 3; ++j) {
        size_t s = dadmm_hyper_wgrad_scratch_bytes(B, net->dec_width[j], din);
        scr = scr > s ? scr : s;
        s = dadmm_hyper_linear_ln_scratch_bytes(B, din, net->dec_width[j]);
        lscr = lscr > s ? lscr : s;
        din = net->dec_width[j];
    }
    {
        const size_t s = dadmm_hyper_wgrad_scratch_bytes(B, 4 * net->H, din);
        scr = scr > s ? scr : s;
    }
    const size_t sizes[7] = {up16(scr + 16), up16(4 * (size_t)B * 4 * net->H), up16(4 * (size_t)rows * mw),
                             up16(4 * (size_t)rows * mw), up16(4 * (size_t)B * md), up16(4 * part), up16(lscr + 16)};
    size_t off = 0;
    float** slots[7] = {&w->wscr, &w->dz, &w->dx[0], &w->dx[1], &w->dv, &w->part, &w->lscr};
    for (int i = 0; i < 7; ++i) {
        if (base) *slots[i] = (float*)(base + off);
        off += sizes[i];
    }
    return off;
}

int check_net(const dadmm_hyper_net* net, int B) {
    if (!net || B < 0 || net->P < 2 || net->P > 64 || net->n < 1 || net->ld < net->n || net->H < 1)
        return DADMM_EINVAL;
    for (int i = 0; i < 5; ++i)
        if (net->width[i] < 4 || (net->width[i] & 3) || !net->conv_w[i] || !net->conv_b[i] || !net->bn_w[i] ||
            !net->bn_b[i])
            return DADMM_EINVAL;
    for (int j = 0; j < 3; ++j)
        if (net->dec_width[j] < 4 || (net->dec_width[j] & 3) || !net->dec_w[j] || !net->dec_b[j] ||
            !net->ln_w[j] || !net->ln_b[j])
            return DADMM_EINVAL;
    if (!net->norm_w || !net->norm_b || !net->fc_w || !net->fc_b) return DADMM_EINVAL;
    return DADMM_OK;
}

#define TRY(call)                       \
    do {                                \
        const int rc_ = (call);         \
        if (rc_ != DADMM_OK) return rc_; \
    } while (0)

}  // namespace

extern "C" {

size_t dadmm_hyper_train_work_bytes(const dadmm_hyper_net* net, int32_t B) {
    if (check_net(net, B) != DADMM_OK) return 0;
    Work w;
    return layout(net, B, &w, nullptr);
}

int dadmm_hyper_train_forward(const dadmm_hyper_net* net, int32_t B, const float* AtAy, const float* Atb,
                              const float* ahat, int32_t ahat_per_sample, uint64_t seed,
                              const dadmm_hyper_saved* sv, void* work, void* stream) {
    if (check_net(net, B) != DADMM_OK || !sv || !work) return DADMM_EINVAL;
    if (B == 0) return DADMM_OK;
    Work w;
    layout(net, B, &w, (char*)work);
    const int P = net->P, n = net->n, rows = B * P;
    // layer 1 reads cat(AtAy, Atb) in place (two segments; the kernels need 16-column segments)
    const float* x1 = AtAy;
    const float* x2 = Atb;
    int ld1 = net->ld, ld2 = net->ld, K1 = n, K = 2 * n;
    if (n & 15) return DADMM_EUNSUPPORTED;   // the caller concatenates in that case (dadmm_hip)
    for (int i = 0; i < 5; ++i) {
        const int N = net->width[i];
        TRY(dadmm_hyper_gcn_train(B, P, K, N, x1, ld1, K1, x2, ld2, net->conv_w[i], net->conv_b[i], ahat,
                                  ahat_per_sample, net->bn_w[i], net->bn_b[i], net->bn_eps[i], LEAKY,
                                  i < 4 ? net->drop_enc : 0.0f, seed, i, sv->y[i], N, sv->m[i], sv->mean[i],
                                  sv->var[i], stream));
        x1 = sv->y[i];
        ld1 = N;
        K1 = N;
        K = N;
        x2 = nullptr;
        ld2 = 0;
    }
    // self.norm (:69) over 4h per node -> the flattened decoder input [B][P 4h]
    const int C = net->width[4];
    TRY(dadmm_hyper_rownorm(rows, C, sv->y[4], net->norm_w, net->norm_b, net->norm_eps, 0, 0.0f, sv->e, stream));
    const float* x = sv->e;
    int width = P * C;
    for (int j = 0; j < 3; ++j) {
        const int N = net->dec_width[j];
        TRY(dadmm_hyper_linear_ln_train(B, width, N, x, width, net->dec_w[j], net->dec_b[j], net->ln_w[j],
                                        net->ln_b[j], net->ln_eps[j], 1, net->dec_slope[j], net->dec_drop[j],
                                        seed, 4 + j, sv->dec_y[j], sv->dec_xd[j], w.lscr, stream));
        x = sv->dec_y[j];
        width = N;
    }
    const int H4 = 4 * net->H;
    TRY(dadmm_hyper_linear(B, width, H4, x, width, width, nullptr, 0, net->fc_w, net->fc_b, sv->z, H4, stream));
    TRY(dadmm_hyper_head_act(0, B, net->H, sv->z, nullptr, net->maxv[0], net->maxv[1], net->maxv[2],
                             net->maxv[3], sv->hyp, stream));
    return DADMM_OK;
}

int dadmm_hyper_train_backward(const dadmm_hyper_net* net, int32_t B, const float* AtAy, const float* Atb,
                               const float* ahat, int32_t ahat_per_sample, uint64_t seed,
                               const dadmm_hyper_saved* sv, const float* dhyp, const dadmm_hyper_grads* g,
                               float* dAtAy, void* work, void* stream) {
    if (check_net(net, B) != DADMM_OK || !sv || !dhyp || !g || !dAtAy || !work) return DADMM_EINVAL;
    if (B == 0) return DADMM_OK;
    Work w;
    layout(net, B, &w, (char*)work);
    const int P = net->P, n = net->n, rows = B * P, H4 = 4 * net->H;
    if (n & 15) return DADMM_EUNSUPPORTED;
    // head (sigmoid, clamps, maxima) -> d logits
    TRY(dadmm_hyper_head_act(1, B, net->H, sv->z, dhyp, net->maxv[0], net->maxv[1], net->maxv[2],
                             net->maxv[3], w.dz, stream));
    // fc: dW, db; dx = dz fc
    const int hid = net->dec_width[2];
    TRY(dadmm_hyper_wgrad(B, H4, hid, w.dz, H4, sv->dec_y[2], hid, hid, nullptr, 0, g->fc_w, g->fc_b, 1, w.wscr,
                          stream));
    float* dx = w.dx[0];
    TRY(dadmm_hyper_linear(B, H4, hid, w.dz, H4, H4, nullptr, 0, g->fc_wt, nullptr, dx, hid, stream));
    // decoder blocks, last to first
    for (int j = 2; j >= 0; --j) {
        const int N = net->dec_width[j];
        const int Kin = j > 0 ? net->dec_width[j - 1] : P * net->width[4];
        const float* xin = j > 0 ? sv->dec_y[j - 1] : sv->e;
        TRY(dadmm_hyper_rownorm_bwd(B, N, dx, sv->dec_xd[j], net->ln_w[j], net->ln_b[j], net->ln_eps[j], 1,
                                    net->dec_slope[j], net->dec_drop[j], seed, 4 + j, w.dv, w.part, stream));
        const int nblk = (int)(dadmm_hyper_rownorm_bwd_part_bytes(B, N) / (4 * 2 * (size_t)N));
        TRY(dadmm_hyper_colsum(w.part, 1, nblk, 2 * N, g->ln_wb[j], 1, stream));
        TRY(dadmm_hyper_wgrad(B, N, Kin, w.dv, N, xin, Kin, Kin, nullptr, 0, g->dec_w[j], g->dec_b[j], 1, w.wscr,
                              stream));
        float* nx = dx == w.dx[0] ? w.dx[1] : w.dx[0];
        TRY(dadmm_hyper_linear(B, N, Kin, w.dv, N, N, nullptr, 0, g->dec_wt[j], nullptr, nx, Kin, stream));
        dx = nx;
    }
    // self.norm backward (no dropout, no activation): dx [B][P 4h] = [rows][4h]
    const int C = net->width[4];
    {
        float* nx = dx == w.dx[0] ? w.dx[1] : w.dx[0];
        TRY(dadmm_hyper_rownorm_bwd(rows, C, dx, sv->y[4], net->norm_w, net->norm_b, net->norm_eps, 0, 0.0f, 0.0f,
                                    seed, 99, nx, w.part, stream));
        const int nblk = (int)(dadmm_hyper_rownorm_bwd_part_bytes(rows, C) / (4 * 2 * (size_t)C));
        TRY(dadmm_hyper_colsum(w.part, 1, nblk, 2 * C, g->norm_wb, 1, stream));
        dx = nx;
    }
    // GCN layers, last to first: dZ (gcn backward), [dgamma, dbeta, dbias], dW, dX
    for (int i = 4; i >= 0; --i) {
        const int N = net->width[i];
        float* dZ = dx == w.dx[0] ? w.dx[1] : w.dx[0];
        TRY(dadmm_hyper_gcn_train_bwd(B, P, N, dx, sv->m[i], sv->mean[i], sv->var[i], net->bn_w[i],
                                      net->bn_eps[i], ahat, ahat_per_sample, LEAKY, i < 4 ? net->drop_enc : 0.0f,
                                      seed, i, dZ, w.part, stream));
        TRY(dadmm_hyper_colsum(w.part, 3, B, N, g->bn_wbc[i], 1, stream));
        if (i > 0) {
            const int Kin = net->width[i - 1];
            TRY(dadmm_hyper_wgrad(rows, N, Kin, dZ, N, sv->y[i - 1], Kin, Kin, nullptr, 0, g->conv_w[i], nullptr,
                                  1, w.wscr, stream));
            // dX into the buffer dx held (gcn backward consumed it)
            TRY(dadmm_hyper_linear(rows, N, Kin, dZ, N, N, nullptr, 0, g->conv_wt[i], nullptr, dx, Kin, stream));
        } else {
            // layer 1's input cat(AtAy, Atb); only d AtAy (its first n columns) flows back
            TRY(dadmm_hyper_wgrad(rows, N, 2 * n, dZ, N, AtAy, net->ld, n, Atb, net->ld, g->conv_w[0], nullptr,
                                  1, w.wscr, stream));
            TRY(dadmm_hyper_linear(rows, N, n, dZ, N, N, nullptr, 0, g->conv_wt[0], nullptr, dAtAy, net->ld,
                                   stream));
        }
    }
    return DADMM_OK;
}

}  // extern "C"
