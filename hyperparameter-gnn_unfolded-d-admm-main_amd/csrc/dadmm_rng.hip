// dadmm_rng.hip — the forward's prologue: the reference's random inits and the per-forward
// zeroing of the guard words, in ONE launch.
//
// The reference draws y_k, U_k, delta = torch.randn((B, P, n, 1)) * 1e-2, in that order
// (unfolded_DLASSO.py:49-51). On a ROCm device that is three calls of torch's Philox normal
// kernel (ATen/native/hip/DistributionTemplates.h, distribution_elementwise_grid_stride_kernel
// with unroll 4): a grid of G blocks of 256 threads; virtual thread idx runs hiprand_init(seed,
// subsequence = idx, offset) and, for it = 0, 1, ..., writes hiprand_normal4's four values to
// elements idx + T (4 it + ii) (T = 256 G); each call advances the generator's offset by
// 4 ceil(numel / 4T). This kernel replays exactly that mapping for all three tensors at once (one
// real thread per virtual idx, drawing for the three tensors), so its output is bit-identical to
//   torch.randn(shape) * 1e-2  ==  torch.empty(shape).normal_(0, 1e-2)
// (tests/test_gpu_parity.py::test_prologue_draws_match_torch), and zeroes `nzero` int32 words
// (the status word and the stepwise guard flags) — replacing 3 RNG launches, 2 fills and a memset.
// Outputs may use a padded row length n_store >= n (padding columns are left untouched).

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dadmm_internal.h"

namespace dadmm {
namespace {

// hiprand_normal4 (rocrand box_muller on the four Philox words) evaluated exactly as torch's own
// build of it rounds — established on the device by tests/hip/probe_rng.hip + scripts/rng_probe.py
// over 2M draws: the uniforms u, v contracted to one fma each, then logf, a correctly rounded
// sqrtf, __sincosf and two separately rounded products (this file: -ffp-contract=off).
__device__ __forceinline__ float2 box_muller(unsigned x, unsigned y) {
    const float u = __builtin_fmaf((float)x, 2.3283064e-10f, 2.3283064e-10f);     // ROCRAND_2POW32_INV
    const float v = __builtin_fmaf((float)y, 1.46291807e-09f, 1.46291807e-09f);   // ..._INV_2PI
    const float s = sqrtf(-2.0f * logf(u));
    float sn, cs;
    __sincosf(v, &sn, &cs);
    return make_float2(sn * s, cs * s);
}


// The Philox counter of draw `it` of virtual thread idx is formed directly
// (rocrand's engine state after hiprand_init(seed, idx, offset) and `it` next4() calls: counter =
// (offset / 4 + it, subsequence idx) as a 128-bit sum, key = seed) and its ten rounds evaluated
// once. hiprand4 also evaluates the NEXT counter eagerly after each call, one Philox of four per
// thread that no element uses; and the last draw's second Box-Muller pair is skipped when none of
// its elements exists. Same words, same floats (offset % 4 == 0, so next4 never interleaves).

// The launch is bound by these rounds (~60 % of its time at the headline shape), so each round
// is 2 v_mad_u64_u32 (both halves of a product in one instruction; __umulhi plus a separate low
// multiply compiled to v_mul_hi_u32 + v_mul_lo_u32) and 2 gfx950 v_bitop3_b32 (LUT 0x96 =
// a ^ b ^ c; LLVM leaves the 3-way xors as pairs of v_xor_b32). The key word is wave-uniform.
// Same integer results.
__device__ __forceinline__ unsigned xor3(unsigned a, unsigned b, unsigned c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint4 philox_round(uint4 c, uint2 k) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
    return make_uint4(xor3((unsigned)(p1 >> 32), c.y, k.x), (unsigned)p1,
                      xor3((unsigned)(p0 >> 32), c.w, k.y), (unsigned)p0);
}

__device__ __forceinline__ uint4 philox10(uint4 c, uint2 k) {
#pragma unroll
    for (int r = 0; r < 9; ++r) {
        c = philox_round(c, k);
        k.x += 0x9E3779B9u;   // ROCRAND_PHILOX_W32_0
        k.y += 0xBB67AE85u;   // ROCRAND_PHILOX_W32_1
    }
    return philox_round(c, k);
}

// 32-bit index arithmetic (numel < 2^31 is checked by the launcher): the 64-bit divisions of a
// straightforward port cost more than the Philox rounds themselves.
// One real thread per virtual thread idx draws for all three tensors (round 6): the three
// counters' Philox rounds are independent, so they interleave in one instruction stream, and the
// grid is torch's T threads (2048 workgroups of 256 on 256 CUs: one dispatch round) instead of
// 3 T. At B = 1024 every virtual thread draws one block per tensor, and the 6,144 short
// workgroups of the per-(tensor, idx) form were paced by workgroup dispatch, not by the rounds.
template <bool PADDED>
__global__ __launch_bounds__(256) void prologue_kernel(PrologueArgs a) {
    const uint32_t gid = blockIdx.x * 256u + threadIdx.x;
    for (uint32_t i = gid; i < (uint32_t)a.nzero; i += gridDim.x * 256u) a.zero[i] = 0;
    if (a.numel == 0) return;
    const uint32_t T = (uint32_t)a.threads;       // torch's 256 G virtual threads per tensor
    if (gid >= T) return;
    const uint32_t idx = gid;
    float* const out[3] = {a.y0, a.U0, a.d0};
    const uint32_t numel = (uint32_t)a.numel, n = (uint32_t)a.n, ns = (uint32_t)a.n_store;
    const uint32_t iters = (numel - 1) / (T * 4) + 1;
    auto put = [&](int t, uint32_t li, float v) {
        uint32_t o = li;
        if (PADDED) {
            const uint32_t row = li / n;
            o = row * ns + (li - row * n);
        }
        // transformation::normal (val * std + mean), contracted as torch's build does
        out[t][o] = __builtin_fmaf(v, a.stddev, a.mean);
    };
    // tensor t's counter after discard_subsequence(idx) then discard(offset_t): (x, y) =
    // offset_t / 4, (z, w) = idx plus the carry out of y; offset_t = offset + t * offset_step
    // (the generator advanced by each torch call in turn)
    uint64_t c0[3];
#pragma unroll
    for (int t = 0; t < 3; ++t) c0[t] = (a.offset + (uint64_t)t * a.offset_step) / 4;
    const uint2 key = make_uint2((unsigned)a.seed, (unsigned)(a.seed >> 32));
    uint32_t li = idx;
    for (uint32_t it = 0; it < iters; ++it, li += 4 * T) {
        uint4 r[3];
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            const uint64_t cx = c0[t] + it;                   // the counter's low 64 bits
            const unsigned carry = cx < c0[t] ? 1u : 0u;      // into the subsequence words
            r[t] = philox10(make_uint4((unsigned)cx, (unsigned)(cx >> 32), idx + carry,
                                       (idx + carry < idx) ? 1u : 0u), key);
        }
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            const float2 p0 = box_muller(r[t].x, r[t].y);
            if (li < numel) put(t, li, p0.x);
            if (li + T < numel) put(t, li + T, p0.y);
            if (li + 2 * T < numel) {
                const float2 p1 = box_muller(r[t].z, r[t].w);
                put(t, li + 2 * T, p1.x);
                if (li + 3 * T < numel) put(t, li + 3 * T, p1.y);
            }
        }
    }
}

}  // namespace

hipError_t launch_prologue(const PrologueArgs& a, hipStream_t stream) {
    int64_t work = a.numel > 0 ? a.threads : 0;
    if (work < a.nzero) work = a.nzero < 2048 * 256 ? a.nzero : 2048 * 256;   // the zeroing strides
    if (work == 0) return hipSuccess;
    if (a.numel >= ((int64_t)1 << 31) || work >= ((int64_t)1 << 31)) return hipErrorInvalidValue;
    if (a.n_store != a.n)
        hipLaunchKernelGGL(prologue_kernel<true>, dim3((unsigned)((work + 255) / 256)), dim3(256), 0,
                           stream, a);
    else
        hipLaunchKernelGGL(prologue_kernel<false>, dim3((unsigned)((work + 255) / 256)), dim3(256), 0,
                           stream, a);
    return hipGetLastError();
}

}  // namespace dadmm
