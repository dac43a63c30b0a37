// probe_rng.hip — TEST-ONLY diagnostic: Box-Muller rounding variants of hiprand_normal4 for
// Philox4x32-10, to find the evaluation torch's own build uses (scripts/rng_probe.py).
#include <hip/hip_runtime.h>
#include <hiprand/hiprand_kernel.h>
#include <stdint.h>

#define INV 2.3283064e-10f
#define INV2PI 1.46291807e-09f

__device__ float2 bm(unsigned x, unsigned y, int var) {
    float u, v;
    if (var & 1) {
        u = __builtin_fmaf((float)x, INV, INV);
        v = __builtin_fmaf((float)y, INV2PI, INV2PI);
    } else {
        u = INV + (float)x * INV;
        v = INV2PI + (float)y * INV2PI;
    }
    float l = (var & 2) ? __logf(u) : logf(u);
    float t = -2.0f * l;
    float s = (var & 4) ? __builtin_amdgcn_sqrtf(t) : sqrtf(t);
    float sn, cs;
    if (var & 8) sincosf(v, &sn, &cs);
    else __sincosf(v, &sn, &cs);
    return make_float2(sn * s, cs * s);
}

__global__ void probe(uint64_t seed, uint64_t offset, int64_t T, float* out) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= T) return;
    hiprandStatePhilox4_32_10_t st;
    hiprand_init(seed, idx, offset, &st);
    const uint4 r = hiprand4(&st);
    for (int var = 0; var < 16; ++var) {
        float2 a = bm(r.x, r.y, var), b = bm(r.z, r.w, var);
        float* o = out + (size_t)var * 4 * T;
        o[idx] = a.x; o[idx + T] = a.y; o[idx + 2 * T] = b.x; o[idx + 3 * T] = b.y;
    }
}

extern "C" int probe_rng(uint64_t seed, uint64_t offset, int64_t T, float* out) {
    hipLaunchKernelGGL(probe, dim3((T + 255) / 256), dim3(256), 0, 0, seed, offset, T, out);
    return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}
