// Probe: which Box-Muller arithmetic reproduces torch's CUDA-generator normal_ bitwise on this image?
// Variant bits: 1 = fused u/v (fma), 2 = __logf, 4 = native sqrt, 8 = accurate sincosf.
#include <hip/hip_runtime.h>
#include <hiprand/hiprand_kernel.h>
#include <stdint.h>

__global__ void bm_kernel(float* out, int64_t n, uint64_t seed, uint64_t off, int variant) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    hiprandStatePhilox4_32_10_t st;
    hiprand_init(seed, i, off, &st);
    uint4 r = hiprand4(&st);
    const float C = ROCRAND_2POW32_INV, C2 = ROCRAND_2POW32_INV_2PI;
    float u, v;
    if (variant & 1) { u = fmaf((float)r.x, C, C); v = fmaf((float)r.y, C2, C2); }
    else {
#pragma clang fp contract(off)
        u = C + ((float)r.x * C);
        v = C2 + ((float)r.y * C2);
    }
    float lg = (variant & 2) ? __logf(u) : logf(u);
    float a = -2.0f * lg;
    float s = (variant & 4) ? __builtin_amdgcn_sqrtf(a) : sqrtf(a);
    float sn, cs;
    if (variant & 8) sincosf(v, &sn, &cs); else __sincosf(v, &sn, &cs);
    out[i] = sn * s;
}

__global__ void lib_kernel(float* out, int64_t n, uint64_t seed, uint64_t off) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    hiprandStatePhilox4_32_10_t st;
    hiprand_init(seed, i, off, &st);
    out[i] = hiprand_normal4(&st).x;
}

extern "C" int bm_probe(float* out, int64_t n, uint64_t seed, uint64_t off, int variant) {
    if (variant < 0) hipLaunchKernelGGL(lib_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, out, n, seed, off);
    else hipLaunchKernelGGL(bm_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, out, n, seed, off, variant);
    return hipDeviceSynchronize() != hipSuccess;
}
