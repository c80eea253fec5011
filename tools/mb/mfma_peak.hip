// Peak fp32 MFMA throughput probe (development tool): every wave runs ITERS x CH independent-chain
// v_mfma_f32_32x32x2_f32 from registers; 256 workgroups x WAVES waves.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float floatx16 __attribute__((ext_vector_type(16)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int CH>
__global__ void __launch_bounds__(1024) probe(float* out, int iters, float seed) {
    floatx16 acc[CH];
    for (int c = 0; c < CH; ++c)
        for (int e = 0; e < 16; ++e) acc[c][e] = 0.f;
    float a = seed * threadIdx.x, b = seed + threadIdx.x;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int c = 0; c < CH; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[c], 0, 0, 0);
    }
    float s = 0.f;
    for (int c = 0; c < CH; ++c)
        for (int e = 0; e < 16; ++e) s += acc[c][e];
    if (s == 12345.f) out[threadIdx.x] = s;
}

template <int CH>
int run(int waves, int iters) {
    float* out;
    CK(hipMalloc(&out, 4096));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(probe<CH>, dim3(256), dim3(64 * waves), 0, 0, out, iters, 1.f);
    CK(hipEventRecord(e0));
    const int reps = 10;
    for (int w = 0; w < reps; ++w) hipLaunchKernelGGL(probe<CH>, dim3(256), dim3(64 * waves), 0, 0, out, iters, 1.f);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    const double fl = 2.0 * 32 * 32 * 2 * 64.0 / 64 * CH * iters * waves * 256.0 * reps;   // 4096 flop per MFMA per wave
    printf("chains %d waves/WG %2d: %8.2f us/launch  %6.1f TFLOP/s  (%.1f cycles per MFMA per SIMD at 2.4 GHz)\n", CH, waves,
           ms * 1e3 / reps, fl / (ms * 1e-3) / 1e12, (ms * 1e-3 / reps) * 2.4e9 / (CH * iters * waves / 4.0));
    return 0;
}

int main() {
    run<1>(8, 2048); run<2>(8, 1024); run<4>(8, 512); run<2>(4, 1024); run<4>(4, 512); run<1>(16, 2048); run<2>(16, 1024);
    return 0;
}
