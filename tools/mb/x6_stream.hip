// x6 weight-stream probe (development tool, not shipped): what bounds the x6 chain kernel's M x M layer.
// Each wave runs the chain kernel's own inner loop (ring6_run / ring6x2_run from tdmpc_kernels.hip) over a
// K = 512 layer of the x6 weight layout, REPS times, and variants strip parts of it:
//   P  production loop: weights streamed from the L2-resident panel (one 1.5 MB panel per head, 2 heads)
//   M  MFMA only (operands in registers)
//   S  MFMA + LDS reads + the activation split (no global loads)
//   L  MFMA + weight loads (no split, no LDS reads)
// Shapes: "r32" = 4-wave workgroups x TN 4 (the bench kernel, two per CU), "r64" = 8-wave x TN 2 x 2 row tiles
// (chain64, one per CU). Prints us per launch and MFMA busy = MFMA cycles per SIMD / elapsed shader cycles.
#include "../../tdmpc_amd/csrc/tdmpc_kernels.hip"
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

enum { VP = 0, VM = 1, VS = 2, VL = 3 };

template <int TN, int TR, int D, int V>
DEVI void probe_loop(floatx16 (&acc)[TN][TR], uint4 (&wr)[D][TN][3], const float* sA, const unsigned short* Wp,
                     long wbs, int G, int r, int h) {
    const int gl = G - 1;
    const float* ap = sA + (h * 32 + r) * 4;
    float4 n0 = *(const float4*)ap, n1 = *(const float4*)(ap + 256);
    for (int gb = 0; gb < G; gb += D) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const int g = gb + d;
            bf16x8_t bh, bm, bl;
            if constexpr (V == VS) {
                const float4 a0 = n0, a1 = n1;
                const size_t gn = (size_t)min(g + 1, gl) * 512;
                n0 = *(const float4*)(ap + gn);
                n1 = *(const float4*)(ap + gn + 256);
                __builtin_amdgcn_sched_barrier(0);
                split8(a0, a1, bh, bm, bl);
            } else {
                bh = as_bf16x8(make_uint4(__float_as_uint(n0.x), g, 2, 3));
                bm = as_bf16x8(make_uint4(__float_as_uint(n0.y), 1, g, 3));
                bl = as_bf16x8(make_uint4(__float_as_uint(n1.x), 1, 2, g));
            }
#pragma unroll
            for (int t = 0; t < TR; ++t)
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    acc[j][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(wr[d][j][1]), bm, acc[j][t], 0, 0, 0);
                    acc[j][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(wr[d][j][2]), bh, acc[j][t], 0, 0, 0);
                    acc[j][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(wr[d][j][0]), bl, acc[j][t], 0, 0, 0);
                    acc[j][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(wr[d][j][1]), bh, acc[j][t], 0, 0, 0);
                    acc[j][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(wr[d][j][0]), bm, acc[j][t], 0, 0, 0);
                    acc[j][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(wr[d][j][0]), bh, acc[j][t], 0, 0, 0);
                }
            if constexpr (V == VL) {
#pragma unroll
                for (int j = 0; j < TN; ++j)
#pragma unroll
                    for (int p = 0; p < 3; ++p)
                        wr[d][j][p] = *(const uint4*)(Wp + j * wbs + ((size_t)min(g + D, gl) * 3 + p) * 512);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    }
}

template <int TN, int TR, int D, int NW, int V>
__global__ void __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(2)))
probe(const unsigned short* X, float* out, unsigned long long* clk, int reps) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 31, h = lane >> 5;
    for (int i = tid; i < TR * 16384; i += 64 * NW) smem[i] = 1e-3f * (float)((i * 7) % 113);
    lds_barrier();
    const int G = 32;
    const long wb = (long)G * 1536;                     // one 32-column block of a K = 512 x6 panel
    const int head = blockIdx.x & 1;
    const unsigned short* Wp = X + (size_t)head * 16 * wb + (size_t)(wave * TN) * wb + lane * 8;
    unsigned long long c0 = 0, t0 = 0;
    if (tid == 0 && blockIdx.x == 0) { c0 = __builtin_amdgcn_s_memtime(); t0 = __builtin_amdgcn_s_memrealtime(); }
    floatx16 acc[TN][TR];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int t = 0; t < TR; ++t)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[j][t][e] = 0.f;
    uint4 wr[D][TN][3];
    for (int rep = 0; rep < reps; ++rep) {
        ring6_fill<TN, D>(wr, Wp, wb, 0, G);
        if constexpr (V == VP) {
            if constexpr (TR == 1) {
                floatx16 a1[TN];
#pragma unroll
                for (int j = 0; j < TN; ++j) a1[j] = acc[j][0];
                ring6_run<TN, D>(a1, wr, smem, Wp, wb, 0, G, r, h);
#pragma unroll
                for (int j = 0; j < TN; ++j) acc[j][0] = a1[j];
            } else {
                ring6x2_run<TN, D>(acc, wr, smem, 16384, Wp, wb, 0, G, r, h);
            }
        } else {
            probe_loop<TN, TR, D, V>(acc, wr, smem, Wp, wb, G, r, h);
        }
    }
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int t = 0; t < TR; ++t)
#pragma unroll
            for (int e = 0; e < 16; ++e) s += acc[j][t][e];
    if (s == 12345.f) out[tid] = s;
    if (tid == 0 && blockIdx.x == 0) {
        clk[0] = __builtin_amdgcn_s_memtime() - c0;
        clk[1] = __builtin_amdgcn_s_memrealtime() - t0;
    }
}

template <int TN, int TR, int D, int NW, int V>
void run(const char* name, const unsigned short* X, float* out, unsigned long long* clk, int nwg, int reps) {
    auto k = probe<TN, TR, D, NW, V>;
    const size_t lds = (size_t)TR * 16384 * 4;
    CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(k, dim3(nwg), dim3(64 * NW), lds, 0, X, out, clk, reps);
    CK(hipGetLastError());
    const int it = 5;
    CK(hipEventRecord(e0));
    for (int w = 0; w < it; ++w) hipLaunchKernelGGL(k, dim3(nwg), dim3(64 * NW), lds, 0, X, out, clk, reps);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    unsigned long long c[2];
    CK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
    const double us = ms * 1e3 / it;
    const double ghz = c[1] ? (double)c[0] / (double)c[1] * 0.1 : 0.0;   // s_memrealtime runs at 100 MHz
    const double mfma_per_simd = (double)nwg * NW * reps * 32 * 6 * TN * TR / 1024.0;
    const double busy = mfma_per_simd * 32.0 / (us * 1e3 * (ghz > 0 ? ghz : 2.1));
    const double wbytes = (double)nwg * NW * reps * 32 * TN * 3 * 1024;
    printf("%-26s wg %4d x %d waves  %9.2f us  clock %.2f GHz  MFMA busy %.3f  weights %.1f GB/s per CU\n", name, nwg,
           NW, us, ghz, busy, wbytes / (us * 1e3) / 256.0);
}

int main() {
    const size_t xb = (size_t)2 * 16 * 32 * 1536 * 2;   // two heads x 16 blocks x K 512 in the x6 layout
    unsigned short* X; float* out; unsigned long long* clk;
    CK(hipMalloc(&X, xb)); CK(hipMalloc(&out, 4096 * 4)); CK(hipMalloc(&clk, 16));
    {
        std::vector<unsigned short> hx(xb / 2);
        for (size_t i = 0; i < hx.size(); ++i) hx[i] = (unsigned short)(0x3c00 + (i * 2654435761u >> 24) % 64);
        CK(hipMemcpy(X, hx.data(), xb, hipMemcpyHostToDevice));
    }
    const int reps = 8;
    // the bench kernel's geometry: 1024 four-wave workgroups (4 per CU over the launch, 2 co-resident)
    run<4, 1, 2, 4, VM>("r32 D2 mfma only", X, out, clk, 1024, reps);
    run<4, 1, 2, 4, VS>("r32 D2 mfma+lds+split", X, out, clk, 1024, reps);
    run<4, 1, 2, 4, VL>("r32 D2 mfma+loads", X, out, clk, 1024, reps);
    run<4, 1, 2, 4, VP>("r32 D2 production", X, out, clk, 1024, reps);
    run<4, 1, 1, 4, VL>("r32 D1 mfma+loads", X, out, clk, 1024, reps);
    run<4, 1, 1, 4, VP>("r32 D1 production", X, out, clk, 1024, reps);
    run<2, 1, 4, 8, VL>("r32x8w TN2 D4 mfma+loads", X, out, clk, 512, reps);
    run<2, 1, 4, 8, VP>("r32x8w TN2 D4 production", X, out, clk, 512, reps);
    // chain64 geometry: 256 eight-wave workgroups, TN 2 x 2 row tiles
    run<2, 2, 2, 8, VM>("r64 D2 mfma only", X, out, clk, 512, reps);
    run<2, 2, 2, 8, VL>("r64 D2 mfma+loads", X, out, clk, 512, reps);
    run<2, 2, 2, 8, VP>("r64 D2 production", X, out, clk, 512, reps);
    run<2, 2, 4, 8, VL>("r64 D4 mfma+loads", X, out, clk, 512, reps);
    run<2, 2, 4, 8, VP>("r64 D4 production", X, out, clk, 512, reps);
    return 0;
}
