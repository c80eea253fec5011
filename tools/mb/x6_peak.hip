// x6 inner-loop probe (development tool): what one k group of the chain kernels costs per SIMD.
// 256 workgroups x 8 waves (two per SIMD), each wave runs ITERS groups of
//   V0: 24 v_mfma_f32_32x32x16_bf16 on 4 accumulators (operands in registers)
//   V1: V0 + the three-way split of two 8-element activation fragments (split8 x 2: the chain64 group)
//   V2: V1 + 4 ds_read_b128 of the next fragments from LDS
//   V3: V2 + 12 global_load_dwordx4 weight refills from a 1 MiB L2-resident panel (ring depth 2)
// and prints us per launch and cycles per MFMA per SIMD at the measured clock (s_memtime on the device).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
#define DEVI __device__ __forceinline__

DEVI bf16x8_t as_bf16x8(const uint4& v) { return __builtin_bit_cast(bf16x8_t, v); }
DEVI void split3_act(float x, __bf16& hi, __bf16& mid, __bf16& lo) {
    const uint32_t u = __float_as_uint(x);
    const float h = __uint_as_float(u & 0xffff0000u);
    hi = __builtin_bit_cast(__bf16, (unsigned short)(u >> 16));
    const float r1 = __fsub_rn(x, h);
    mid = (__bf16)r1;
    lo = (__bf16)__fsub_rn(r1, (float)mid);
}
DEVI void split8(const float4& a0, const float4& a1, bf16x8_t& bh, bf16x8_t& bm, bf16x8_t& bl) {
    const float x[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        __bf16 h, m, l;
        split3_act(x[e], h, m, l);
        bh[e] = h; bm[e] = m; bl[e] = l;
    }
}

template <int V>
__global__ void __launch_bounds__(512) probe(const uint4* W, float* out, int iters, unsigned long long* cyc) {
    __shared__ float sA[2][4096];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int i = tid; i < 8192; i += 512) (&sA[0][0])[i] = 0.001f * (i % 97);
    __syncthreads();
    floatx16 acc[2][2];
    for (int j = 0; j < 2; ++j)
        for (int t = 0; t < 2; ++t)
            for (int e = 0; e < 16; ++e) acc[j][t][e] = 0.f;
    uint4 wr[2][2][3];
    const uint4* wp = W + (size_t)(blockIdx.x % 64) * 1024 + wave * 128 + lane;
    for (int d = 0; d < 2; ++d)
        for (int j = 0; j < 2; ++j)
            for (int p = 0; p < 3; ++p) wr[d][j][p] = wp[(d * 6 + j * 3 + p) * 64 % 1024];
    float4 n0 = make_float4(lane, 1.f, 2.f, 3.f), n1 = n0, m0 = n0, m1 = n0;
    const float* ap = &sA[0][0] + (lane & 31) * 4 + (lane >> 5) * 128;
    const unsigned long long t0 = 0;   // (no s_memtime: a pending SMEM event turns every lgkmcnt wait into 0)
    if (V == 4) {
        // software pipeline: group g's 24 MFMAs interleaved with group g+1's split, group g+2's LDS reads and
        // group g+2's weight refills (sched_group_barrier: 1 MFMA, then ~4 VALU / 1 DS / 1 VMEM per slot)
        bf16x8_t ch, cm, cl, dh, dm, dl;
        split8(n0, n1, ch, cm, cl);
        split8(m0, m1, dh, dm, dl);
        for (int it = 0; it < iters; it += 2) {
#pragma unroll
            for (int d = 0; d < 2; ++d) {
                const int o = ((it + d + 1) & 7) * 512;
                const float4 a0 = *(const float4*)(ap + o), a1 = *(const float4*)(ap + o + 256);
                const float4 b0 = *(const float4*)(ap + 4096 + o), b1 = *(const float4*)(ap + 4096 + o + 256);
                bf16x8_t ah, am, al, bh, bm, bl;
                split8(a0, a1, ah, am, al);
                split8(b0, b1, bh, bm, bl);
#pragma unroll
                for (int term = 0; term < 6; ++term) {
                    const int wi = term == 1 ? 2 : (term == 0 || term == 3) ? 1 : 0;
                    const bf16x8_t xa = (term == 1 || term == 3 || term == 5) ? ch : (term == 0 || term == 4) ? cm : cl;
                    const bf16x8_t xb = (term == 1 || term == 3 || term == 5) ? dh : (term == 0 || term == 4) ? dm : dl;
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        acc[j][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(wr[d][j][wi]), xa, acc[j][0], 0, 0, 0);
                        acc[j][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(wr[d][j][wi]), xb, acc[j][1], 0, 0, 0);
                    }
                }
#pragma unroll
                for (int j = 0; j < 2; ++j)
#pragma unroll
                    for (int p = 0; p < 3; ++p) wr[d][j][p] = wp[((it + d) * 6 + j * 3 + p) * 64 % 1024];
                // schedule: DS reads first spread, then MFMA / VALU / VMEM interleave
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // DS read
                }
#pragma unroll
                for (int k = 0; k < 20; ++k) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
                    __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);   // VALU
                    __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);   // VMEM read
                }
                __builtin_amdgcn_sched_barrier(0);
                ch = ah; cm = am; cl = al; dh = bh; dm = bm; dl = bl;
            }
        }
    } else
    for (int it = 0; it < iters; it += 2) {
#pragma unroll
        for (int d = 0; d < 2; ++d) {
            const float4 a0 = n0, a1 = n1, b0 = m0, b1 = m1;
            if (V >= 2 && V != 5 && V != 6) {
                const int o = ((it + d) & 7) * 512;
                n0 = *(const float4*)(ap + o); n1 = *(const float4*)(ap + o + 256);
                m0 = *(const float4*)(ap + 4096 + o); m1 = *(const float4*)(ap + 4096 + o + 256);
            } else {
                n0.x += 1.f; m0.y += 1.f;
            }
            __builtin_amdgcn_sched_barrier(0);
            bf16x8_t ah, am, al, bh, bm, bl;
            if (V >= 1) {
                split8(a0, a1, ah, am, al);
                split8(b0, b1, bh, bm, bl);
            } else {
                ah = am = al = as_bf16x8(make_uint4(__float_as_uint(a0.x), 1, 2, 3));
                bh = bm = bl = as_bf16x8(make_uint4(__float_as_uint(b0.y), 1, 2, 3));
            }
#pragma unroll
            for (int term = 0; term < 6; ++term) {
                const int wi = term == 1 ? 2 : (term == 0 || term == 3) ? 1 : 0;
                const bf16x8_t xa = (term == 1 || term == 3 || term == 5) ? ah : (term == 0 || term == 4) ? am : al;
                const bf16x8_t xb = (term == 1 || term == 3 || term == 5) ? bh : (term == 0 || term == 4) ? bm : bl;
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    acc[j][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(wr[d][j][wi]), xa, acc[j][0], 0, 0, 0);
                    acc[j][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(wr[d][j][wi]), xb, acc[j][1], 0, 0, 0);
                }
            }
            if (V >= 3 && V != 5 && V != 6) {
#pragma unroll
                for (int j = 0; j < 2; ++j)
#pragma unroll
                    for (int p = 0; p < 3; ++p) wr[d][j][p] = wp[((it + d) * 6 + j * 3 + p) * 64 % 1024];
            }
            if (V == 5 || V == 6) {
                // the next group's LDS reads spread between the MFMAs (one per six), V6 with the refills too
                const int o = ((it + d) & 7) * 512;
                n0 = *(const float4*)(ap + o); n1 = *(const float4*)(ap + o + 256);
                m0 = *(const float4*)(ap + 4096 + o); m1 = *(const float4*)(ap + 4096 + o + 256);
                if (V == 6) {
#pragma unroll
                    for (int j = 0; j < 2; ++j)
#pragma unroll
                        for (int p = 0; p < 3; ++p) wr[d][j][p] = wp[((it + d) * 6 + j * 3 + p) * 64 % 1024];
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 6, 0);   // 6 MFMA
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // 1 DS read
                    if (V == 6) __builtin_amdgcn_sched_group_barrier(0x020, 3, 0);   // 3 VMEM
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    const unsigned long long t1 = iters;
    float s = 0.f;
    for (int j = 0; j < 2; ++j)
        for (int t = 0; t < 2; ++t)
            for (int e = 0; e < 16; ++e) s += acc[j][t][e];
    if (s == 12345.f) out[tid] = s;
    if (tid == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

template <int V>
int run(const uint4* W, float* out, unsigned long long* cyc, int iters) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(probe<V>, dim3(256), dim3(512), 0, 0, W, out, iters, cyc);
    CK(hipEventRecord(e0));
    const int reps = 5;
    for (int w = 0; w < reps; ++w) hipLaunchKernelGGL(probe<V>, dim3(256), dim3(512), 0, 0, W, out, iters, cyc);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    unsigned long long c;
    CK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost));
    const double us = ms * 1e3 / reps;
    const double mfma_per_simd = 24.0 * iters * 2;   // 2 waves per SIMD
    // s_memtime counts at the constant 100 MHz reference on gfx950? report both views
    printf("V%d: %8.2f us/launch, %.1f ns per MFMA per SIMD (%.1f cycles at 2.1 GHz); wave0 memtime %llu\n", V, us,
           us * 1e3 / mfma_per_simd, us * 1e3 / mfma_per_simd * 2.1, c);
    return 0;
}

int main() {
    uint4* W; float* out; unsigned long long* cyc;
    CK(hipMalloc(&W, 64 * 1024 * 16)); CK(hipMemset(W, 0, 64 * 1024 * 16));
    CK(hipMalloc(&out, 4096 * 4)); CK(hipMalloc(&cyc, 8));
    const int iters = 2048;
    run<0>(W, out, cyc, iters); run<1>(W, out, cyc, iters); run<2>(W, out, cyc, iters); run<3>(W, out, cyc, iters);
    run<4>(W, out, cyc, iters); run<5>(W, out, cyc, iters); run<6>(W, out, cyc, iters);
    return 0;
}
