// LDS-DMA weight-ring probe (development tool, not shipped): what bounds the wide kernels' L2 -> LDS weight stream.
// One 512-thread workgroup per CU (256), 8 waves; per pipeline step every wave waits for its own DMAs up to the ring
// depth (counted vmcnt), joins a workgroup barrier, issues D 1-KiB global_load_lds_dwordx4 of the next step into the
// ring slot freed two steps ago, then (optionally) reads its step's fragments from LDS and runs MF MFMAs per fragment
// -- the wide_step_kernel skeleton without its arithmetic. The source stream is a head's x6q fragment stream: every
// workgroup of an XCD group (blockIdx % 8 in one half) walks the same SRC-byte panel in the same order.
//   ./dma_ring NS D STEPS MF SRC_KB NT   -> us per launch, us per step, GB/s per CU, TB/s chip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

template <int NT>
__device__ __forceinline__ void glds(const void* g, unsigned voff, unsigned lds) {
    unsigned keep;
    if constexpr (NT)
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %3 nt\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(voff), "s"(lds), "s"(g) : "memory");
    else
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %3\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(voff), "s"(lds), "s"(g) : "memory");
}

template <int NS, int D, int MF, int NT, int V>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2)))
ring_kernel(const char* src, long src_bytes, int steps, float* out) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    constexpr int SLOT = 8 * D * 1024;
    constexpr int VM = D * (NS - 3);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const unsigned base = (unsigned)(size_t)(__attribute__((address_space(3))) char*)lds;
    const unsigned voff = lane * 16;
    const char* s0 = src + ((blockIdx.x & 7) >> 2) * src_bytes;   // XCD groups 0-3 / 4-7: two panels
    auto addr = [&](int k, int d) -> const char* {
        const long off = ((long)k * 8 * D + wave * D + d) * 1024 % src_bytes;
        return s0 + off;
    };
    // V 6 / 7: only waves 4-7 / 0-3 issue (each the step's DMAs of itself and its SIMD partner wave ^ 4)
    auto issue = [&](int k) {
        if constexpr (V == 1 || V == 4 || V == 5 || V == 8 || V == 11 || V == 13) return;
        if constexpr (V == 6 || V == 7) {
            if ((V == 6) != (wave >= 4)) return;
#pragma unroll
            for (int d = 0; d < 2 * D; ++d) {
                const int w = d < D ? wave : wave ^ 4, dd = d % D;
                const long off = ((long)k * 8 * D + w * D + dd) * 1024 % src_bytes;
                glds<NT>(s0 + off, voff, base + (k % NS) * SLOT + (w * D + dd) * 1024);
            }
            return;
        }
#pragma unroll
        for (int d = 0; d < D; ++d) glds<NT>(addr(k, d), voff, base + (k % NS) * SLOT + (wave * D + d) * 1024);
    };
    // V 8: every wave issues its D DMAs spread over the step, one after fragment 2d + 1
    auto issue_one = [&](int k, int d) {
        glds<NT>(addr(k, d), voff, base + (k % NS) * SLOT + (wave * D + d) * 1024);
    };
    for (int k = 0; k < NS - 1; ++k) {
        if constexpr (V == 8 || V == 11 || V == 13) { for (int d = 0; d < D; ++d) issue_one(k, d); }
        else issue(k);
    }
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    floatx4 acc[8];
    for (int j = 0; j < 8; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < steps; ++k) {
        if constexpr (V != 4) asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" :: "n"(VM) : "memory");
        issue(k + NS - 1);
        if constexpr (MF > 0) {
            const char* sl = lds + (k % NS) * SLOT + lane * 16;
#pragma unroll
            for (int f = 0; f < 8 * D / 3; ++f) {
                uint4 w0, w1, w2;
                if constexpr (V == 2 || V == 5) {
                    w0 = make_uint4(f, lane, k, 1); w1 = make_uint4(f, 2, k, lane); w2 = make_uint4(3, f, lane, k);
                } else {
                    w0 = *(const uint4*)(sl + f * 3072); w1 = *(const uint4*)(sl + f * 3072 + 1024);
                    w2 = *(const uint4*)(sl + f * 3072 + 2048);
                }
                const bf16x8_t a0 = __builtin_bit_cast(bf16x8_t, w0), a1 = __builtin_bit_cast(bf16x8_t, w1),
                               a2 = __builtin_bit_cast(bf16x8_t, w2);
                if constexpr (V == 3) { acc[f & 7][0] += __builtin_bit_cast(float, w0.x ^ w1.y ^ w2.z); continue; }
                if constexpr (V == 8) { if ((f & 1) && f / 2 < D) issue_one(k + NS - 1, f / 2); }
                // V 11: DMA d of wave w after fragment (3w + d) % 8 -- three per fragment slot, SIMD partners (w, w + 4)
                // never in the same slot; V 13: waves 0-3 after fragments 0-2, waves 4-7 after fragments 4-6
                if constexpr (V == 11) {
#pragma unroll
                    for (int d = 0; d < D; ++d)
                        if (f == (3 * wave + d) % 8) issue_one(k + NS - 1, d);
                }
                if constexpr (V == 13) {
#pragma unroll
                    for (int d = 0; d < D; ++d)
                        if (f == d + (wave >= 4 ? 4 : 0)) issue_one(k + NS - 1, d);
                }
#pragma unroll
                for (int m = 0; m < MF; ++m) {
                    const bf16x8_t a = m % 3 == 0 ? a0 : m % 3 == 1 ? a1 : a2;
                    acc[(f + m) & 7] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, a1, acc[(f + m) & 7], 0, 0, 0);
                }
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    float s = 0.f;
    for (int j = 0; j < 8; ++j) s += acc[j][0] + acc[j][3];
    if (s == 12345.f) out[tid] = s;
}

// V 10: the weights streamed as fp32 (2 KiB per wave per step, 2/3 of the x6 bytes) into an fp32 ring, each step's
// landed slot split once per workgroup into the three bf16 planes of a double-buffered plane buffer (each thread 8
// weights: 2 ds_read_b128, the three-way split, 3 ds_write_b128), the MFMAs reading the planes split one step earlier.
__device__ __forceinline__ void split8(const float4& a, const float4& b, uint4& h, uint4& m, uint4& l) {
    const float x[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    unsigned short hh[8], mm[8], ll[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const __bf16 bh = (__bf16)x[i];
        const float r1 = x[i] - (float)bh;
        const __bf16 bm = (__bf16)r1;
        const __bf16 bl = (__bf16)(r1 - (float)bm);
        hh[i] = __builtin_bit_cast(unsigned short, bh);
        mm[i] = __builtin_bit_cast(unsigned short, bm);
        ll[i] = __builtin_bit_cast(unsigned short, bl);
    }
    h = make_uint4(hh[0] | (hh[1] << 16), hh[2] | (hh[3] << 16), hh[4] | (hh[5] << 16), hh[6] | (hh[7] << 16));
    m = make_uint4(mm[0] | (mm[1] << 16), mm[2] | (mm[3] << 16), mm[4] | (mm[5] << 16), mm[6] | (mm[7] << 16));
    l = make_uint4(ll[0] | (ll[1] << 16), ll[2] | (ll[3] << 16), ll[4] | (ll[5] << 16), ll[6] | (ll[7] << 16));
}

template <int NS, int MF>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2)))
ring10_kernel(const char* src, long src_bytes, int steps, float* out) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    constexpr int SLOT = 16 * 1024, PLANES = 24 * 1024;
    constexpr int VM = 2 * (NS - 3);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const unsigned base = (unsigned)(size_t)(__attribute__((address_space(3))) char*)lds;
    const unsigned voff = lane * 16;
    char* pb = lds + NS * SLOT;
    const char* s0 = src + ((blockIdx.x & 7) >> 2) * src_bytes;
    auto issue = [&](int k) {
#pragma unroll
        for (int d = 0; d < 2; ++d) {
            const long off = ((long)k * 16 + wave * 2 + d) * 1024 % src_bytes;
            glds<0>(s0 + off, voff, base + (k % NS) * SLOT + (wave * 2 + d) * 1024);
        }
    };
    auto split = [&](int k) {   // slot of step k -> plane buffer k & 1
        const char* sl = lds + (k % NS) * SLOT + tid * 32;
        const float4 a = *(const float4*)sl, b = *(const float4*)(sl + 16);
        uint4 h, m, l;
        split8(a, b, h, m, l);
        char* d = pb + (k & 1) * PLANES;
        *(uint4*)(d + tid * 16) = h;
        *(uint4*)(d + 8192 + tid * 16) = m;
        *(uint4*)(d + 16384 + tid * 16) = l;
    };
    for (int k = 0; k < NS - 1; ++k) issue(k);
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    split(0);
    floatx4 acc[8];
    for (int j = 0; j < 8; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < steps; ++k) {
        asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" :: "n"(VM) : "memory");
        issue(k + NS - 1);
        split(k + 1);
        const char* sl = pb + (k & 1) * PLANES + lane * 16;
#pragma unroll
        for (int f = 0; f < 8; ++f) {
            // fragment f's three planes (the probe's layout: 1 KiB per plane and fragment)
            const uint4 w0 = *(const uint4*)(sl + f * 1024), w1 = *(const uint4*)(sl + 8192 + f * 1024),
                        w2 = *(const uint4*)(sl + 16384 + f * 1024);
            const bf16x8_t a0 = __builtin_bit_cast(bf16x8_t, w0), a1 = __builtin_bit_cast(bf16x8_t, w1),
                           a2 = __builtin_bit_cast(bf16x8_t, w2);
#pragma unroll
            for (int mm = 0; mm < MF; ++mm) {
                const bf16x8_t a = mm % 3 == 0 ? a0 : mm % 3 == 1 ? a1 : a2;
                acc[(f + mm) & 7] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, a1, acc[(f + mm) & 7], 0, 0, 0);
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    float s = 0.f;
    for (int j = 0; j < 8; ++j) s += acc[j][0] + acc[j][3];
    if (s == 12345.f) out[tid] = s;
}

// Interference probe: no barriers. Waves 0-3 (one per SIMD) run 96 MFMAs per step on register operands (a SIMD's
// whole step of matrix work); waves 4-7 (their SIMD partners) either leave at once (L = 0) or stream 6 KiB per step
// into their own LDS area with global_load_lds_dwordx4 (L = 1; vmcnt keeps one step in flight) -- does an LDS-DMA
// stream on a SIMD slow its partner's MFMAs?  out[wave] = the wave's s_memtime cycles.
template <int L>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2)))
split_kernel(const char* src, long src_bytes, int steps, unsigned long long* out) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (wave < 4) {
        floatx4 acc[8];
        for (int j = 0; j < 8; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
        const bf16x8_t a0 = __builtin_bit_cast(bf16x8_t, make_uint4(lane, 1, 2, 3));
        const bf16x8_t a1 = __builtin_bit_cast(bf16x8_t, make_uint4(3, lane, 1, 2));
        for (int k = 0; k < steps; ++k) {
#pragma unroll
            for (int m = 0; m < 96; ++m)
                acc[m & 7] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(m & 1 ? a0 : a1, a1, acc[m & 7], 0, 0, 0);
        }
        float s = 0.f;
        for (int j = 0; j < 8; ++j) s += acc[j][0] + acc[j][3];
        if (s == 12345.f) out[4096 + tid] = (unsigned long long)s;
    } else if (L == 1) {
        const unsigned base = (unsigned)(size_t)(__attribute__((address_space(3))) char*)lds + (wave - 4) * 12 * 1024;
        const unsigned voff = lane * 16;
        const char* s0 = src + ((blockIdx.x & 7) >> 2) * src_bytes;
        for (int k = 0; k < steps; ++k) {
#pragma unroll
            for (int d = 0; d < 6; ++d) {
                const long off = ((long)k * 24 + (wave - 4) * 6 + d) * 1024 % src_bytes;
                glds<0>(s0 + off, voff, base + ((k & 1) * 6 + d) * 1024);
            }
            asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[blockIdx.x * 8 + wave] = t1 - t0;
}

template <int L>
void run_split(int steps, long src_kb) {
    const long sb = src_kb * 1024;
    char* src;
    CK(hipMalloc(&src, 2 * sb));
    CK(hipMemset(src, 0, 2 * sb));
    unsigned long long* out;
    CK(hipMalloc(&out, 8192 * 8));
    CK(hipFuncSetAttribute((const void*)split_kernel<L>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((split_kernel<L>), dim3(256), dim3(512), 48 * 1024, 0, src, sb, steps, out);
    CK(hipDeviceSynchronize());
    const int R = 20;
    CK(hipEventRecord(e0));
    for (int i = 0; i < R; ++i) hipLaunchKernelGGL((split_kernel<L>), dim3(256), dim3(512), 48 * 1024, 0, src, sb, steps, out);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<unsigned long long> h(2048);
    CK(hipMemcpy(h.data(), out, 2048 * 8, hipMemcpyDeviceToHost));
    double cmp = 0, ld = 0;
    for (int b = 0; b < 256; ++b)
        for (int w = 0; w < 8; ++w) (w < 4 ? cmp : ld) += (double)h[b * 8 + w];
    printf("split L=%d steps=%d: %.2f us/launch; MFMA waves %.0f memtime ticks/step, loader waves %.0f ticks/step\n", L, steps,
           ms * 1e3 / R, cmp / 1024 / steps, ld / 1024 / steps);
    CK(hipFree(src));
    CK(hipFree(out));
}

template <int NS, int MF>
void run10(int steps, long src_kb) {
    const long sb = src_kb * 1024;
    char* src;
    CK(hipMalloc(&src, 2 * sb));
    CK(hipMemset(src, 0, 2 * sb));
    float* out;
    CK(hipMalloc(&out, 4096));
    const size_t lds = (size_t)NS * 16 * 1024 + 2 * 24 * 1024;
    CK(hipFuncSetAttribute((const void*)ring10_kernel<NS, MF>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((ring10_kernel<NS, MF>), dim3(256), dim3(512), lds, 0, src, sb, steps, out);
    CK(hipDeviceSynchronize());
    const int R = 50;
    CK(hipEventRecord(e0));
    for (int i = 0; i < R; ++i) hipLaunchKernelGGL((ring10_kernel<NS, MF>), dim3(256), dim3(512), lds, 0, src, sb, steps, out);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / R;
    printf("V=10 (fp32 stream + split) NS=%d MF=%d steps=%d src=%ldKB: %.2f us/launch, %.3f us/step\n", NS, MF, steps,
           src_kb, us, us / steps);
    CK(hipFree(src));
    CK(hipFree(out));
}

template <int NS, int D, int MF, int NT, int V = 0>
void run(int steps, long src_kb, bool rnd = false) {
    const long sb = src_kb * 1024;
    char* src;
    CK(hipMalloc(&src, 2 * sb));
    CK(hipMemset(src, 0, 2 * sb));
    if (rnd) {   // random bf16 bit patterns (finite: exponent kept moderate) -- the clock a real stream holds
        std::vector<unsigned short> h(sb);
        unsigned x = 12345;
        for (auto& v : h) { x = x * 1664525u + 1013904223u; v = (unsigned short)(0x3c00 | ((x >> 8) & 0x83ff)); }
        CK(hipMemcpy(src, h.data(), sb * 2 > 2 * sb ? 2 * sb : sb * 2, hipMemcpyHostToDevice));
    }
    float* out;
    CK(hipMalloc(&out, 4096));
    const size_t lds = (size_t)NS * 8 * D * 1024;
    CK(hipFuncSetAttribute((const void*)ring_kernel<NS, D, MF, NT, V>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((ring_kernel<NS, D, MF, NT, V>), dim3(256), dim3(512), lds, 0, src, sb, steps, out);
    CK(hipDeviceSynchronize());
    const int R = 50;
    CK(hipEventRecord(e0));
    for (int i = 0; i < R; ++i) hipLaunchKernelGGL((ring_kernel<NS, D, MF, NT, V>), dim3(256), dim3(512), lds, 0, src, sb, steps, out);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / R;
    const double bytes = 256.0 * steps * 8 * D * 1024;
    printf("V=%d rnd=%d NS=%d D=%d MF=%d NT=%d steps=%d src=%ldKB: %.2f us/launch, %.3f us/step, %.1f GB/s per CU, %.2f TB/s chip\n",
           V, (int)rnd, NS, D, MF, NT, steps, src_kb, us, us / steps, bytes / 256 / (us * 1e-6) / 1e9, bytes / (us * 1e-6) / 1e12);
    CK(hipFree(src));
    CK(hipFree(out));
}

int main(int argc, char** argv) {
    const int steps = argc > 1 ? atoi(argv[1]) : 94;
    const long kb = argc > 2 ? atol(argv[2]) : 2304;
    if (argc > 3) {   // one case only (PMC passes per case): full | mfma | mfma_dma | mfma_lds | dma
        const char* c = argv[3];
        if (!strcmp(c, "full")) run<4, 3, 6, 0, 0>(steps, kb);
        else if (!strcmp(c, "mfma")) run<4, 3, 6, 0, 5>(steps, kb);
        else if (!strcmp(c, "mfma_dma")) run<4, 3, 6, 0, 2>(steps, kb);
        else if (!strcmp(c, "mfma_lds")) run<4, 3, 6, 0, 1>(steps, kb);
        else if (!strcmp(c, "dma")) run<4, 3, 0, 0, 0>(steps, kb);
        else if (!strcmp(c, "stagger")) {
            for (int i = 0; i < 2; ++i) {
                run<4, 3, 6, 0, 0>(steps, kb); run<4, 3, 6, 0, 8>(steps, kb); run<4, 3, 6, 0, 11>(steps, kb);
                run<4, 3, 6, 0, 13>(steps, kb); run<4, 3, 6, 0, 5>(steps, kb);
                run<5, 3, 6, 0, 11>(steps, kb);
            }
        }
        else if (!strcmp(c, "split")) { run_split<0>(steps, kb); run_split<1>(steps, kb); run_split<0>(steps, kb); run_split<1>(steps, kb); }
        else { printf("unknown case %s\n", c); return 2; }
        return 0;
    }
    run<4, 3, 6, 0, 0>(steps, kb);          // full: every wave issues 3 DMAs right after the barrier
    run<4, 3, 6, 0, 5>(steps, kb);          // MFMA + barrier only (the floor)
    run10<4, 6>(steps, kb);                 // fp32 stream + one split per workgroup
    run10<5, 6>(steps, kb);
    run10<4, 0>(steps, kb);                 // (its stream + split alone)
    run<4, 3, 0, 0, 0>(steps, kb);          // (the x6 stream alone)
    return 0;
}
