// learner_conv.hip -- the pixel encoder's convolutions for the learner engine on MI355X (gfx950).
//
// Reference: helper.enc for pixels (/root/reference/src/algorithm/helper.py:119-133): NormalizeImg (x / 255), four
// Conv2d(-> 32 channels, kernel 7 / 5 / 3 / 3, stride 2, no padding) + ReLU, Flatten, Linear; trained by
// TDMPC.update (tdmpc.py:192-245) through the online encoder on the augmented observations, and run forward only
// on the augmented next observations by the online (TD target, tdmpc.py:184-190) and the target encoder
// (consistency target, tdmpc.py:206-207). The Linear and its backward are tdmpc_lg_gemm jobs; this file holds the
// three convolution passes (include/tdmpc_learner.h), each an implicit GEMM on the exact f32 MFMA
// (v_mfma_f32_32x32x2_f32, the learner's default product), with every sum in a fixed order (no atomics): a graph
// replay equals the eager pass bit for bit.
//   * conv_fwd: output pixels x 32 channels; a workgroup = 4 waves x 32 pixels of one image; the weights [K][32] and
//     the im2col offset of every k in LDS, the input gathered from L2 (buffer loads, 8 MFMA steps in flight).
//   * conv_bwd_data: the transposed conv, split by the input pixel's parity class (py, px) so that each class is a
//     dense GEMM over only the (co, ky, kx) taps that reach it (ky = py (mod 2), kx = px (mod 2)); the ReLU mask of
//     the layer below fused into the store.
//   * conv_bwd_weight: 32 channels x (cin k k + 1) columns (the last one the bias), reduced over a slice of images
//     and their output pixels; one partial slice per workgroup row, summed in order by tdmpc_lg_finalize.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>

#include "../../include/tdmpc_hip.h"
#include "../../include/tdmpc_learner.h"

namespace tdmpc_internal {
void set_error(const char* msg);
}

namespace {

#define DEVI __device__ __forceinline__
typedef float floatx16 __attribute__((ext_vector_type(16)));
constexpr unsigned CV_OOB = 0x7ffffff0u;   // buffer offsets >= this read 0
constexpr int CV_D = 16;                    // MFMA steps of operand loads in flight

int cv_bad(const char* m) {
    tdmpc_internal::set_error(m);
    return TDMPC_E_DIMS;
}

// q = e / d for 0 <= e < 2^16 and 0 < d <= 2^16 by a float multiply (exact: (e + 0.5) / d sits >= 0.5 / d away from an
// integer, far beyond the product's rounding) -- the staging loops' index splits without an integer division
DEVI int cv_div(int e, float inv_d) { return (int)__fmul_rn((float)e + 0.5f, inv_d); }
DEVI float relu_f(float v) { return v != v ? v : fmaxf(v, 0.f); }   // (torch.relu keeps a NaN)
DEVI __amdgpu_buffer_rsrc_t cv_rsrc(const float* p) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)CV_OOB, 0x00020000);
}
DEVI float cv_ld(__amdgpu_buffer_rsrc_t r, unsigned off_elems, bool ok) {
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, ok ? (int)(off_elems * 4u) : (int)CV_OOB, 0, 0));
}

// ---------------------------------------------------------------------------------------------------- forward
// grid (ceil(ho^2 / 128), n, nprob), 256 threads; LDS sW [K2][32] | koff [K2] (K2 = K rounded up to even)
__global__ void __launch_bounds__(256) conv_fwd_kernel(const tdmpc_lg_conv a, int ho, int K2) {
    extern __shared__ float cv_sm[];
    const int img = blockIdx.y, pr = blockIdx.z;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 31, h = lane >> 5;
    const int kk = a.k * a.k, K = a.cin * kk, H = a.hin, HoHo = ho * ho;
    const float* w = pr ? a.w[1] : a.w[0];
    float* sW = cv_sm;
    int* koff = (int*)(cv_sm + (size_t)K2 * 32);
    for (int i = tid; i < K2 * 32; i += 256) {
        const int k = i >> 5, co = i & 31;
        sW[i] = k < K ? w[(size_t)co * K + k] : 0.f;
    }
    for (int k = tid; k < K2; k += 256) {
        const int ci = k / kk, rem = k % kk;
        koff[k] = k < K ? ci * H * H + (rem / a.k) * H + rem % a.k : 0;
    }
    __syncthreads();
    const int p0 = blockIdx.x * 128 + wave * 32;
    if (p0 >= HoHo) return;   // (wave-uniform; no barrier below)
    const int p = p0 + r;
    const int pp = p < HoHo ? p : HoHo - 1;
    const int pixbase = 2 * (pp / ho) * H + 2 * (pp % ho);
    const __amdgpu_buffer_rsrc_t rx = cv_rsrc(a.x + (size_t)img * a.cin * H * H);
    const float div = a.in_div;
    const int ns = K2 / 2;
    floatx16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
    float av[CV_D];
#pragma unroll
    for (int d = 0; d < CV_D - 1; ++d) av[d] = cv_ld(rx, (unsigned)(pixbase + koff[min(2 * d + h, K2 - 1)]), d < ns);
    for (int s0 = 0; s0 < ns; s0 += CV_D) {
#pragma unroll
        for (int d = 0; d < CV_D; ++d) {
            const int s = s0 + d, sl = s + CV_D - 1;
            av[(d + CV_D - 1) % CV_D] = cv_ld(rx, (unsigned)(pixbase + koff[min(2 * sl + h, K2 - 1)]), sl < ns);
            if (s < ns) {
                float x = av[d];
                if (div > 0.f) x = __fdiv_rn(x, div);
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(x, sW[(2 * s + h) * 32 + r], acc, 0, 0, 0);
            }
        }
    }
    // C/D map of the 32x32 MFMA: col = lane & 31 (the channel), row = (e & 3) + 8 (e >> 2) + 4 (lane >> 5) (the pixel)
    const float bias = (pr ? a.b[1] : a.b[0])[r];
    float* y = (pr ? a.y[1] : a.y[0]) + ((size_t)img * 32 + r) * HoHo;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        const int pix = p0 + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (pix < HoHo) y[pix] = relu_f(acc[e] + bias);
    }
}

// The same forward for the large layers (ho^2 >= 256: the first two), input staged in LDS: a workgroup = 8 waves x
// 32 output pixels = the 256-pixel block [P0, P0 + 256) of one image, for both weight sets of the launch (NP). The
// block's output rows need input rows [2 oy0, 2 oy1 + k): a contiguous run of SR rows per channel, copied in chunks of
// CC channels (<= 32 KB of slab, <= 208 k-values of weights) with coalesced loads; the next chunk's loads are in
// flight in registers while this chunk's MFMAs run on LDS operands (one ds_read of the slab per MFMA step and set,
// no global-latency chain). The division by in_div (NormalizeImg) happens once per staged element, the same rounding.
// Sums: chunk by chunk in k order, every chunk but the last an even number of k-values -- the direct kernel's MFMA
// pairs and order, so both give the same bits (tests/test_learner.py). TDMPC_CONV_DIRECT=1: the direct kernel (A/B).
constexpr int CVS_SLAB = 8192, CVS_KC = 208;   // slab floats, k-values per chunk

template <int NP, int TP>
__global__ void __launch_bounds__(512) conv_fwd_slab_kernel(const tdmpc_lg_conv a, int ho, int CC, int SRM) {
    extern __shared__ float cv_sm[];
    const int img = blockIdx.y;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 31, h = lane >> 5;
    const int k = a.k, kk = k * k, H = a.hin, HoHo = ho * ho, cin = a.cin;
    constexpr int BP = 256 * TP;   // block pixels: 8 waves x TP tiles of 32
    const int P0 = blockIdx.x * BP;
    const int oy0 = P0 / ho, oy1 = min(ho - 1, (P0 + BP - 1) / ho);
    const int SR = 2 * (oy1 - oy0) + k, plane = SR * H;
    const float inv_plane = 1.0f / (float)plane;
    const int KCM = (CC * kk + 1) & ~1, KT = ((KCM / 2) + 3) & ~3;
    float* slab = cv_sm;                                   // [CC + 1][SR][H] (plane cc: zeros for an odd chunk's pad)
    float* sW = slab + (((CC + 1) * SRM * H + 3) & ~3);    // [NP][KCM][32] (16-byte aligned: kt's int4 reads)
    int* kt = (int*)(sW + (size_t)NP * KCM * 32);          // [2][KT]: slab offset of k-value 2 s + h, step s
    const __amdgpu_buffer_rsrc_t rx = cv_rsrc(a.x + ((size_t)img * cin * H + 2 * oy0) * H);
    __amdgpu_buffer_rsrc_t rw[NP];
#pragma unroll
    for (int q = 0; q < NP; ++q) rw[q] = cv_rsrc(a.w[q]);
    const float div = a.in_div;
    const int nchunk = (cin + CC - 1) / CC;
    const int pw0 = P0 + wave * 32 * TP;       // this wave's TP tiles: pixels [pw0, pw0 + 32 TP)
    const bool live = pw0 < HoHo;              // (wave-uniform)
    int pixbase[TP];
#pragma unroll
    for (int t = 0; t < TP; ++t) {
        const int pp = min(pw0 + 32 * t + r, HoHo - 1);
        pixbase[t] = 2 * (pp / ho - oy0) * H + 2 * (pp % ho);
    }
    constexpr int NS = CVS_SLAB / 512, NW = (CVS_KC * 32 + 511) / 512;
    float sv[NS], wv[NP][NW];
    auto fetch = [&](int c) __attribute__((always_inline)) {
        const int c0 = c * CC, cc = min(CC, cin - c0), ns = cc * plane, nk = cc * kk;
#pragma unroll
        for (int i = 0; i < NS; ++i) {
            const int e = tid + 512 * i, ci = cv_div(e, inv_plane);
            sv[i] = cv_ld(rx, (unsigned)((c0 + ci) * H * H + e - ci * plane), e < ns);
        }
#pragma unroll
        for (int q = 0; q < NP; ++q)
#pragma unroll
            for (int i = 0; i < NW; ++i) {
                const int e = tid + 512 * i, kl = e >> 5, co = e & 31;
                wv[q][i] = cv_ld(rw[q], (unsigned)(co * cin * kk + c0 * kk + kl), kl < nk);
            }
    };
    auto stash = [&](int c) __attribute__((always_inline)) {
        const int c0 = c * CC, cc = min(CC, cin - c0), ns = cc * plane, nk = cc * kk;
        if (div > 0.f) {   // (a uniform branch: the division is not computed when there is none)
#pragma unroll
            for (int i = 0; i < NS; ++i) {
                const int e = tid + 512 * i;
                if (e < ns) slab[e] = __fdiv_rn(sv[i], div);
            }
        } else {
#pragma unroll
            for (int i = 0; i < NS; ++i) {
                const int e = tid + 512 * i;
                if (e < ns) slab[e] = sv[i];
            }
        }
        if (nk & 1)   // the pad k-value nk reads plane cc at the pixel's base: zeros (times a zero weight)
            for (int e = tid; e < plane; e += 512) slab[ns + e] = 0.f;
        for (int e = tid; e < 2 * KT; e += 512) {
            const int hh = e / KT, st = e - hh * KT, j = 2 * st + hh;
            const int ci = j / kk, t = j - ci * kk;
            kt[e] = j < nk ? ci * plane + (t / k) * H + t % k : cc * plane;
        }
#pragma unroll
        for (int q = 0; q < NP; ++q)
#pragma unroll
            for (int i = 0; i < NW; ++i) {
                const int e = tid + 512 * i;
                if ((e >> 5) < KCM) sW[(q * KCM) * 32 + e] = wv[q][i];
            }
    };
    floatx16 acc[NP][TP];
#pragma unroll
    for (int q = 0; q < NP; ++q)
#pragma unroll
        for (int t = 0; t < TP; ++t)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[q][t][e] = 0.f;
    fetch(0);
    stash(0);
    __syncthreads();
    for (int c = 0; c < nchunk; ++c) {
        if (c + 1 < nchunk) fetch(c + 1);
        if (live) {
            // k-value j = 2 s + h of the chunk is tap (ci, ky, kx) at slab offset kt[h][s] = ci plane + ky H + kx from
            // the pixel's base: four steps' offsets per 16-byte LDS read, a step's reads then independent of each other
            const int nk = min(CC, cin - c * CC) * kk, nst = (nk + 1) / 2;
            const int* kth = kt + h * KT;
            for (int s0 = 0; s0 < nst; s0 += 4) {
                const int4 o4 = *(const int4*)(kth + s0);
                const int ov[4] = {o4.x, o4.y, o4.z, o4.w};
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int s = s0 + u;
                    if (s < nst) {
                        float av[TP];
#pragma unroll
                        for (int t = 0; t < TP; ++t) av[t] = slab[pixbase[t] + ov[u]];
#pragma unroll
                        for (int q = 0; q < NP; ++q) {
                            const float bw = sW[(q * KCM + 2 * s + h) * 32 + r];
#pragma unroll
                            for (int t = 0; t < TP; ++t)
                                acc[q][t] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[t], bw, acc[q][t], 0, 0, 0);
                        }
                    }
                }
            }
        }
        if (c + 1 < nchunk) {
            __syncthreads();
            stash(c + 1);
            __syncthreads();
        }
    }
    if (!live) return;
#pragma unroll
    for (int q = 0; q < NP; ++q) {
        const float bias = a.b[q][r];
        float* y = a.y[q] + ((size_t)img * 32 + r) * HoHo;
#pragma unroll
        for (int t = 0; t < TP; ++t)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int pix = pw0 + 32 * t + (e & 3) + 8 * (e >> 2) + 4 * h;
                if (pix < HoHo) y[pix] = relu_f(acc[q][t][e] + bias);
            }
    }
}

// ------------------------------------------------------------------------------------------------ data gradient
// grid (ceil(max class pixels / 128), 4 parity classes, n), 256 threads; LDS sW [Kc][32] | tab [Kc] (int2)
__global__ void __launch_bounds__(256) conv_bwd_data_kernel(const float* dy, const float* w, const float* xact,
                                                            float* dx, int cin, int H, int k, int ho) {
    extern __shared__ float cv_sm[];
    const int py = blockIdx.y >> 1, px = blockIdx.y & 1, img = blockIdx.z;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 31, h = lane >> 5;
    const int Wc = (H - px + 1) / 2, Pc = ((H - py + 1) / 2) * Wc;
    const int nky = (k - py + 1) / 2, nkx = (k - px + 1) / 2, Kc = 32 * nky * nkx;   // (even)
    const int HoHo = ho * ho, kk = k * k;
    float* sW = cv_sm;
    int2* tab = (int2*)(cv_sm + (size_t)Kc * 32);
    // tap j = (co nky + iy) nkx + ix: ky = py + 2 iy, kx = px + 2 ix; dy[co][cy - iy][cx - ix] for class pixel (cy, cx)
    for (int i = tid; i < Kc * 32; i += 256) {
        const int j = i >> 5, ci = i & 31;
        const int ix = j % nkx, iy = (j / nkx) % nky, co = j / (nkx * nky);
        sW[i] = w[((size_t)co * cin + ci) * kk + (py + 2 * iy) * k + px + 2 * ix];
    }
    for (int j = tid; j < Kc; j += 256) {
        const int ix = j % nkx, iy = (j / nkx) % nky, co = j / (nkx * nky);
        tab[j] = make_int2(co * HoHo - iy * ho - ix, iy | (ix << 8));
    }
    __syncthreads();
    const int q0 = blockIdx.x * 128 + wave * 32;
    if (q0 >= Pc) return;
    const int q = min(q0 + r, Pc - 1);
    const int cy = q / Wc, cx = q % Wc;
    const __amdgpu_buffer_rsrc_t rd = cv_rsrc(dy + (size_t)img * 32 * HoHo);
    const int ns = Kc / 2;
    auto ld = [&](int s) -> float {
        const int j = min(2 * s + h, Kc - 1);
        const int2 t = tab[j];
        const int oy = cy - (t.y & 255), ox = cx - (t.y >> 8);
        const bool ok = s < ns && (unsigned)oy < (unsigned)ho && (unsigned)ox < (unsigned)ho;
        return cv_ld(rd, (unsigned)(t.x + cy * ho + cx), ok);
    };
    floatx16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
    float av[CV_D];
#pragma unroll
    for (int d = 0; d < CV_D - 1; ++d) av[d] = ld(d);
    for (int s0 = 0; s0 < ns; s0 += CV_D) {
#pragma unroll
        for (int d = 0; d < CV_D; ++d) {
            const int s = s0 + d;
            av[(d + CV_D - 1) % CV_D] = ld(s + CV_D - 1);
            if (s < ns) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[d], sW[(2 * s + h) * 32 + r], acc, 0, 0, 0);
        }
    }
    // col = lane & 31: input channel ci; rows: class pixels
    const size_t plane = ((size_t)img * cin + r) * H * H;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        const int qq = q0 + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (qq >= Pc) continue;
        const int o = (2 * (qq / Wc) + py) * H + 2 * (qq % Wc) + px;
        dx[plane + o] = xact[plane + o] > 0.f ? acc[e] : 0.f;   // (threshold_backward of the ReLU below)
    }
}

// ---------------------------------------------------------------------------------------------- weight gradient
// grid (ceil(column tiles / 4), slices), 256 threads: wave = one 32-column tile of [32][K + 1]
__global__ void __launch_bounds__(256) conv_bwd_weight_kernel(const float* dy, const float* x, float div, float* part,
                                                              int n, int cin, int H, int k, int ho, int ips) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 31, h = lane >> 5;
    const int kk = k * k, K = cin * kk, K1 = K + 1, ntile = (K1 + 31) / 32;
    const int t = blockIdx.x * 4 + wave;
    if (t >= ntile) return;
    const int slice = blockIdx.y, n0 = slice * ips, n1 = min(n, n0 + ips), HoHo = ho * ho;
    // this lane's B column (t 32 + r): an im2col tap, the bias column (ones) or padding (zeros)
    const int col = t * 32 + r;
    const int ci = col / kk, rem = col % kk;
    const int koff = col < K ? ci * H * H + (rem / k) * H + rem % k : 0;
    const bool tap = col < K, one = col == K;
    const int ns = (HoHo + 1) / 2;
    floatx16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
    for (int img = n0; img < n1; ++img) {
        const __amdgpu_buffer_rsrc_t rd = cv_rsrc(dy + ((size_t)img * 32 + r) * HoHo);
        const __amdgpu_buffer_rsrc_t rx = cv_rsrc(x + (size_t)img * cin * H * H);
        // pixel 2s + h of the image; its (oy, ox) advanced incrementally (two pixels per step, 2 < ho)
        int loy = 0, lox = h;   // the loads' position (CV_D - 1 steps ahead of the products)
        float av[CV_D], bv[CV_D];
        auto ld = [&](int s, float& A, float& Bv) {
            const int pix = 2 * s + h;
            const bool ok = s < ns && pix < HoHo;
            A = cv_ld(rd, (unsigned)pix, ok);
            const float xv = cv_ld(rx, (unsigned)(2 * loy * H + 2 * lox + koff), ok && tap);
            Bv = one ? (ok ? 1.f : 0.f) : xv;
            lox += 2;
            if (lox >= ho) { lox -= ho; ++loy; }
        };
#pragma unroll
        for (int d = 0; d < CV_D - 1; ++d) ld(d, av[d], bv[d]);
        for (int s0 = 0; s0 < ns; s0 += CV_D) {
#pragma unroll
            for (int d = 0; d < CV_D; ++d) {
                const int s = s0 + d;
                ld(s + CV_D - 1, av[(d + CV_D - 1) % CV_D], bv[(d + CV_D - 1) % CV_D]);
                if (s < ns) {
                    float b = bv[d];
                    if (div > 0.f && tap) b = __fdiv_rn(b, div);
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[d], b, acc, 0, 0, 0);
                }
            }
        }
    }
    // col = lane & 31 (the B column), row = (e & 3) + 8 (e >> 2) + 4 h (the output channel)
    if (col >= K1) return;
    float* o = part + (size_t)slice * 32 * K1 + col;
#pragma unroll
    for (int e = 0; e < 16; ++e) o[(size_t)((e & 3) + 8 * (e >> 2) + 4 * h) * K1] = acc[e];
}

// The weight gradient with its operands staged in LDS: a workgroup = 8 waves over the images of one slice, the
// image's output pixels in blocks of PB (dy [32][PB] and the block's input slab [cin][SR][H] copied with coalesced
// loads), wave w owning the 32-column tiles w + 8 u (u < TPW: one dy read feeds TPW MFMAs). Pixel pairs and their
// order are the direct kernel's (PB even), so both give the same bits; TDMPC_CONV_DIRECT=1 runs the direct one.
template <int TPW>
__global__ void __launch_bounds__(512) conv_bwd_weight_slab_kernel(const float* dy, const float* x, float div,
                                                                   float* part, int n, int cin, int H, int k, int ho,
                                                                   int ips, int PB, int SRM) {
    extern __shared__ float cv_sm[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 31, h = lane >> 5;
    const int kk = k * k, K = cin * kk, K1 = K + 1, HoHo = ho * ho;
    const int slice = blockIdx.x, n0 = slice * ips, n1 = min(n, n0 + ips);
    const int PBP = PB + 1;
    float* dyl = cv_sm;                              // [32][PB + 1]
    float* slab = cv_sm + 32 * PBP;                  // [cin][SR][H]
    int tapoff[TPW];
    bool tap[TPW], one[TPW];
#pragma unroll
    for (int u = 0; u < TPW; ++u) {
        const int col = (wave + 8 * u) * 32 + r;
        const int ci = col / kk, rem = col % kk;
        tap[u] = col < K;
        one[u] = col == K;
        tapoff[u] = tap[u] ? ci * SRM * H + (rem / k) * H + rem % k : 0;   // (plane stride SRM H: see the staging)
    }
    floatx16 acc[TPW];
#pragma unroll
    for (int u = 0; u < TPW; ++u)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[u][e] = 0.f;
    for (int img = n0; img < n1; ++img) {
        const float* dyi = dy + (size_t)img * 32 * HoHo;
        const float* xi = x + (size_t)img * cin * H * H;
        for (int P0 = 0; P0 < HoHo; P0 += PB) {
            const int npx = min(PB, HoHo - P0);
            const int oy0 = P0 / ho, oy1 = (P0 + npx - 1) / ho;
            const int SR = 2 * (oy1 - oy0) + k, plane = SR * H;
            const float inv_npx = 1.0f / (float)npx, inv_plane = 1.0f / (float)plane;
            __syncthreads();   // (the previous block's reads are done)
            for (int e = tid; e < 32 * npx; e += 512) {
                const int co = cv_div(e, inv_npx), p = e - co * npx;
                dyl[co * PBP + p] = dyi[(size_t)co * HoHo + P0 + p];
            }
            if (div > 0.f)
                for (int e = tid; e < cin * plane; e += 512) {
                    const int ci = cv_div(e, inv_plane), o = e - ci * plane;
                    slab[ci * SRM * H + o] = __fdiv_rn(xi[(size_t)ci * H * H + (size_t)(2 * oy0) * H + o], div);
                }
            else
                for (int e = tid; e < cin * plane; e += 512) {
                    const int ci = cv_div(e, inv_plane), o = e - ci * plane;
                    slab[ci * SRM * H + o] = xi[(size_t)ci * H * H + (size_t)(2 * oy0) * H + o];
                }
            __syncthreads();
            const int nst = (npx + 1) / 2;
            int P = P0 + h, ox = P % ho;
            int po = 2 * (P / ho - oy0) * H + 2 * ox;
#pragma unroll 2
            for (int s = 0; s < nst; ++s) {
                const bool pv = 2 * s + h < npx;
                const float av = pv ? dyl[r * PBP + 2 * s + h] : 0.f;
#pragma unroll
                for (int u = 0; u < TPW; ++u) {
                    const float xv = slab[(pv && tap[u]) ? tapoff[u] + po : 0];
                    const float bv = tap[u] ? (pv ? xv : 0.f) : (one[u] && pv ? 1.f : 0.f);
                    acc[u] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc[u], 0, 0, 0);
                }
                ox += 2;
                const bool w = ox >= ho;
                ox -= w ? ho : 0;
                po += w ? 4 + 2 * H - 2 * ho : 4;
            }
        }
    }
    // col = lane & 31 (the B column), row = (e & 3) + 8 (e >> 2) + 4 h (the output channel)
#pragma unroll
    for (int u = 0; u < TPW; ++u) {
        const int col = (wave + 8 * u) * 32 + r;
        if (col >= K1) continue;
        float* o = part + (size_t)slice * 32 * K1 + col;
#pragma unroll
        for (int e = 0; e < 16; ++e) o[(size_t)((e & 3) + 8 * (e >> 2) + 4 * h) * K1] = acc[u][e];
    }
}

}  // namespace

extern "C" {

int tdmpc_lg_conv_fwd(const tdmpc_lg_conv* a, void* stream) {
    if (!a || !a->x || !a->w[0] || !a->b[0] || !a->y[0]) return TDMPC_E_NULL;
    if (a->nprob < 1 || a->nprob > 2 || (a->nprob == 2 && (!a->w[1] || !a->b[1] || !a->y[1])))
        return cv_bad("tdmpc_lg_conv_fwd: nprob");
    if (a->n <= 0 || a->cin <= 0 || a->k <= 0 || a->hin < a->k) return cv_bad("tdmpc_lg_conv_fwd: shape");
    const int ho = (a->hin - a->k) / 2 + 1, K = a->cin * a->k * a->k, K2 = (K + 1) & ~1;
    static bool attr = false;
    if (!attr) {
        if (hipFuncSetAttribute((const void*)conv_fwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) !=
                hipSuccess ||
            hipFuncSetAttribute((const void*)conv_fwd_slab_kernel<1, 1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                160 * 1024) != hipSuccess ||
            hipFuncSetAttribute((const void*)conv_fwd_slab_kernel<2, 1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                160 * 1024) != hipSuccess ||
            hipFuncSetAttribute((const void*)conv_fwd_slab_kernel<1, 2>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                160 * 1024) != hipSuccess ||
            hipFuncSetAttribute((const void*)conv_fwd_slab_kernel<2, 2>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                160 * 1024) != hipSuccess)
            return TDMPC_E_HIP;
        attr = true;
    }
    const int kk = a->k * a->k, H = a->hin;
    // the LDS-staged form for the large layers: slab rows of a 256 TP-pixel block (TP = 2 tiles per wave on both
    // large layers: two MFMA chains per weight read), channels per chunk within both caps
    const int TP = ho * ho >= 300 ? 2 : 1, BP = 256 * TP;
    const int SRM = std::min(H, 2 * (std::min(ho, (BP - 1) / ho + 2) - 1) + a->k);
    int CC = std::min(a->cin, std::min(CVS_SLAB / (SRM * H), CVS_KC / kk));
    if ((kk & 1) && CC < a->cin) CC &= ~1;   // (even k-values per chunk but the last: the direct kernel's MFMA pairs)
    if (ho * ho >= 256 && CC >= 1 && getenv("TDMPC_CONV_DIRECT") == nullptr) {
        const int KCM = (CC * kk + 1) & ~1, KT = ((KCM / 2) + 3) & ~3;
        const size_t lds = ((size_t)(((CC + 1) * SRM * H + 3) & ~3) + (size_t)a->nprob * KCM * 32 + 2 * KT) * 4;
        const dim3 grid((ho * ho + BP - 1) / BP, a->n);
        if (a->nprob == 2 && TP == 2)
            hipLaunchKernelGGL((conv_fwd_slab_kernel<2, 2>), grid, dim3(512), lds, (hipStream_t)stream, *a, ho, CC, SRM);
        else if (a->nprob == 2)
            hipLaunchKernelGGL((conv_fwd_slab_kernel<2, 1>), grid, dim3(512), lds, (hipStream_t)stream, *a, ho, CC, SRM);
        else if (TP == 2)
            hipLaunchKernelGGL((conv_fwd_slab_kernel<1, 2>), grid, dim3(512), lds, (hipStream_t)stream, *a, ho, CC, SRM);
        else
            hipLaunchKernelGGL((conv_fwd_slab_kernel<1, 1>), grid, dim3(512), lds, (hipStream_t)stream, *a, ho, CC, SRM);
        return hipGetLastError() == hipSuccess ? 0 : TDMPC_E_HIP;
    }
    const size_t lds = (size_t)K2 * 32 * 4 + (size_t)K2 * 4;
    if (lds > 160 * 1024) return cv_bad("tdmpc_lg_conv_fwd: cin k k too large");
    hipLaunchKernelGGL(conv_fwd_kernel, dim3((ho * ho + 127) / 128, a->n, a->nprob), dim3(256), lds,
                       (hipStream_t)stream, *a, ho, K2);
    return hipGetLastError() == hipSuccess ? 0 : TDMPC_E_HIP;
}

int tdmpc_lg_conv_bwd_data(const float* dy, const float* w, const float* xact, float* dx, int32_t n, int32_t cin,
                           int32_t hin, int32_t k, void* stream) {
    if (!dy || !w || !xact || !dx) return TDMPC_E_NULL;
    if (n <= 0 || cin != 32 || k <= 0 || hin < k) return cv_bad("tdmpc_lg_conv_bwd_data: shape (cin must be 32)");
    const int ho = (hin - k) / 2 + 1, kh = (k + 1) / 2, Kmax = 32 * kh * kh;
    const size_t lds = (size_t)Kmax * 32 * 4 + (size_t)Kmax * 8;
    if (lds > 160 * 1024) return cv_bad("tdmpc_lg_conv_bwd_data: kernel too large");
    static bool attr = false;
    if (!attr) {
        if (hipFuncSetAttribute((const void*)conv_bwd_data_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                160 * 1024) != hipSuccess)
            return TDMPC_E_HIP;
        attr = true;
    }
    const int pmax = ((hin + 1) / 2) * ((hin + 1) / 2);
    hipLaunchKernelGGL(conv_bwd_data_kernel, dim3((pmax + 127) / 128, 4, n), dim3(256), lds, (hipStream_t)stream, dy, w,
                       xact, dx, cin, hin, k, ho);
    return hipGetLastError() == hipSuccess ? 0 : TDMPC_E_HIP;
}

int tdmpc_lg_conv_bwd_weight(const float* dy, const float* x, float in_div, float* part, int32_t n, int32_t cin,
                             int32_t hin, int32_t k, int32_t img_per_slice, void* stream) {
    if (!dy || !x || !part) return TDMPC_E_NULL;
    if (n <= 0 || cin <= 0 || k <= 0 || hin < k || img_per_slice <= 0) return cv_bad("tdmpc_lg_conv_bwd_weight: shape");
    const int ho = (hin - k) / 2 + 1, ntile = (cin * k * k + 1 + 31) / 32;
    const int nsl = (n + img_per_slice - 1) / img_per_slice;
    if (ntile <= 32 && getenv("TDMPC_CONV_DIRECT") == nullptr) {
        // the largest even pixel block whose input slab fits 64 KB of LDS
        int PB = 0, SRM = 0;
        for (int pb = 256; pb >= 2 && !PB; pb /= 2) {
            const int srm = std::min(hin, 2 * (std::min(ho, (pb - 1) / ho + 2) - 1) + k);
            if (cin * srm * hin <= 16384) PB = pb, SRM = srm;
        }
        if (PB) {
            static bool attr = false;
            if (!attr) {
                if (hipFuncSetAttribute((const void*)conv_bwd_weight_slab_kernel<2>,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess ||
                    hipFuncSetAttribute((const void*)conv_bwd_weight_slab_kernel<4>,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess)
                    return TDMPC_E_HIP;
                attr = true;
            }
            const size_t lds = ((size_t)32 * (PB + 1) + (size_t)cin * SRM * hin) * 4;
            if (ntile <= 16)
                hipLaunchKernelGGL(conv_bwd_weight_slab_kernel<2>, dim3(nsl), dim3(512), lds, (hipStream_t)stream, dy, x,
                                   in_div, part, n, cin, hin, k, ho, img_per_slice, PB, SRM);
            else
                hipLaunchKernelGGL(conv_bwd_weight_slab_kernel<4>, dim3(nsl), dim3(512), lds, (hipStream_t)stream, dy, x,
                                   in_div, part, n, cin, hin, k, ho, img_per_slice, PB, SRM);
            return hipGetLastError() == hipSuccess ? 0 : TDMPC_E_HIP;
        }
    }
    hipLaunchKernelGGL(conv_bwd_weight_kernel, dim3((ntile + 3) / 4, nsl), dim3(256), 0, (hipStream_t)stream, dy, x,
                       in_div, part, n, cin, hin, k, ho, img_per_slice);
    return hipGetLastError() == hipSuccess ? 0 : TDMPC_E_HIP;
}

}  // extern "C"
