// learner_engine.hip -- the learner's forward / backward passes over the TOLD heads for MI355X (gfx950).
//
// Reference: TDMPC.update / update_pi / _td_target, /root/reference/src/algorithm/tdmpc.py:165-245, over the
// TOLD heads of helper.py:150-176 (enc, mlp, q) and TruncatedNormal.sample (helper.py:71-96). The reference
// runs them as ~1,500 one-op launches through autograd; tdmpc_amd/learner_engine.py runs the same math as ~80
// launches of four kernel families (include/tdmpc_learner.h):
//   * lg_gemm_kernel: grouped fp32 GEMM -- fp32-accurate x6 products on v_mfma_f32_32x32x16_bf16 by default (see
//     seg_loop_x6), exact v_mfma_f32_32x32x2_f32 products with TDMPC_LG_X6=0 -- with the bias, a residual, ELU /
//     policy-sampling / activation-backward epilogues fused.
//     Operands are read straight from L2 into the MFMA lane layout (each lane loads 4 consecutive k of its row /
//     column; the MFMA's two k slots per step are then k and k + 4, a permutation of the sum), four waves of a
//     workgroup split K and add through LDS, and up to 12 GEMMs of one pass (the heads, or every weight gradient
//     of an update) share one launch.
//   * lg_rows_fwd / lg_rows_bwd: one wave per row of 256 / 512 / 1024 features: LayerNorm + Tanh / ELU (+ the
//     scalar output layer of the Q and reward heads as a row dot), and their backward, with the column sums that
//     are the LayerNorm-affine and scalar-layer weight gradients written as per-workgroup partials.
//   * lg_finalize / lg_adam: the gradient slices summed in a fixed order into one flat gradient, the global
//     norm (clip_grad_norm_), Adam (torch.optim.Adam's update) over the flat parameter range; lg_lerp: the EMA.
// Every reduction runs in a fixed order (no float atomics), so a graph replay equals the eager pass bit for bit.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <type_traits>

#include "../../include/tdmpc_hip.h"
#include "../../include/tdmpc_learner.h"

namespace tdmpc_internal {
void set_error(const char* msg);
}

namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int LG_MAXJ = 12;
constexpr unsigned LG_OOB = 0x7ffffff0u;   // buffer range of the operand descriptors; offsets >= it read 0

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float4 u2f4(const u32x4 v) {
    return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}

struct KJob {
    tdmpc_lg_job j;
    int tiles_m, block0, nb_mem[3];
};
struct KArgs {
    KJob job[LG_MAXJ];
    int njobs;
    int diag;   // (timing diagnostics, TDMPC_LG_DIAG: macro tiles 1 no loads after the prologue, 2 no products;
                //  register tiles 4 no K loop, 8 no reduction / stores)
};

__device__ __forceinline__ float wsum(float v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ float elu_f(float x) { return x > 0.f ? x : expm1f(x); }

// One K segment [k_lo, k_hi) of a wave's 32TM x 32TN tile: lane (r = lane & 31, h = lane >> 5) holds k0 + 4h ..
// k0 + 4h + 3 of its rows / columns; MFMA step e then sums k0 + e and k0 + 4 + e. Waves take every fourth group
// of 8 k. Out-of-range rows / columns / k read a clamped (valid) address and are replaced by 0; the next group
// is loaded before the current one is multiplied.
template <int AM, int BM, bool AV, bool BV, int TM, int TN, int NW = 4>
__device__ __forceinline__ void seg_loop(const tdmpc_lg_seg& S, int nb_mem, int k_lo, int k_hi, int m0, int n0,
                                         int M, int N, floatx16 (&acc)[TM][TN], int wave, int r, int h) {
    constexpr int KS = 8 * NW;   // the k stride of one wave's groups
    const int kb0 = k_lo + 8 * wave;
    if (kb0 >= k_hi) return;
    const int nit = (k_hi - kb0 + KS - 1) / KS;
    const float* __restrict__ A = S.a;
    const float* __restrict__ B = S.b;
    const int lda = S.lda, ldb = S.ldb;
    int mrow[TM], ncol[TN];
    bool mok[TM], nok[TN], one[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const int m = m0 + 32 * i + r;
        mok[i] = m < M;
        mrow[i] = mok[i] ? m : M - 1;
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int n = n0 + 32 * j + r;
        nok[j] = n < N;
        one[j] = n == S.ones_col;
        ncol[j] = min(n, nb_mem - 1);
    }
    // buffer loads: an out-of-range offset returns 0 without a branch (a guarded plain load makes the compiler
    // branch around it and wait for every load in flight)
    const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, (int)LG_OOB, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsb = __builtin_amdgcn_make_buffer_rsrc((void*)B, (short)0, (int)LG_OOB, 0x00020000);
    auto load = [&](int kb, float4 (&a)[TM], float4 (&b)[TN]) {
        const bool kin = kb < k_hi;     // vector paths: whole groups of 8 (K % 8 == 0); past the end -> zeros
        const int kc = kb;
        const int k = kb + 4 * h;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            if constexpr (AM == 0 && AV) {
                const unsigned off = (mok[i] && kin) ? (unsigned)(mrow[i] * lda + kc + 4 * h) * 4u : LG_OOB;
                const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rsa, (int)off, 0, 0);
                a[i] = make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z),
                                   __uint_as_float(v.w));
            } else {
                float e[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const unsigned idx = AM == 0 ? (unsigned)(mrow[i] * lda + k + q) : (unsigned)((k + q) * lda + mrow[i]);
                    const unsigned off = (mok[i] && k + q < k_hi) ? idx * 4u : LG_OOB;
                    e[q] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsa, (int)off, 0, 0));
                }
                a[i] = make_float4(e[0], e[1], e[2], e[3]);
            }
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            if constexpr (BM == 0 && BV) {
                const unsigned off = (nok[j] && kin) ? (unsigned)(ncol[j] * ldb + kc + 4 * h) * 4u : LG_OOB;
                const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rsb, (int)off, 0, 0);
                b[j] = make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z),
                                   __uint_as_float(v.w));
            } else {
                float e[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const bool kv = k + q < k_hi;
                    const unsigned idx = BM == 0 ? (unsigned)(ncol[j] * ldb + k + q) : (unsigned)((k + q) * ldb + ncol[j]);
                    const unsigned off = (nok[j] && !one[j] && kv) ? idx * 4u : LG_OOB;
                    e[q] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsb, (int)off, 0, 0));
                }
                b[j] = make_float4(e[0], e[1], e[2], e[3]);
            }
        }
    };
    // a ring of D groups in flight: the loads of group g + D - 1 are issued (sched_barrier keeps them ahead of
    // the MFMAs) before group g is multiplied; groups past the end load zeros, so the trip count needs no tail
    // (deeper rings, 4 / 8 groups, measured 15-20 % slower on MI355X: the loads are throughput-, not latency-bound)
    constexpr int D = TM * TN >= 4 ? 2 : 4;
    float4 ra[D][TM], rb[D][TN];
#pragma unroll
    for (int d = 0; d < D - 1; ++d) load(kb0 + KS * d, ra[d], rb[d]);
    for (int it = 0; it < nit; it += D) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            load(kb0 + KS * (it + d + D - 1), ra[(d + D - 1) % D], rb[(d + D - 1) % D]);
            __builtin_amdgcn_sched_barrier(0);
            // (no arithmetic on freshly loaded registers before the barrier: it would wait for those loads)
            float4 bu[TN];
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                bu[j] = rb[d][j];
                if constexpr (AM == 1) {   // weight gradients: the bias column of ones, inside K only
                    const int k = kb0 + KS * (it + d) + 4 * h;
                    bu[j].x += (one[j] && k < k_hi) ? 1.f : 0.f;
                    bu[j].y += (one[j] && k + 1 < k_hi) ? 1.f : 0.f;
                    bu[j].z += (one[j] && k + 2 < k_hi) ? 1.f : 0.f;
                    bu[j].w += (one[j] && k + 3 < k_hi) ? 1.f : 0.f;
                }
            }
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(ra[d][i].x, bu[j].x, acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(ra[d][i].y, bu[j].y, acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(ra[d][i].z, bu[j].z, acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(ra[d][i].w, bu[j].w, acc[i][j], 0, 0, 0);
                }
            __builtin_amdgcn_sched_barrier(0);
        }
    }
}

// ---- x6 products (tdmpc_kernels.hip's chain kernels): both fp32 operands split exactly into three
// round-to-nearest bf16 parts x = hi + mid + lo, six v_mfma_f32_32x32x16_bf16 per product pair (hi.hi, hi.mid,
// mid.hi, hi.lo, lo.hi, mid.mid; the dropped mid.lo, lo.mid, lo.lo are <= 2^-25 of |a b| each), fp32 accumulation:
// fp32-accurate products at 6/16 of the f32 MFMA's cycles. (A non-finite operand gives NaN products, where an
// fp32 GEMM gives +-inf: the learner's losses are NaN either way.)
typedef __bf16 lg_bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void lg_split8(const float4& a0, const float4& a1, lg_bf16x8& bh, lg_bf16x8& bm,
                                          lg_bf16x8& bl) {
    const float x[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const __bf16 hi = (__bf16)x[e];
        const float r1 = __fsub_rn(x[e], (float)hi);
        const __bf16 mid = (__bf16)r1;
        bh[e] = hi;
        bm[e] = mid;
        bl[e] = (__bf16)__fsub_rn(r1, (float)mid);
    }
}

// One K segment of a wave's 32TM x 32TN tile on x6 products: lane (r, h) holds k0 + 8h .. k0 + 8h + 7 of its rows /
// columns (the 16-deep k group of one v_mfma_f32_32x32x16_bf16); waves take every NW-th group of 16 k.
template <int AM, int BM, bool AV, bool BV, int TM, int TN, int NW>
__device__ __forceinline__ void seg_loop_x6(const tdmpc_lg_seg& S, int nb_mem, int k_lo, int k_hi, int m0, int n0,
                                            int M, int N, floatx16 (&acc)[TM][TN], int wave, int r, int h) {
    constexpr int KS = 16 * NW;
    const int kb0 = k_lo + 16 * wave;
    if (kb0 >= k_hi) return;
    const int nit = (k_hi - kb0 + KS - 1) / KS;
    const int lda = S.lda, ldb = S.ldb;
    int mrow[TM], ncol[TN];
    bool mok[TM], nok[TN], one[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const int m = m0 + 32 * i + r;
        mok[i] = m < M;
        mrow[i] = mok[i] ? m : M - 1;
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int n = n0 + 32 * j + r;
        nok[j] = n < N;
        one[j] = n == S.ones_col;
        ncol[j] = min(n, nb_mem - 1);
    }
    const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc((void*)S.a, (short)0, (int)LG_OOB, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsb = __builtin_amdgcn_make_buffer_rsrc((void*)S.b, (short)0, (int)LG_OOB, 0x00020000);
    // 8 consecutive k of one row (MODE 0: element (x, k) at x * ld + k) or column (MODE 1: at k * ld + x)
    auto load8 = [&](auto MODE_, auto VEC_, const __amdgpu_buffer_rsrc_t& rs, int ld, int x, bool xok, bool zero,
                     int k, float4& v0, float4& v1) {
        constexpr int MODE = decltype(MODE_)::value;
        constexpr bool VEC = decltype(VEC_)::value;
        if constexpr (MODE == 0 && VEC) {   // (K % 8 == 0: a group's 8 k are all in or all out)
            const bool in = xok && !zero && k < k_hi;
            v0 = u2f4(__builtin_amdgcn_raw_buffer_load_b128(rs, (int)(in ? (unsigned)(x * ld + k) * 4u : LG_OOB), 0, 0));
            v1 = u2f4(__builtin_amdgcn_raw_buffer_load_b128(rs, (int)(in ? (unsigned)(x * ld + k + 4) * 4u : LG_OOB), 0, 0));
        } else {
            float e[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const unsigned idx = MODE == 0 ? (unsigned)(x * ld + k + q) : (unsigned)((k + q) * ld + x);
                const unsigned off = (xok && !zero && k + q < k_hi) ? idx * 4u : LG_OOB;
                e[q] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, (int)off, 0, 0));
            }
            v0 = make_float4(e[0], e[1], e[2], e[3]);
            v1 = make_float4(e[4], e[5], e[6], e[7]);
        }
    };
    using IA = std::integral_constant<int, AM>;
    using IB = std::integral_constant<int, BM>;
    using VA = std::integral_constant<bool, AV>;
    using VB = std::integral_constant<bool, BV>;
    auto load = [&](int kb, float4 (&a)[TM][2], float4 (&b)[TN][2]) {
        const int k = kb + 8 * h;
#pragma unroll
        for (int i = 0; i < TM; ++i) load8(IA{}, VA{}, rsa, lda, mrow[i], mok[i], false, k, a[i][0], a[i][1]);
#pragma unroll
        for (int j = 0; j < TN; ++j) load8(IB{}, VB{}, rsb, ldb, ncol[j], nok[j], one[j], k, b[j][0], b[j][1]);
    };
    constexpr int D = 2;
    float4 ra[D][TM][2], rb[D][TN][2];
    load(kb0, ra[0], rb[0]);
    for (int it = 0; it < nit; it += D) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            load(kb0 + KS * (it + d + 1), ra[(d + 1) % D], rb[(d + 1) % D]);
            __builtin_amdgcn_sched_barrier(0);
            lg_bf16x8 ah[TM], am[TM], al[TM], bh[TN], bm[TN], bl[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) lg_split8(ra[d][i][0], ra[d][i][1], ah[i], am[i], al[i]);
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                float4 b0 = rb[d][j][0], b1 = rb[d][j][1];
                if constexpr (AM == 1) {   // weight gradients: the bias column of ones, inside K only
                    const int k = kb0 + KS * (it + d) + 8 * h;
                    if (one[j]) {
                        b0 = make_float4(k < k_hi, k + 1 < k_hi, k + 2 < k_hi, k + 3 < k_hi);
                        b1 = make_float4(k + 4 < k_hi, k + 5 < k_hi, k + 6 < k_hi, k + 7 < k_hi);
                    }
                }
                lg_split8(b0, b1, bh[j], bm[j], bl[j]);
            }
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[i], bm[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[i], bh[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bm[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
                }
            __builtin_amdgcn_sched_barrier(0);
        }
    }
}

// One output element of a job: the split-K partial as is, else bias / residual / epilogue (tdmpc_lg_job).
__device__ __forceinline__ void lg_store(const tdmpc_lg_job& JJ, int splits, int split, int row, int col, float v) {
    if (splits > 1) {
        JJ.c[(size_t)split * JJ.slice + (size_t)row * JJ.ldc + col] = v;
        return;
    }
    float x = v;
    if (JJ.bias) x += JJ.bias[col];
    if (JJ.res) x += JJ.res[(size_t)row * JJ.ldres + col];
    switch (JJ.epi) {
    case TDMPC_LG_EPI_ELU: x = elu_f(x); break;
    case TDMPC_LG_EPI_PI: {
        const float mu = tanhf(x);
        const float e2 = fminf(fmaxf(JJ.std_ * JJ.aux[(size_t)row * JJ.ldaux + col], -0.3f), 0.3f);
        x = fminf(fmaxf(mu + e2, -1.0f + 1e-6f), 1.0f - 1e-6f);
        JJ.c2[(size_t)row * JJ.ldc2 + col] = mu;
        break;
    }
    case TDMPC_LG_EPI_ELU_BWD: {
        const float y = JJ.aux[(size_t)row * JJ.ldaux + col];
        x *= y > 0.f ? 1.f : y + 1.f;
        break;
    }
    case TDMPC_LG_EPI_PI_BWD: {
        const float mu = JJ.aux[(size_t)row * JJ.ldaux + col];
        x *= 1.f - mu * mu;
        break;
    }
    case TDMPC_LG_EPI_RELU_BWD:   // (threshold_backward: the gradient where the ReLU's output is > 0, else 0)
        x = JJ.aux[(size_t)row * JJ.ldaux + col] > 0.f ? x : 0.f;
        break;
    default:
        if (JJ.c2) JJ.c2[(size_t)row * JJ.ldc2 + col] = x;
    }
    JJ.c[(size_t)row * JJ.ldc + col] = x;
}

__device__ __forceinline__ bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// (amdgpu_waves_per_eu(2): left to itself the compiler gave the 64 x 64 form 224 VGPRs + 128 AGPRs, one wave per SIMD;
// bounded, 210 VGPRs and no spills: two)
// NW waves per workgroup split K (wave w takes every NW-th group of 8 k, 16 for x6). (8 and 16 waves -- 2 / 4 per
// SIMD, a wave's whole K share in flight at once -- measured no faster on the 512-row products and slower for the
// update: profiles/r06/lg_rollout_tiles.txt)
template <int TM, int TN, bool X6 = false, int NW = 4>
__global__ void __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(2))) lg_gemm_kernel(const KArgs P) {
    __shared__ float red[NW][TM * TN * 16][64];
    int jb = 0;
    for (int q = 1; q < P.njobs; ++q)
        if ((int)blockIdx.x >= P.job[q].block0) jb = q;
    const KJob& J = P.job[jb];
    const int local = (int)blockIdx.x - J.block0;
    const int splits = J.j.splits, split = local % splits, tile = local / splits;
    const int m0 = (tile % J.tiles_m) * 32 * TM, n0 = (tile / J.tiles_m) * 32 * TN;
    const int M = J.j.m, N = J.j.n;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;

    floatx16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

    for (int s = 0; s < (P.diag & 4 ? 0 : J.j.nseg); ++s) {
        const tdmpc_lg_seg& S = J.j.seg[s];
        int k_lo = 0, k_hi = S.k;
        if (splits > 1) {
            const int chunk = ((S.k + splits - 1) / splits + 7) & ~7;
            k_lo = min(S.k, split * chunk);
            k_hi = min(S.k, k_lo + chunk);
        }
        if (k_hi <= k_lo) continue;
        const int nbm = J.nb_mem[s];
        const bool av = S.amode == 0 && S.lda % 4 == 0 && S.k % 8 == 0 && al16(S.a);
        const bool bv = S.bmode == 0 && S.ldb % 4 == 0 && S.k % 8 == 0 && al16(S.b);
        if (S.amode == 1) {
            { if constexpr (X6) seg_loop_x6<1, 1, false, false, TM, TN, NW>(S, nbm, k_lo, k_hi, m0, n0, M, N, acc, wave, r, h); else seg_loop<1, 1, false, false, TM, TN, NW>(S, nbm, k_lo, k_hi, m0, n0, M, N, acc, wave, r, h); }
        } else if (S.bmode == 1) {
            if (av) { if constexpr (X6) seg_loop_x6<0, 1, true, false, TM, TN, NW>(S, nbm, k_lo, k_hi, m0, n0, M, N, acc, wave, r, h); else seg_loop<0, 1, true, false, TM, TN, NW>(S, nbm, k_lo, k_hi, m0, n0, M, N, acc, wave, r, h); }
            else { if constexpr (X6) seg_loop_x6<0, 1, false, false, TM, TN, NW>(S, nbm, k_lo, k_hi, m0, n0, M, N, acc, wave, r, h); else seg_loop<0, 1, false, false, TM, TN, NW>(S, nbm, k_lo, k_hi, m0, n0, M, N, acc, wave, r, h); }
        } else {
            if (av && bv) { if constexpr (X6) seg_loop_x6<0, 0, true, true, TM, TN, NW>(S, nbm, k_lo, k_hi, m0, n0, M, N, acc, wave, r, h); else seg_loop<0, 0, true, true, TM, TN, NW>(S, nbm, k_lo, k_hi, m0, n0, M, N, acc, wave, r, h); }
            else if (av) { if constexpr (X6) seg_loop_x6<0, 0, true, false, TM, TN, NW>(S, nbm, k_lo, k_hi, m0, n0, M, N, acc, wave, r, h); else seg_loop<0, 0, true, false, TM, TN, NW>(S, nbm, k_lo, k_hi, m0, n0, M, N, acc, wave, r, h); }
            else if (bv) { if constexpr (X6) seg_loop_x6<0, 0, false, true, TM, TN, NW>(S, nbm, k_lo, k_hi, m0, n0, M, N, acc, wave, r, h); else seg_loop<0, 0, false, true, TM, TN, NW>(S, nbm, k_lo, k_hi, m0, n0, M, N, acc, wave, r, h); }
            else { if constexpr (X6) seg_loop_x6<0, 0, false, false, TM, TN, NW>(S, nbm, k_lo, k_hi, m0, n0, M, N, acc, wave, r, h); else seg_loop<0, 0, false, false, TM, TN, NW>(S, nbm, k_lo, k_hi, m0, n0, M, N, acc, wave, r, h); }
        }
    }

    if (P.diag & 8) {   // (diagnostics: one store per lane keeps the products live)
        if (acc[0][0][0] == 12345.f) J.j.c[lane] = acc[0][0][1];
        return;
    }
    // the NW waves' K partials -> LDS; each wave finishes 1 / NW of the tile (C/D map of the 32x32 MFMA:
    // col = lane & 31, row = (e & 3) + 8 (e >> 2) + 4 (lane >> 5))
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) red[wave][(i * TN + j) * 16 + e][lane] = acc[i][j][e];
    __syncthreads();
    constexpr int QN = TM * TN * 16 / NW;
    const tdmpc_lg_job& JJ = J.j;
    for (int q = wave * QN; q < (wave + 1) * QN; ++q) {
        float v = red[0][q][lane];
#pragma unroll
        for (int w = 1; w < NW; ++w) v += red[w][q][lane];
        const int i = q / (TN * 16), j = (q / 16) % TN, e = q % 16;
        const int row = m0 + 32 * i + (e & 3) + 8 * (e >> 2) + 4 * h, col = n0 + 32 * j + r;
        if (row >= M || col >= N) continue;
        lg_store(JJ, splits, split, row, col, v);
    }
}

// ---- LDS-staged macro tiles (tdmpc_lg_gemm tile 3 / 4: 64 x 64 / 64 x 128 outputs per workgroup) for
// the large products (the heads' layers over H B = 2,560 - 3,072 rows, tdmpc.py:199-245). Four waves in 2 x 2, each
// a (32 TM) x (32 TN) tile of v_mfma_f32_32x32x2_f32 accumulators over ALL of K (no K split, no LDS reduction). K
// runs in chunks of 32 staged through LDS, double buffered: the next chunk's global loads are in flight in registers
// while the current chunk is multiplied, then go to the other buffer; one barrier per chunk. Per chunk and operand
// the LDS holds [kq = 0..7][row or column] float4s (k = 4 kq .. 4 kq + 3), each kq row padded by one float4 so the
// eight lanes of a ds_write_b128 group (one row, kq 0..7) land on eight different 16-B slots; MFMA lane (r, h) reads
// the float4 at kq = 2 g + h of its row / column r (16 consecutive float4 per ds_read_b128 lane group). The k order
// inside a group of 8 is lg_gemm's (steps .x .. .w pair k and k + 4), and the groups of 8 go to NACC chains by their
// index within the chunk: every output is a fixed-order sum of fixed-order f32 fma chains.
// FORM (one per launch, from the host): LGB_AV -- every A segment takes 16-B loads (row stride a multiple of 4,
// aligned base; a quad past K is zeroed), else four 4-B loads per float4; LGB_BT -- B(k, n) = b[k ldb + n] (bmode 1) for every segment, else
// b[n ldb + k]; LGB_BV -- (bmode 0) 16-B loads of B. Branch-free loads let the compiler count the ring's vmcnt.
enum { LGB_AV = 1, LGB_BT = 2, LGB_BV = 4 };

template <int TM, int TN, int FORM, int KC, int D>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) lg_big_kernel(const KArgs P) {
    constexpr bool AV = FORM & LGB_AV, BT = FORM & LGB_BT, BV = (FORM & LGB_BV) && !BT;
    constexpr int BM = 64 * TM, BN = 64 * TN, SA = BM + 1, SB = BN + 1;
    constexpr int KQ = KC / 4, NG = KC / 8;               // k quads and MFMA k groups of 8 per chunk
    constexpr int NA = BM * KQ / 256, NB = BN * KQ / 256;  // float4 per thread per chunk and operand
    constexpr int BUF = KQ * (SA + SB);                    // float4 per buffer
    constexpr int LC = KC == 64 ? 6 : 5;                   // log2 KC
    extern __shared__ float4 lg_lds[];
    int jb = 0;
    for (int q = 1; q < P.njobs; ++q)
        if ((int)blockIdx.x >= P.job[q].block0) jb = q;
    const KJob& J = P.job[jb];
    const int tile = (int)blockIdx.x - J.block0;
    const int m0 = (tile % J.tiles_m) * BM, n0 = (tile / J.tiles_m) * BN;
    const int M = J.j.m, N = J.j.n;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 31, h = lane >> 5;
    const int wm = (wave & 1) * 32 * TM, wn = (wave >> 1) * 32 * TN;

    // NACC independent accumulator chains per output tile (k group g of a chunk -> chain g % NACC, summed in a fixed
    // order at the end): one v_mfma_f32_32x32x2_f32 chain alone runs at about half the issue rate
    constexpr int NACC = TM * TN >= 4 ? 1 : 4 / (TM * TN);
    floatx16 acc[NACC][TM][TN];
#pragma unroll
    for (int q = 0; q < NACC; ++q)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int e = 0; e < 16; ++e) acc[q][i][j][e] = 0.f;

    // the segments' chunk ranges (nseg <= 3): chunk c is segment (c >= e0) + (c >= e1)
    const int nseg = J.j.nseg;
    const int c0n = (J.j.seg[0].k + KC - 1) >> LC;
    const int c1n = nseg > 1 ? (J.j.seg[1].k + KC - 1) >> LC : 0;
    const int c2n = nseg > 2 ? (J.j.seg[2].k + KC - 1) >> LC : 0;
    const int e0 = c0n, e1 = c0n + c1n, nch = e1 + c2n;

    float4 ra[D][NA], rb[D][NB];   // a ring of D chunks in flight in registers
    // chunk c of the job's segments -> registers (zeros past M / N / the segment's K)
    auto gload = [&](int c, float4 (&sa)[NA], float4 (&sb)[NB]) {
        const int s = (c >= e0) + (c >= e1);
        const tdmpc_lg_seg& S = J.j.seg[s];
        const int k0 = (c - (s >= 1 ? e0 : 0) - (s >= 2 ? c1n : 0)) * KC, kh = S.k, lda = S.lda, ldb = S.ldb;
        const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc((void*)S.a, (short)0, (int)LG_OOB, 0x00020000);
        const __amdgpu_buffer_rsrc_t rsb = __builtin_amdgcn_make_buffer_rsrc((void*)S.b, (short)0, (int)LG_OOB, 0x00020000);
#pragma unroll
        for (int i = 0; i < NA; ++i) {
            const int u = tid + 256 * i, m = m0 + u / KQ, k = k0 + 4 * (u % KQ);
            if constexpr (AV) {   // (a quad straddling K stays inside the row, lda % 4 == 0; its tail is zeroed)
                const unsigned off = (m < M && k < kh) ? (unsigned)(m * lda + k) * 4u : LG_OOB;
                sa[i] = u2f4(__builtin_amdgcn_raw_buffer_load_b128(rsa, (int)off, 0, 0));
                sa[i].y = k + 1 < kh ? sa[i].y : 0.f;
                sa[i].z = k + 2 < kh ? sa[i].z : 0.f;
                sa[i].w = k + 3 < kh ? sa[i].w : 0.f;
            } else {
                float e[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const unsigned off = (m < M && k + q < kh) ? (unsigned)(m * lda + k + q) * 4u : LG_OOB;
                    e[q] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsa, (int)off, 0, 0));
                }
                sa[i] = make_float4(e[0], e[1], e[2], e[3]);
            }
        }
#pragma unroll
        for (int j = 0; j < NB; ++j) {
            if constexpr (!BT) {   // B(k, n) = b[n ldb + k]: a Linear weight, k contiguous (as A)
                const int u = tid + 256 * j, n = n0 + u / KQ, k = k0 + 4 * (u % KQ);
                if constexpr (BV) {
                    const unsigned off = (n < N && k < kh) ? (unsigned)(n * ldb + k) * 4u : LG_OOB;
                    sb[j] = u2f4(__builtin_amdgcn_raw_buffer_load_b128(rsb, (int)off, 0, 0));
                    sb[j].y = k + 1 < kh ? sb[j].y : 0.f;
                    sb[j].z = k + 2 < kh ? sb[j].z : 0.f;
                    sb[j].w = k + 3 < kh ? sb[j].w : 0.f;
                } else {
                    float e[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const unsigned off = (n < N && k + q < kh) ? (unsigned)(n * ldb + k + q) * 4u : LG_OOB;
                        e[q] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsb, (int)off, 0, 0));
                    }
                    sb[j] = make_float4(e[0], e[1], e[2], e[3]);
                }
            } else {               // B(k, n) = b[k ldb + n]: a lane takes one column, 4 k (coalesced rows)
                const int u = tid + 256 * j, n = n0 + u % BN, k = k0 + 4 * (u / BN);
                float e[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const unsigned off = (n < N && k + q < kh) ? (unsigned)((k + q) * ldb + n) * 4u : LG_OOB;
                    e[q] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsb, (int)off, 0, 0));
                }
                sb[j] = make_float4(e[0], e[1], e[2], e[3]);
            }
        }
    };
    auto sstore = [&](float4* buf, const float4 (&sa)[NA], const float4 (&sb)[NB]) {
#pragma unroll
        for (int i = 0; i < NA; ++i) {
            const int u = tid + 256 * i;
            buf[(u % KQ) * SA + u / KQ] = sa[i];
        }
        float4* bs = buf + KQ * SA;
#pragma unroll
        for (int j = 0; j < NB; ++j) {
            const int u = tid + 256 * j;
            if constexpr (!BT) bs[(u % KQ) * SB + u / KQ] = sb[j];
            else bs[(u / BN) * SB + u % BN] = sb[j];
        }
    };
    // a chunk: all four k groups' operands read first (the reads of later groups land under earlier products)
    auto compute = [&](const float4* buf) {
        const float4* as = buf + wm + r;
        const float4* bs = buf + KQ * SA + wn + r;
        float4 a[NG][TM], b[NG][TN];
#pragma unroll
        for (int g = 0; g < NG; ++g) {
#pragma unroll
            for (int i = 0; i < TM; ++i) a[g][i] = as[(2 * g + h) * SA + 32 * i];
#pragma unroll
            for (int j = 0; j < TN; ++j) b[g][j] = bs[(2 * g + h) * SB + 32 * j];
        }
#pragma unroll
        for (int g = 0; g < NG; ++g)
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    floatx16& t = acc[g % NACC][i][j];
                    t = __builtin_amdgcn_mfma_f32_32x32x2f32(a[g][i].x, b[g][j].x, t, 0, 0, 0);
                    t = __builtin_amdgcn_mfma_f32_32x32x2f32(a[g][i].y, b[g][j].y, t, 0, 0, 0);
                    t = __builtin_amdgcn_mfma_f32_32x32x2f32(a[g][i].z, b[g][j].z, t, 0, 0, 0);
                    t = __builtin_amdgcn_mfma_f32_32x32x2f32(a[g][i].w, b[g][j].w, t, 0, 0, 0);
                }
    };

    // chunk c + 1 goes to LDS as chunk c is multiplied; chunk c + 1 + D is then loaded into its registers, so
    // every chunk's loads have D chunks of products to land. The barrier waits for the LDS stores only
    // (__syncthreads' fence would also drain the global loads in flight: vmcnt(0) every chunk)
    auto lds_barrier = [] { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
#pragma unroll
    for (int d = 0; d < D; ++d)
        if (d < nch) gload(d, ra[d], rb[d]);
    sstore(lg_lds, ra[0], rb[0]);
    if (D < nch) gload(D, ra[0], rb[0]);
    lds_barrier();
    for (int c0 = 0; c0 < nch; c0 += D) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const int c = c0 + d;
            if (c >= nch) break;
            // chunk c + 1 to the other buffer first (its last readers, chunk c - 1's products, passed the last
            // barrier): the stores then drain under chunk c's products
            const int dn = (d + 1) % D;
            if (c + 1 < nch) {
                sstore(lg_lds + ((c + 1) & 1) * BUF, ra[dn], rb[dn]);
                if (c + 1 + D < nch && !(P.diag & 1)) gload(c + 1 + D, ra[dn], rb[dn]);
            }
            if (!(P.diag & 2)) compute(lg_lds + (c & 1) * BUF);
            lds_barrier();
        }
    }

    // C/D map of the 32x32 MFMA: col = lane & 31, row = (e & 3) + 8 (e >> 2) + 4 (lane >> 5)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int row = m0 + wm + 32 * i + (e & 3) + 8 * (e >> 2) + 4 * h, col = n0 + wn + 32 * j + r;
                float v;
                if constexpr (NACC == 4) v = (acc[0][i][j][e] + acc[1][i][j][e]) + (acc[2][i][j][e] + acc[3][i][j][e]);
                else if constexpr (NACC == 2) v = acc[0][i][j][e] + acc[1][i][j][e];
                else v = acc[0][i][j][e];
                if (row < M && col < N) lg_store(J.j, 1, 0, row, col, v);
            }
}

template <int TM, int TN, int KC>
constexpr size_t lg_big_lds() { return (size_t)2 * (KC / 4) * (64 * TM + 1 + 64 * TN + 1) * sizeof(float4); }

// ---------------------------------------------------------------------------------------------------- rows
// Lane l of a row's wave holds features 4 l + 256 c + j (c < NC / 4, j < 4): 16-B loads and stores. Every head's
// row is loaded before the first reduction (the heads' latencies overlap).
template <int NC>
__global__ void __launch_bounds__(256) lg_rows_fwd_kernel(const tdmpc_lg_rows a) {
    constexpr int NQ = NC / 4;   // float4 per lane
    const int lane = threadIdx.x & 63;
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= a.rows) return;
    const int m = a.m;
    const float inv_m = 1.f / (float)m;
    float4 x[3][NQ];
#pragma unroll
    for (int hh = 0; hh < 3; ++hh)
        if (hh < a.nh) {
            const tdmpc_lg_rowhead& H = a.hd[hh];
#pragma unroll
            for (int c = 0; c < NQ; ++c) x[hh][c] = *(const float4*)(H.x + (size_t)r * H.ldx + 4 * lane + 256 * c);
        }
    float outv[3] = {0.f, 0.f, 0.f};
#pragma unroll
    for (int hh = 0; hh < 3; ++hh) {
        if (hh >= a.nh) break;
        const tdmpc_lg_rowhead& H = a.hd[hh];
        float v[NC];
#pragma unroll
        for (int c = 0; c < NQ; ++c) {
            v[4 * c] = x[hh][c].x; v[4 * c + 1] = x[hh][c].y; v[4 * c + 2] = x[hh][c].z; v[4 * c + 3] = x[hh][c].w;
        }
        if (H.ln) {
            float s = 0.f;
#pragma unroll
            for (int c = 0; c < NC; ++c) s += v[c];
            const float mean = wsum(s) * inv_m;
            float d = 0.f;
#pragma unroll
            for (int c = 0; c < NC; ++c) d += (v[c] - mean) * (v[c] - mean);
            const float rs = 1.f / sqrtf(wsum(d) * inv_m + 1e-5f);
#pragma unroll
            for (int c = 0; c < NQ; ++c) {
                const int n = 4 * lane + 256 * c;
                const float4 g = *(const float4*)(H.g + n), be = *(const float4*)(H.beta + n);
                float4 xh;
                xh.x = (v[4 * c] - mean) * rs; xh.y = (v[4 * c + 1] - mean) * rs;
                xh.z = (v[4 * c + 2] - mean) * rs; xh.w = (v[4 * c + 3] - mean) * rs;
                if (H.xhat) *(float4*)(H.xhat + (size_t)r * m + n) = xh;
                v[4 * c] = xh.x * g.x + be.x; v[4 * c + 1] = xh.y * g.y + be.y;
                v[4 * c + 2] = xh.z * g.z + be.z; v[4 * c + 3] = xh.w * g.w + be.w;
            }
            if (H.rstd && lane == 0) H.rstd[r] = rs;
        }
        float dot = 0.f;
#pragma unroll
        for (int c = 0; c < NQ; ++c) {
            const int n = 4 * lane + 256 * c;
            float y[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float u = v[4 * c + j];
                y[j] = H.act == 1 ? tanhf(u) : H.act == 2 ? elu_f(u) : u;
            }
            if (H.y) *(float4*)(H.y + (size_t)r * H.ldy + n) = make_float4(y[0], y[1], y[2], y[3]);
            if (H.tail) {
                const float4 w = *(const float4*)(H.w3 + n);
                dot += y[0] * w.x + y[1] * w.y + y[2] * w.z + y[3] * w.w;
            }
        }
        if (H.tail) {
            const float o = wsum(dot) + H.b3[0];
            outv[hh] = o;
            if (H.out && lane == 0) H.out[r] = o;
        }
    }
    if (a.td && lane == 0) a.td[r] = a.reward[r] + a.gamma * fminf(outv[0], outv[1]);
}

// NW waves per workgroup (16 for m <= 512: four rows in flight per SIMD), a wave per row, the workgroup's column
// partials summed over its waves in a fixed order; features as in lg_rows_fwd_kernel.
template <int NC, int NW>
__global__ void __launch_bounds__(64 * NW) lg_rows_bwd_kernel(const tdmpc_lg_rows a) {
    constexpr int NQ = NC / 4;
    __shared__ float red[NW][3 * NC * 64 + 1];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int m = a.m;
    const float inv_m = 1.f / (float)m;
    const int stride = gridDim.x * NW;
    for (int hh = 0; hh < a.nh; ++hh) {
        const tdmpc_lg_rowhead& H = a.hd[hh];
        float pg[NC], pb[NC], pw[NC], pq = 0.f;
#pragma unroll
        for (int c = 0; c < NC; ++c) pg[c] = pb[c] = pw[c] = 0.f;
        for (int r = blockIdx.x * NW + wave; r < a.rows; r += stride) {
            float d[NC], y[NC], xh[NC];
#pragma unroll
            for (int c = 0; c < NQ; ++c) {
                const float4 v = *(const float4*)(H.yact + (size_t)r * m + 4 * lane + 256 * c);
                y[4 * c] = v.x; y[4 * c + 1] = v.y; y[4 * c + 2] = v.z; y[4 * c + 3] = v.w;
                if (H.ln) {
                    const float4 u = *(const float4*)(H.xhat + (size_t)r * m + 4 * lane + 256 * c);
                    xh[4 * c] = u.x; xh[4 * c + 1] = u.y; xh[4 * c + 2] = u.z; xh[4 * c + 3] = u.w;
                }
                if (!H.tail) {
                    const float4 u = *(const float4*)(H.x + (size_t)r * H.ldx + 4 * lane + 256 * c);
                    d[4 * c] = u.x; d[4 * c + 1] = u.y; d[4 * c + 2] = u.z; d[4 * c + 3] = u.w;
                }
            }
            if (H.tail) {
                float dq;
                if (a.q1) {   // update_pi: d(-sum_t rho^t mean_b min(q1, q2)) / dq_head
                    const float q1 = a.q1[r], q2 = a.q2[r];
                    const float base = -a.rho[r / a.bsz] / (float)a.bsz;
                    dq = q1 == q2 ? 0.5f * base : ((q1 < q2) == (hh == 0) ? base : 0.f);
                } else {
                    dq = H.dq[r];
                }
#pragma unroll
                for (int c = 0; c < NQ; ++c) {
                    const float4 w = *(const float4*)(H.w3 + 4 * lane + 256 * c);
                    d[4 * c] = dq * w.x; d[4 * c + 1] = dq * w.y; d[4 * c + 2] = dq * w.z; d[4 * c + 3] = dq * w.w;
                }
#pragma unroll
                for (int c = 0; c < NC; ++c) pw[c] += dq * y[c];
                pq += dq;
            }
#pragma unroll
            for (int c = 0; c < NC; ++c)
                d[c] *= H.act == 1 ? 1.f - y[c] * y[c] : H.act == 2 ? (y[c] > 0.f ? 1.f : y[c] + 1.f) : 1.f;
            if (H.ln) {
                const float rs = H.rstd[r];
                float s1 = 0.f, s2 = 0.f;
#pragma unroll
                for (int c = 0; c < NQ; ++c) {
                    const float4 g = *(const float4*)(H.g + 4 * lane + 256 * c);
                    const float gg[4] = {g.x, g.y, g.z, g.w};
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int e = 4 * c + j;
                        pb[e] += d[e];
                        pg[e] += d[e] * xh[e];
                        d[e] *= gg[j];
                        s1 += d[e];
                        s2 += d[e] * xh[e];
                    }
                }
                s1 = wsum(s1) * inv_m;
                s2 = wsum(s2) * inv_m;
#pragma unroll
                for (int c = 0; c < NC; ++c) d[c] = rs * (d[c] - s1 - xh[c] * s2);
            }
#pragma unroll
            for (int c = 0; c < NQ; ++c)
                *(float4*)(H.y + (size_t)r * H.ldy + 4 * lane + 256 * c) =
                    make_float4(d[4 * c], d[4 * c + 1], d[4 * c + 2], d[4 * c + 3]);
        }
        if (!H.part) continue;
        // partial column sums of this workgroup: [dg (m), dbeta (m)] if ln, then [dW3 (m), db3] if tail; feature n of
        // element e = 4 c + j is 4 lane + 256 c + j
#pragma unroll
        for (int c = 0; c < NQ; ++c)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int n = 4 * lane + 256 * c + j, e = 4 * c + j;
                red[wave][n] = pg[e];
                red[wave][m + n] = pb[e];
                red[wave][2 * m + n] = pw[e];
            }
        if (lane == 0) red[wave][3 * m] = pq;   // the same in every lane (dq is a per-row scalar)
        __syncthreads();
        const int pw_n = (H.ln ? 2 * m : 0) + (H.tail ? m + 1 : 0);
        float* out = H.part + (size_t)blockIdx.x * pw_n;
        for (int i = threadIdx.x; i < pw_n; i += 64 * NW) {
            int src;
            if (H.ln && i < 2 * m) src = i;                       // dg | dbeta
            else {
                const int t = i - (H.ln ? 2 * m : 0);
                src = t < m ? 2 * m + t : 3 * m;                  // dW3 | db3
            }
            float v = red[0][src];
#pragma unroll
            for (int w = 1; w < NW; ++w) v += red[w][src];
            out[i] = v;
        }
        __syncthreads();
    }
}

__global__ void __launch_bounds__(256) lg_pi_loss_kernel(const float* q1, const float* q2, const float* rho,
                                                         int nt, int bsz, float* out) {
    __shared__ float red[4];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    float loss = 0.f;
    for (int t = 0; t < nt; ++t) {
        float s = 0.f;
        for (int b = threadIdx.x; b < bsz; b += 256) s += fminf(q1[t * bsz + b], q2[t * bsz + b]);
        s = wsum(s);
        if (lane == 0) red[wave] = s;
        __syncthreads();
        const float tot = red[0] + red[1] + red[2] + red[3];
        __syncthreads();
        loss += -(tot / (float)bsz) * rho[t];
    }
    if (threadIdx.x == 0) out[0] = loss;
}

// ------------------------------------------------------------------------------------------ optimiser
constexpr int LG_MAXT = 48;
constexpr int LG_FIN_PER = 2048;   // gradient elements per lg_finalize workgroup (8 per thread)
constexpr int LG_FIN_MANY = 32;    // from this many slices a workgroup sums 64 elements with all its threads
struct FArgs {
    tdmpc_lg_gsrc t[LG_MAXT];
    int block0[LG_MAXT];
    int nt;
};

__device__ __forceinline__ float block_sum256(float v, float* red) {
    v = wsum(v);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) red[wave] = v;
    __syncthreads();
    return red[0] + red[1] + red[2] + red[3];
}

// workgroup -> (tensor, chunk): 2048 elements of a tensor with few slices (8 per thread), or 64 elements of one
// with many (the row kernels' per-workgroup column sums: 4 thread groups split the slices, 8 loads in flight
// each, combined in a fixed order)
__global__ void __launch_bounds__(256) lg_finalize_kernel(const FArgs F, float* g, float* normp, int* step) {
    __shared__ float red[4];
    __shared__ float part[4][64];
    int ti = 0;
    for (int q = 1; q < F.nt; ++q)
        if ((int)blockIdx.x >= F.block0[q]) ti = q;
    const tdmpc_lg_gsrc& T = F.t[ti];
    const int n = T.rows * T.cols;
    float sq = 0.f;
    if (T.nslices < LG_FIN_MANY) {
        const int e0 = (blockIdx.x - F.block0[ti]) * LG_FIN_PER;
#pragma unroll
        for (int u = 0; u < LG_FIN_PER / 256; ++u) {
            const int loc = e0 + u * 256 + threadIdx.x;
            if (loc < n) {
                const int rr = loc / T.cols, cc = loc - rr * T.cols;
                const float* p = T.src + (size_t)rr * T.ld + cc;
                float v = 0.f;
                for (int k = 0; k < T.nslices; ++k) v += p[(size_t)k * T.sstride];
                g[T.dst + loc] = v;
                sq += v * v;
            }
        }
    } else {
        const int e = threadIdx.x & 63, grp = threadIdx.x >> 6;
        const int loc = (blockIdx.x - F.block0[ti]) * 64 + e;
        float v = 0.f;
        if (loc < n) {
            const int rr = loc / T.cols, cc = loc - rr * T.cols;
            const float* p = T.src + (size_t)rr * T.ld + cc;
            float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            int k = grp;
            for (; k + 28 < T.nslices; k += 32) {
#pragma unroll
                for (int u = 0; u < 8; ++u) acc[u] += p[(size_t)(k + 4 * u) * T.sstride];
            }
            for (int u = 0; k < T.nslices; k += 4, ++u) acc[u & 7] += p[(size_t)k * T.sstride];
            v = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
        }
        part[grp][e] = v;
        __syncthreads();
        if (grp == 0 && loc < n) {
            const float t = (part[0][e] + part[1][e]) + (part[2][e] + part[3][e]);
            g[T.dst + loc] = t;
            sq = t * t;
        }
    }
    const float tot = block_sum256(sq, red);
    if (threadIdx.x == 0) {
        normp[blockIdx.x] = tot;
        if (blockIdx.x == 0 && step) step[0] += 1;
    }
}

__global__ void __launch_bounds__(256) lg_adam_kernel(float* p, float* g, float* m, float* v, long n,
                                                      const float* normp, int nblk, const int* step, float lr,
                                                      float b1, float b2, float eps, float max_norm,
                                                      float* norm_out) {
    __shared__ float red[4];
    float s = 0.f;
    for (int i = threadIdx.x; i < nblk; i += 256) s += normp[i];
    const float total = sqrtf(block_sum256(s, red));
    // torch.nn.utils.clip_grad_norm_ as the reference's pinned torch 1.9 runs it (/root/reference/environment.yaml:6):
    // `if clip_coef < 1: grad.mul_(clip_coef)`. A NaN norm fails the test, so the gradients go unscaled and only the
    // entries whose gradient is NaN turn NaN (torch >= 1.13 clamps instead and poisons every parameter); an inf norm
    // scales by 0. fminf(NaN, 1) = 1 is exactly that test.
    const float coef = fminf(max_norm / (total + 1e-6f), 1.0f);
    if (blockIdx.x == 0 && threadIdx.x == 0 && norm_out) norm_out[0] = total;
    const int t = step[0];
    const double bc1 = 1.0 - pow((double)b1, (double)t), bc2 = 1.0 - pow((double)b2, (double)t);
    const float step_size = (float)(lr / bc1);
    const float bc2_sqrt = (float)sqrt(bc2);
    auto upd = [&](float& pi, float& gr, float& mi, float& vi) {
        const float gi = gr * coef;
        gr = gi;   // (clip_grad_norm_ leaves the clipped gradient in .grad)
        mi = mi + (1.f - b1) * (gi - mi);         // exp_avg.lerp_(grad, 1 - beta1)
        vi = vi * b2 + (1.f - b2) * gi * gi;      // exp_avg_sq.mul_(beta2).addcmul_(g, g, 1 - beta2)
        const float denom = sqrtf(vi) / bc2_sqrt + eps;
        pi = pi - step_size * (mi / denom);
    };
    // 16-B accesses where the four ranges are 16-B aligned (the engine's flat buffers are), the tail by elements
    const bool vec = (((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) == 0;
    const long n4 = vec ? n / 4 : 0;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
        float4 P4 = ((float4*)p)[i], G4 = ((float4*)g)[i], M4 = ((float4*)m)[i], V4 = ((float4*)v)[i];
        upd(P4.x, G4.x, M4.x, V4.x);
        upd(P4.y, G4.y, M4.y, V4.y);
        upd(P4.z, G4.z, M4.z, V4.z);
        upd(P4.w, G4.w, M4.w, V4.w);
        ((float4*)p)[i] = P4;
        ((float4*)g)[i] = G4;
        ((float4*)m)[i] = M4;
        ((float4*)v)[i] = V4;
    }
    for (long i = 4 * n4 + (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
        upd(p[i], g[i], m[i], v[i]);
}

__global__ void __launch_bounds__(256) lg_lerp_kernel(float* t, const float* p, long n, float w) {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
        const float a = t[i], b = p[i];
        t[i] = w < 0.5f ? a + w * (b - a) : b - (b - a) * (1.f - w);
    }
}

__global__ void __launch_bounds__(256) lg_act_kernel(float4* x, const float4* y, long n4, int mode) {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
        float4 v = x[i];
        if (mode == 0) {
            v = make_float4(elu_f(v.x), elu_f(v.y), elu_f(v.z), elu_f(v.w));
        } else {
            const float4 a = y[i];
            v.x *= a.x > 0.f ? 1.f : a.x + 1.f;
            v.y *= a.y > 0.f ? 1.f : a.y + 1.f;
            v.z *= a.z > 0.f ? 1.f : a.z + 1.f;
            v.w *= a.w > 0.f ? 1.f : a.w + 1.f;
        }
        x[i] = v;
    }
}

int fail(hipError_t e, const char* what) {
    char msg[256];
    snprintf(msg, sizeof msg, "learner_engine %s: %s", what, hipGetErrorString(e));
    tdmpc_internal::set_error(msg);
    return TDMPC_E_HIP;
}

int bad(const char* what) {
    tdmpc_internal::set_error(what);
    return TDMPC_E_DIMS;
}

int launched(const char* what) {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : fail(e, what);
}

}  // namespace

extern "C" {

int tdmpc_lg_gemm(const tdmpc_lg_job* jobs, int32_t njobs, int32_t tile, void* stream) {
    if (!jobs) return TDMPC_E_NULL;
    const bool x6 = !(tile & TDMPC_LG_TILE_EXACT);   // x6 products unless the caller asks for the exact f32 MFMA
    tile &= ~TDMPC_LG_TILE_EXACT;
    if (njobs <= 0 || njobs > LG_MAXJ || tile < 1 || tile > 4) return bad("tdmpc_lg_gemm: njobs / tile");
    KArgs P;
    memset(&P, 0, sizeof P);
    const bool big = tile == 3 || tile == 4;   // LDS-staged macro tiles (exact f32 MFMA)
    const int twm = tile == 1 ? 32 : 64, twn = tile == 1 ? 32 : tile == 2 || tile == 3 ? 64 : 128;
    long blocks = 0;
    for (int q = 0; q < njobs; ++q) {
        const tdmpc_lg_job& j = jobs[q];
        if (!j.c || j.m <= 0 || j.n <= 0 || j.nseg < 1 || j.nseg > 3 || j.splits < 1 || j.splits > 64)
            return bad("tdmpc_lg_gemm: job shape");
        if (big && j.splits != 1) return bad("tdmpc_lg_gemm: split-K job on a macro tile");
        for (int s = 0; s < j.nseg && big; ++s)
            if (j.seg[s].amode != 0 || j.seg[s].ones_col >= 0) return bad("tdmpc_lg_gemm: macro tiles take amode 0 only");
        if (j.splits > 1 && (j.bias || j.res || j.epi != TDMPC_LG_EPI_NONE || j.c2))
            return bad("tdmpc_lg_gemm: split-K job with an epilogue");
        if ((j.epi == TDMPC_LG_EPI_PI && (!j.aux || !j.c2)) ||
            ((j.epi == TDMPC_LG_EPI_ELU_BWD || j.epi == TDMPC_LG_EPI_PI_BWD || j.epi == TDMPC_LG_EPI_RELU_BWD) && !j.aux))
            return bad("tdmpc_lg_gemm: epilogue operand missing");
        P.job[q].j = j;
        for (int s = 0; s < j.nseg; ++s) {
            const tdmpc_lg_seg& S = j.seg[s];
            if (!S.a || (!S.b && S.ones_col < 0) || S.k <= 0) return bad("tdmpc_lg_gemm: segment");
            if (S.amode == 1 && S.bmode != 1) return bad("tdmpc_lg_gemm: amode 1 needs bmode 1");
            // columns of B that exist in memory: all N, or those before the ones column
            P.job[q].nb_mem[s] = S.ones_col >= 0 ? S.ones_col : j.n;
            if (P.job[q].nb_mem[s] < 1) return bad("tdmpc_lg_gemm: ones column");
        }
        const int tm = (j.m + twm - 1) / twm, tn = (j.n + twn - 1) / twn;
        P.job[q].tiles_m = tm;
        P.job[q].block0 = (int)blocks;
        blocks += (long)tm * tn * j.splits;
    }
    P.njobs = njobs;
    static const int diag = getenv("TDMPC_LG_DIAG") ? atoi(getenv("TDMPC_LG_DIAG")) : 0;
    P.diag = diag;
    if (blocks >= (1L << 31)) return bad("tdmpc_lg_gemm: grid");
    const dim3 g((unsigned)blocks), b(256);
    if (big) {
        // one operand form per launch (lg_big_kernel FORM)
        bool av = true, bv = true;
        const int bt = jobs[0].seg[0].bmode;
        for (int q = 0; q < njobs; ++q)
            for (int s = 0; s < jobs[q].nseg; ++s) {
                const tdmpc_lg_seg& S = jobs[q].seg[s];
                if (S.bmode != bt) return bad("tdmpc_lg_gemm: macro tiles take one bmode per launch");
                av = av && S.lda % 4 == 0 && S.lda >= S.k && ((uintptr_t)S.a & 15) == 0;
                bv = bv && S.ldb % 4 == 0 && S.ldb >= S.k && ((uintptr_t)S.b & 15) == 0;
            }
        const int form = (av ? LGB_AV : 0) | (bt ? LGB_BT : (bv ? LGB_BV : 0));
        // (development knob: the chunk depth of the macro tiles)
        static const int kc = getenv("TDMPC_LG_BIG_KC") ? atoi(getenv("TDMPC_LG_BIG_KC")) : 32;
        static bool attr = false;
#define LG_BIG_FORMS(X, TM, TN, KC) X(TM, TN, 0, KC) X(TM, TN, 1, KC) X(TM, TN, 2, KC) X(TM, TN, 3, KC) X(TM, TN, 4, KC) X(TM, TN, 5, KC)
#define LG_BIG_EACH(X) LG_BIG_FORMS(X, 1, 1, 32) LG_BIG_FORMS(X, 1, 2, 32) LG_BIG_FORMS(X, 1, 1, 64) LG_BIG_FORMS(X, 1, 2, 64)
        if (!attr) {
#define LG_BIG_ATTR(TM, TN, F, KC) \
            if (hipFuncSetAttribute((const void*)lg_big_kernel<TM, TN, F, KC, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                    (int)lg_big_lds<TM, TN, KC>()) != hipSuccess) \
                return fail(hipGetLastError(), "gemm (LDS attribute)");
            LG_BIG_EACH(LG_BIG_ATTR)
#undef LG_BIG_ATTR
            attr = true;
        }
        const int tm = 1, tn = tile == 3 ? 1 : 2;
        bool done = false;
#define LG_BIG_LAUNCH(TM, TN, F, KC) \
        if (!done && tm == TM && tn == TN && form == F && kc == KC) { \
            constexpr size_t lds = lg_big_lds<TM, TN, KC>(); \
            hipLaunchKernelGGL((lg_big_kernel<TM, TN, F, KC, 2>), g, b, lds, (hipStream_t)stream, P); \
            done = true; \
        }
        LG_BIG_EACH(LG_BIG_LAUNCH)
#undef LG_BIG_LAUNCH
#undef LG_BIG_EACH
#undef LG_BIG_FORMS
        if (!done) return bad("tdmpc_lg_gemm: macro tile form / chunk");
        return launched("gemm (macro tiles)");
    }
    if (tile == 1 && x6) hipLaunchKernelGGL((lg_gemm_kernel<1, 1, true>), g, b, 0, (hipStream_t)stream, P);
    else if (tile == 1) hipLaunchKernelGGL((lg_gemm_kernel<1, 1>), g, b, 0, (hipStream_t)stream, P);
    else if (x6) hipLaunchKernelGGL((lg_gemm_kernel<2, 2, true>), g, b, 0, (hipStream_t)stream, P);
    else hipLaunchKernelGGL((lg_gemm_kernel<2, 2>), g, b, 0, (hipStream_t)stream, P);
    return launched("gemm");
}

static int rows_ok(const tdmpc_lg_rows* a) {
    if (!a) return TDMPC_E_NULL;
    if (a->nh < 1 || a->nh > 3 || a->rows <= 0 || (a->m != 256 && a->m != 512 && a->m != 1024))
        return bad("tdmpc_lg_rows: nh / rows / m");
    for (int h = 0; h < a->nh; ++h) {   // 16-B row accesses
        const tdmpc_lg_rowhead& H = a->hd[h];
        const void* ps[] = {H.x, H.y, H.xhat, H.yact, H.g, H.beta, H.w3};
        for (const void* q : ps)
            if ((uintptr_t)q & 15) return bad("tdmpc_lg_rows: a row operand is not 16-B aligned");
        if ((H.x && H.ldx % 4) || (H.y && H.ldy % 4)) return bad("tdmpc_lg_rows: row strides must be multiples of 4");
    }
    return 0;
}

int tdmpc_lg_rows_fwd(const tdmpc_lg_rows* a, void* stream) {
    if (int rc = rows_ok(a)) return rc;
    if (a->td && (a->nh < 2 || !a->reward)) return bad("tdmpc_lg_rows_fwd: td needs two tail heads");
    const dim3 g((a->rows + 3) / 4);
    hipStream_t s = (hipStream_t)stream;
    if (a->m == 256) hipLaunchKernelGGL(lg_rows_fwd_kernel<4>, g, dim3(256), 0, s, *a);
    else if (a->m == 512) hipLaunchKernelGGL(lg_rows_fwd_kernel<8>, g, dim3(256), 0, s, *a);
    else hipLaunchKernelGGL(lg_rows_fwd_kernel<16>, g, dim3(256), 0, s, *a);
    return launched("rows_fwd");
}

int tdmpc_lg_rows_bwd(const tdmpc_lg_rows* a, int32_t nwg, void* stream) {
    if (int rc = rows_ok(a)) return rc;
    if (nwg < 1 || nwg > 4096) return bad("tdmpc_lg_rows_bwd: nwg");
    for (int h = 0; h < a->nh; ++h) {
        const tdmpc_lg_rowhead& H = a->hd[h];
        if (!H.y || !H.yact || (H.ln && (!H.xhat || !H.rstd || !H.g)) || (H.tail && (!H.w3 || (!H.dq && !a->q1))) ||
            (!H.tail && !H.x))
            return TDMPC_E_NULL;
    }
    hipStream_t s = (hipStream_t)stream;
    if (a->m == 256) hipLaunchKernelGGL((lg_rows_bwd_kernel<4, 16>), dim3(nwg), dim3(1024), 0, s, *a);
    else if (a->m == 512) hipLaunchKernelGGL((lg_rows_bwd_kernel<8, 16>), dim3(nwg), dim3(1024), 0, s, *a);
    else hipLaunchKernelGGL((lg_rows_bwd_kernel<16, 4>), dim3(nwg), dim3(256), 0, s, *a);
    return launched("rows_bwd");
}

int tdmpc_lg_pi_loss(const float* q1, const float* q2, const float* rho, int32_t nt, int32_t bsz, float* out,
                     void* stream) {
    if (!q1 || !q2 || !rho || !out) return TDMPC_E_NULL;
    if (nt <= 0 || bsz <= 0) return bad("tdmpc_lg_pi_loss: dims");
    hipLaunchKernelGGL(lg_pi_loss_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, q1, q2, rho, nt, bsz, out);
    return launched("pi_loss");
}

int tdmpc_lg_finalize(const tdmpc_lg_gsrc* t, int32_t nt, float* g, float* normp, int32_t nblk, int32_t* step,
                      void* stream) {
    if (!t || !g || !normp) return TDMPC_E_NULL;
    if (nt <= 0 || nt > LG_MAXT || nblk <= 0) return bad("tdmpc_lg_finalize: nt / nblk");
    FArgs F;
    memset(&F, 0, sizeof F);
    long off = 0;
    int blocks = 0;
    for (int i = 0; i < nt; ++i) {
        if (!t[i].src || t[i].dst < off || t[i].rows <= 0 || t[i].cols <= 0 || t[i].nslices <= 0 ||
            t[i].ld < t[i].cols)
            return bad("tdmpc_lg_finalize: tensors must lie in order without overlap");
        off = t[i].dst;
        F.t[i] = t[i];
        F.block0[i] = blocks;
        const long n = (long)t[i].rows * t[i].cols;
        off += n;
        const int per = t[i].nslices < LG_FIN_MANY ? LG_FIN_PER : 64;
        blocks += (int)((n + per - 1) / per);
    }
    if (blocks > nblk) return bad("tdmpc_lg_finalize: normp holds fewer entries than workgroups");
    F.nt = nt;
    hipLaunchKernelGGL(lg_finalize_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, F, g, normp, step);
    return launched("finalize");
}

int tdmpc_lg_adam(float* p, float* g, float* m, float* v, int64_t n, const float* normp, int32_t nblk,
                  const int32_t* step, float lr, float beta1, float beta2, float eps, float max_norm,
                  float* norm_out, void* stream) {
    if (!p || !g || !m || !v || !normp || !step) return TDMPC_E_NULL;
    if (n <= 0 || nblk <= 0) return bad("tdmpc_lg_adam: dims");
    const unsigned blocks = (unsigned)std::min<long>((n / 4 + 255) / 256 + 1, 1024);
    hipLaunchKernelGGL(lg_adam_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, p, g, m, v, (long)n, normp,
                       nblk, step, lr, beta1, beta2, eps, max_norm, norm_out);
    return launched("adam");
}

int tdmpc_lg_lerp(float* t, const float* p, int64_t n, float w, void* stream) {
    if (!t || !p) return TDMPC_E_NULL;
    if (n <= 0) return bad("tdmpc_lg_lerp: n");
    const unsigned blocks = (unsigned)std::min<long>((n + 255) / 256, 2048);
    hipLaunchKernelGGL(lg_lerp_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, t, p, (long)n, w);
    return launched("lerp");
}

int tdmpc_lg_act(float* x, const float* y, int64_t n, int32_t mode, void* stream) {
    if (!x || (mode == 1 && !y)) return TDMPC_E_NULL;
    if (n <= 0 || n % 4 || (mode != 0 && mode != 1)) return bad("tdmpc_lg_act: n / mode");
    if (((uintptr_t)x & 15) || (y && ((uintptr_t)y & 15))) return bad("tdmpc_lg_act: alignment");
    const unsigned blocks = (unsigned)std::min<long>((n / 4 + 255) / 256, 2048);
    hipLaunchKernelGGL(lg_act_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (float4*)x, (const float4*)y,
                       (long)(n / 4), mode);
    return launched("act");
}

}  // extern "C"
