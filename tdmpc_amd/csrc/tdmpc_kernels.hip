// tdmpc_kernels.hip -- MI355X (gfx950 / CDNA4) kernels for TD-MPC planning (TDMPC.plan + TOLD rollout).
//
// Reference behaviour: /root/reference/src/algorithm/tdmpc.py:83-163 (plan, estimate_value) and the TOLD
// heads tdmpc.py:30-50 built from helper.py:119-133 (enc), 169-176 (mlp), 197-201 (q), 71-96
// (TruncatedNormal). See DESIGN.md for the decomposition, data layout and rooflines.
//
// Kernel families
//   linear_kernel<WN,PRO,KCH>  fused Linear layer on f32 MFMA (v_mfma_f32_32x32x2_f32): one workgroup owns
//                              a 32-row x (32*WN)-column output tile, its waves split K, the partial tiles
//                              are reduced through LDS and a fused epilogue applies bias + ELU / tanh +
//                              TruncatedNormal sampling / LayerNorm partial moments / reward-head dot /
//                              discounted-return accumulation. Prologue may apply LayerNorm + act to A.
//   value_kernel               Q heads' LayerNorm+ELU+Linear(512->1), min(Q1,Q2), G + gamma^H Q, nan_to_num.
//   cem_kernel                 one workgroup per env: top-k, softmax, weighted mean/std refit, momentum,
//                              next-iteration sampling, final elite choice (np.random.choice cdf).
//   encode_state_kernel / conv kernels   TOLD.h for state / pixel observations, z0 broadcast.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <string.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "../../include/tdmpc_hip.h"

typedef float floatx16 __attribute__((ext_vector_type(16)));

#define DEVI __device__ __forceinline__

namespace {

thread_local char g_err[512] = "";

__host__ __device__ inline size_t rup(size_t x, size_t a) { return (x + a - 1) / a * a; }

// ------------------------------------------------------------------------------------------------ layout
// Packed parameter buffer (float offsets, each tensor 64-float aligned). X rows are [a | 0 | z | 0]:
// action columns first so that every 8-wide K group of the MFMA loop is all-action or all-latent.
struct Layout {
    int A, L, M, E, Ap, Lp, Kx, Ar, Lr;
    int modality, obs_dim, img_c, img_hw, nch, conv_hw[5], flat;
    size_t enc_w1, enc_b1, enc_w2, enc_b2;           // state encoder (raw nn.Linear layouts)
    size_t cw[4], cb[4], pl_w, pl_b;                 // pixel encoder
    size_t w1x, b1x;                                 // [2M][Kx]: dynamics.0 rows then reward.0 rows
    size_t w2d, b2d, w2r, b2r;                       // [M][M]
    size_t w3d, b3d, w3r, b3r;                       // [Lr][M], [M]
    size_t wp1, bp1, wp2, bp2, wp3, bp3;             // pi: [M][Lp], [M][M], [Ar][M]
    size_t wq1x, bq1x, g1, be1;                      // [2M][Kx], LN1 gamma/beta [2M]
    size_t wq2, bq2, g2, be2;                        // [2][M][M], LN2 [2M]
    size_t wq3, bq3;                                 // [2][M], [2]
    size_t total;
};

bool make_layout(const tdmpc_dims* d, Layout* w) {
    if (!d || d->action_dim <= 0 || d->latent_dim <= 0 || d->mlp_dim <= 0 || d->mlp_dim % 64) return false;
    w->A = d->action_dim; w->L = d->latent_dim; w->M = d->mlp_dim; w->E = d->enc_dim;
    w->Ap = (int)rup(w->A, 8); w->Lp = (int)rup(w->L, 8); w->Kx = w->Ap + w->Lp;
    w->Ar = (int)rup(w->A, 64); w->Lr = (int)rup(w->L, 64);
    w->modality = d->modality; w->obs_dim = d->obs_dim;
    w->img_c = d->img_c; w->img_hw = d->img_hw; w->nch = d->num_channels;
    size_t o = 0;
    auto take = [&](size_t n) { size_t r = o; o += rup(n, 64); return r; };
    if (d->modality == 0) {
        if (d->obs_dim <= 0 || d->enc_dim <= 0) return false;
        w->enc_w1 = take((size_t)w->E * d->obs_dim); w->enc_b1 = take(w->E);
        w->enc_w2 = take((size_t)w->L * w->E); w->enc_b2 = take(w->L);
        w->flat = 0;
    } else {
        if (d->img_c <= 0 || d->img_hw <= 0 || d->num_channels <= 0) return false;
        static const int ks[4] = {7, 5, 3, 3};
        int s = d->img_hw, cin = d->img_c;
        w->conv_hw[0] = s;
        for (int i = 0; i < 4; ++i) {
            w->cw[i] = take((size_t)w->nch * cin * ks[i] * ks[i]);
            w->cb[i] = take(w->nch);
            s = (s - ks[i]) / 2 + 1; cin = w->nch;
            w->conv_hw[i + 1] = s;
            if (s <= 0) return false;
        }
        w->flat = w->nch * s * s;
        w->pl_w = take((size_t)w->L * w->flat); w->pl_b = take(w->L);
    }
    const size_t M = w->M;
    w->w1x = take(2 * M * w->Kx); w->b1x = take(2 * M);
    w->w2d = take(M * M); w->b2d = take(M); w->w2r = take(M * M); w->b2r = take(M);
    w->w3d = take((size_t)w->Lr * M); w->b3d = take(w->Lr); w->w3r = take(M); w->b3r = take(1);
    w->wp1 = take(M * w->Lp); w->bp1 = take(M); w->wp2 = take(M * M); w->bp2 = take(M);
    w->wp3 = take((size_t)w->Ar * M); w->bp3 = take(w->Ar);
    w->wq1x = take(2 * M * w->Kx); w->bq1x = take(2 * M); w->g1 = take(2 * M); w->be1 = take(2 * M);
    w->wq2 = take(2 * M * M); w->bq2 = take(2 * M); w->g2 = take(2 * M); w->be2 = take(2 * M);
    w->wq3 = take(2 * M); w->bq3 = take(2);
    w->total = o;
    return true;
}

// ------------------------------------------------------------------------------------------------ workspace
struct Work {
    float* X;        // [(Hmax+1)][B*T][Kx] step inputs [a|z]; X_H is the terminal input
    float* H1;       // [B*T][2M]
    float* H2;       // [B*T][2M]
    float2* st1;     // [B*T][2M/64] LayerNorm partial moments of Q layer 0
    float2* st2;     // [B*T][2M/64] of Q layer 1
    float* rpart;    // [B*T][M/32] reward-head partial dots
    float* G;        // [B*T] discounted return so far (physical rows)
    float* rlast;    // [B*T] reward at t = H-1
    float* value;    // [B*T]
    float* z0;       // [B][Lp]
    float* mean;     // [B][Hmax][A]
    float* stdv;     // [B][Hmax][A]
    float* elite;    // [B][Hmax][K][A]
    float* score;    // [B][K]
    float* enc_tmp;  // pixel conv activations [B][max conv act]
    size_t x_stride; // floats per X_t
    size_t total;
};

size_t pixel_act_floats(const Layout& w) {
    size_t m = 0;
    for (int i = 1; i <= 4; ++i) m = std::max(m, (size_t)w.nch * w.conv_hw[i] * w.conv_hw[i]);
    return 2 * m;
}

bool make_work(const tdmpc_dims* d, const Layout& w, char* base, Work* k) {
    const size_t B = d->max_batch, N = d->num_samples, P = d->num_pi, T = N + P, H = d->max_horizon;
    const size_t M = w.M;
    size_t o = 0;
    auto take = [&](size_t bytes) { size_t r = o; o += rup(bytes, 256); return base ? base + r : nullptr; };
    k->x_stride = B * T * w.Kx;
    k->X = (float*)take((H + 1) * k->x_stride * 4);
    k->H1 = (float*)take(B * T * 2 * M * 4);
    k->H2 = (float*)take(B * T * 2 * M * 4);
    k->st1 = (float2*)take(B * T * (2 * M / 64) * 8);
    k->st2 = (float2*)take(B * T * (2 * M / 64) * 8);
    k->rpart = (float*)take(B * T * (M / 32) * 4);
    k->G = (float*)take(B * T * 4);
    k->rlast = (float*)take(B * T * 4);
    k->value = (float*)take(B * T * 4);
    k->z0 = (float*)take(B * w.Lp * 4);
    k->mean = (float*)take(B * H * w.A * 4);
    k->stdv = (float*)take(B * H * w.A * 4);
    k->elite = (float*)take(B * H * d->num_elites * w.A * 4);
    k->score = (float*)take(B * d->num_elites * 4);
    k->enc_tmp = (float*)take(d->modality ? B * pixel_act_floats(w) * 4 : 256);
    k->total = o;
    return true;
}

bool check_dims(const tdmpc_dims* d) {
    if (!d) return false;
    if (d->num_samples <= 0 || d->num_pi < 0 || d->num_elites <= 0 || d->max_horizon <= 0 ||
        d->max_horizon > 16 || d->max_iterations <= 0 || d->max_batch <= 0) return false;
    if (d->num_elites > d->num_samples + d->num_pi || d->num_elites > 1024) return false;
    if (d->num_samples + d->num_pi > 8192) return false;
    Layout w;
    if (!make_layout(d, &w)) return false;
    if (w.Kx > 1024 || w.M > 1024 || w.L > 1024) return false;
    // cem_kernel LDS: values[T] + elite actions [H][K][A] + misc
    size_t lds = (size_t)(d->num_samples + d->num_pi) * 4 + (size_t)d->max_horizon * d->num_elites * w.A * 4 +
                 (size_t)d->num_elites * 12 + (size_t)2 * d->max_horizon * w.A * 4 + 256;
    if (lds > 160 * 1024) return false;
    return true;
}

// ------------------------------------------------------------------------------------------------ device math
DEVI float elu1(float x) { return x > 0.f ? x : expm1f(x); }
DEVI float fmul(float a, float b) { return __fmul_rn(a, b); }
DEVI float fadd(float a, float b) { return __fadd_rn(a, b); }
DEVI float clampf(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }
// torch.clamp propagates NaN; fminf/fmaxf would drop it.
DEVI float tclamp(float x, float lo, float hi) { return x != x ? x : clampf(x, lo, hi); }
DEVI float nan_to_num(float x) {
    if (x != x) return 0.f;
    if (isinf(x)) return x > 0 ? 3.402823466e38f : -3.402823466e38f;
    return x;
}

struct RowMap {  // logical row m -> physical row (m / G) * S + O + m % G
    int G, S, O;
};
DEVI int map_row(const RowMap& r, int m) { return (m / r.G) * r.S + r.O + (m % r.G); }

// ------------------------------------------------------------------------------------------------ linear
enum { PRO_PLAIN = 0, PRO_LN_TANH = 1 };
enum { EPI_ELU = 0, EPI_LIN_Z = 1, EPI_PI = 2, EPI_LNSTATS = 3, EPI_ELU_DOT = 4, EPI_LIN = 5 };

struct LinProb {
    const float* A; int lda;      // activations (A + col offset), row stride in floats
    const float* W; int ldw;      // weights [Npad][K] row-major (nn.Linear layout)
    const float* bias;            // [Npad]
    float* C; int ldc;            // output (EPI-dependent)
    int N;                        // valid output columns
    int epi;
    const float2* ln_stats; int ln_ld; int ln_t0; int ln_nt;   // PRO_LN_*: moments [row][ln_ld] tiles
    const float* ln_g; const float* ln_b;                      // LN affine for this problem's K columns
    float2* st_out; int st_ld;                                 // EPI_LNSTATS
    const float* dotw; float* dot_out; int dot_ld;             // EPI_ELU_DOT
};

struct LinArgs {
    LinProb p[2];
    int M, K, kch;
    int a_mapped, c_mapped;
    RowMap amap, cmap;
    // EPI_LIN_Z (dynamics head of step t): reward bookkeeping
    const float* rpart; int rpart_nt; const float* b3r;
    float* G; float* rlast; float disc; int first, last;
    // EPI_PI
    const float* eps; int eps_G; long eps_env; long eps_off; int A; float min_std; float lo, hi;
};

template <int WN, int PRO, int KCH>
__global__ void __launch_bounds__(512) linear_kernel(const LinArgs args) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int BN = 32 * WN;
    constexpr int LDW = BN + 4;
    const LinProb& P = args.p[blockIdx.z];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nthr = blockDim.x;
    const int r = lane & 31, h = lane >> 5;
    const int m0 = blockIdx.x * 32, n0 = blockIdx.y * BN;
    if (n0 >= P.N) return;  // whole workgroup uniform
    const int m = m0 + r;
    const bool mval = m < args.M;
    const int mm = mval ? m : 0;
    const int arow = args.a_mapped ? map_row(args.amap, mm) : mm;
    const float* Arow = P.A + (size_t)arow * P.lda;

    float mu = 0.f, rs = 1.f;
    if (PRO == PRO_LN_TANH) {
        // Chan-combine the producer's per-64-column (mean, M2) into this row's mean / 1/sqrt(var+eps).
        const float2* st = P.ln_stats + (size_t)mm * P.ln_ld + P.ln_t0;
        float n = 0.f, mean = 0.f, m2 = 0.f;
        for (int i = 0; i < P.ln_nt; ++i) {
            float2 s = st[i];
            float nb = 64.f, nn = n + nb, delta = s.x - mean;
            mean += delta * nb / nn;
            m2 += s.y + delta * delta * n * nb / nn;
            n = nn;
        }
        mu = mean;
        rs = 1.0f / sqrtf(fmaxf(m2 / n, 0.f) + 1e-5f);
    }

    floatx16 acc[WN];
#pragma unroll
    for (int j = 0; j < WN; ++j)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[j][i] = 0.f;

    const int kbeg = wave * args.kch;
    const int kend = min(kbeg + args.kch, args.K);
    const float* Wrow[WN];
#pragma unroll
    for (int j = 0; j < WN; ++j) Wrow[j] = P.W + (size_t)(n0 + 32 * j + r) * P.ldw;

    constexpr int NG = KCH / 8;
    float4 av[NG], bv[NG][WN];
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        const int k = kbeg + 8 * g + 4 * h;
        if (kbeg + 8 * g < kend) {
            av[g] = *(const float4*)(Arow + k);
#pragma unroll
            for (int j = 0; j < WN; ++j) bv[g][j] = *(const float4*)(Wrow[j] + k);
        }
    }
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        if (kbeg + 8 * g < kend) {
            float4 a = av[g];
            if (PRO == PRO_LN_TANH) {
                const int k = kbeg + 8 * g + 4 * h;
                const float4 gg = *(const float4*)(P.ln_g + k);
                const float4 bb = *(const float4*)(P.ln_b + k);
                const float sh = -rs * mu;
                a.x = tanhf(fadd(fmul(fadd(fmul(a.x, rs), sh), gg.x), bb.x));
                a.y = tanhf(fadd(fmul(fadd(fmul(a.y, rs), sh), gg.y), bb.y));
                a.z = tanhf(fadd(fmul(fadd(fmul(a.z, rs), sh), gg.z), bb.z));
                a.w = tanhf(fadd(fmul(fadd(fmul(a.w, rs), sh), gg.w), bb.w));
            }
#pragma unroll
            for (int j = 0; j < WN; ++j) {
                acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, bv[g][j].x, acc[j], 0, 0, 0);
                acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, bv[g][j].y, acc[j], 0, 0, 0);
                acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, bv[g][j].z, acc[j], 0, 0, 0);
                acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, bv[g][j].w, acc[j], 0, 0, 0);
            }
        }
    }

    // partial tile -> LDS [wave][32][LDW]; C/D map: col = lane&31, row = (i&3) + 8*(i>>2) + 4*(lane>>5)
    float* mys = smem + (size_t)wave * 32 * LDW;
#pragma unroll
    for (int j = 0; j < WN; ++j)
#pragma unroll
        for (int i = 0; i < 16; ++i) mys[((i & 3) + 8 * (i >> 2) + 4 * h) * LDW + 32 * j + r] = acc[j][i];
    __syncthreads();

    // ---- epilogue: TPR threads per row, each owns 4-column chunks
    const int nw = nthr >> 6;
    // threads per row: a power of two (<= 16) so a row's threads are consecutive lanes of one wave and
    // the xor-shuffle row reductions are exact; surplus threads sit out the epilogue.
    const int tpr = nthr >= 512 ? 16 : nthr >= 256 ? 8 : nthr >= 128 ? 4 : 2;
    if (threadIdx.x >= 32 * tpr) return;
    const int row = threadIdx.x / tpr, q = threadIdx.x % tpr;
    const int lm = m0 + row;
    const bool rval = lm < args.M;
    const int crow = rval ? (args.c_mapped ? map_row(args.cmap, lm) : lm) : 0;
    const int epi = P.epi;
    float tsum = 0.f, dsum = 0.f;
    float* fin = smem;  // reduced tile is written back over wave 0's partial (each chunk has one owner)
    for (int c = 4 * q; c < BN; c += 4 * tpr) {
        float4 v = *(const float4*)(smem + row * LDW + c);
        for (int w = 1; w < nw; ++w) {
            const float4 u = *(const float4*)(smem + (size_t)w * 32 * LDW + row * LDW + c);
            v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
        }
        const int n = n0 + c;
        const float4 bb = *(const float4*)(P.bias + n);
        float o[4] = {v.x + bb.x, v.y + bb.y, v.z + bb.z, v.w + bb.w};
        if (epi == EPI_ELU || epi == EPI_ELU_DOT) {
#pragma unroll
            for (int i = 0; i < 4; ++i) o[i] = elu1(o[i]);
        }
        if (epi == EPI_ELU_DOT) {
            const float4 dw = *(const float4*)(P.dotw + n);
            dsum += o[0] * dw.x + o[1] * dw.y + o[2] * dw.z + o[3] * dw.w;
            continue;
        }
        if (epi == EPI_PI) {
            // TOLD.pi + TruncatedNormal.sample(clip=0.3) (tdmpc.py:39-45, helper.py:86-96)
            const int e = lm / args.eps_G, rr = lm % args.eps_G;
            const float* ep = args.eps + (size_t)e * args.eps_env + args.eps_off + (size_t)rr * args.A;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                if (n + i < P.N && rval) {
                    const float muv = tanhf(o[i]);
                    float x = muv;
                    if (args.min_std > 0.f) {
                        const float ee = tclamp(fmul(ep[n + i], args.min_std), -0.3f, 0.3f);
                        x = tclamp(fadd(muv, ee), args.lo, args.hi);
                    }
                    P.C[(size_t)crow * P.ldc + n + i] = x;
                }
            }
            continue;
        }
        if (epi == EPI_LNSTATS) {
            tsum += (o[0] + o[1]) + (o[2] + o[3]);
            *(float4*)(fin + row * LDW + c) = make_float4(o[0], o[1], o[2], o[3]);
        }
        if (rval) {
            float* dst = P.C + (size_t)crow * P.ldc + n;
            if (n + 3 < P.N && epi != EPI_LIN_Z) {
                *(float4*)dst = make_float4(o[0], o[1], o[2], o[3]);
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if (n + i < P.N) dst[i] = o[i];
            }
        }
    }
    if (epi == EPI_LNSTATS) {
        // LayerNorm partial moments of this 64-column slice: (mean, sum of squared deviations)
        for (int off = 1; off < tpr; off <<= 1) tsum += __shfl_xor(tsum, off, 64);
        const float tmean = tsum / (float)BN;
        float m2 = 0.f;
        for (int c = 4 * q; c < BN; c += 4 * tpr) {
            const float4 v = *(const float4*)(fin + row * LDW + c);
            const float d0 = v.x - tmean, d1 = v.y - tmean, d2 = v.z - tmean, d3 = v.w - tmean;
            m2 += (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3);
        }
        for (int off = 1; off < tpr; off <<= 1) m2 += __shfl_xor(m2, off, 64);
        if (q == 0 && rval) P.st_out[(size_t)lm * P.st_ld + blockIdx.y] = make_float2(tmean, m2);
    } else if (epi == EPI_ELU_DOT) {
        for (int off = 1; off < tpr; off <<= 1) dsum += __shfl_xor(dsum, off, 64);
        if (q == 0 && rval) P.dot_out[(size_t)lm * P.dot_ld + blockIdx.y] = dsum;
    } else if (epi == EPI_LIN_Z && blockIdx.y == 0 && q == 0 && rval) {
        // reward head (helper.mlp last Linear, M -> 1) from the partial dots, then
        // G += discount * reward (tdmpc.py:89) with float32(discount) like ATen's scalar mul.
        const float* rp = args.rpart + (size_t)lm * args.rpart_nt;
        float s = 0.f;
        for (int i = 0; i < args.rpart_nt; ++i) s += rp[i];
        const float rew = s + args.b3r[0];
        const float dr = fmul(args.disc, rew);
        args.G[crow] = args.first ? dr : fadd(args.G[crow], dr);
        if (args.last) args.rlast[crow] = rew;
    }
}

// ------------------------------------------------------------------------------------------------ value
// q_p = w3_p . ELU(LN_p(y_p)) + b3_p (helper.q last layers), G += gamma^H min(q1, q2), nan_to_num
// (tdmpc.py:91-92). One wave per row.
struct ValueArgs {
    const float* Y; int ldy; const float2* st; int st_ld; int M_;
    const float* g2; const float* be2; const float* w3; const float* b3;
    const float* G; float disc; float* value; float* value_out; int rows, T, I, iter;
};

__global__ void __launch_bounds__(256) value_kernel(const ValueArgs a) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= a.rows) return;
    const int ntile = a.M_ / 64;
    float q[2];
    for (int p = 0; p < 2; ++p) {
        const float2* st = a.st + (size_t)row * a.st_ld + p * ntile;
        float n = 0.f, mean = 0.f, m2 = 0.f;
        for (int i = 0; i < ntile; ++i) {
            float2 s = st[i];
            float nb = 64.f, nn = n + nb, delta = s.x - mean;
            mean += delta * nb / nn;
            m2 += s.y + delta * delta * n * nb / nn;
            n = nn;
        }
        const float rs = 1.0f / sqrtf(fmaxf(m2 / n, 0.f) + 1e-5f);
        const float sh = -rs * mean;
        const float* y = a.Y + (size_t)row * a.ldy + p * a.M_;
        const float* g = a.g2 + p * a.M_;
        const float* b = a.be2 + p * a.M_;
        const float* w = a.w3 + p * a.M_;
        float s = 0.f;
        for (int c = 4 * lane; c < a.M_; c += 256) {
            const float4 yv = *(const float4*)(y + c), gv = *(const float4*)(g + c), bv = *(const float4*)(b + c),
                         wv = *(const float4*)(w + c);
            s += elu1(fadd(fmul(fadd(fmul(yv.x, rs), sh), gv.x), bv.x)) * wv.x;
            s += elu1(fadd(fmul(fadd(fmul(yv.y, rs), sh), gv.y), bv.y)) * wv.y;
            s += elu1(fadd(fmul(fadd(fmul(yv.z, rs), sh), gv.z), bv.z)) * wv.z;
            s += elu1(fadd(fmul(fadd(fmul(yv.w, rs), sh), gv.w), bv.w)) * wv.w;
        }
        for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
        q[p] = s + a.b3[p];
    }
    if (lane == 0) {
        const float qm = fminf(q[0], q[1]);
        const float qmin = (q[0] != q[0] || q[1] != q[1]) ? NAN : qm;  // torch.min propagates NaN
        const float v = nan_to_num(fadd(a.G[row], fmul(a.disc, qmin)));
        a.value[row] = v;
        if (a.value_out) a.value_out[((size_t)(row / a.T) * a.I + a.iter) * a.T + row % a.T] = v;
    }
}

// ------------------------------------------------------------------------------------------------ CEM
// One workgroup per environment. mode 0: initialise mean/std (tdmpc.py:122-125) and sample iteration 0;
// mode 1: refit (tdmpc.py:138-149) and sample the next iteration (tdmpc.py:130-132);
// mode 2: refit and pick the output action (tdmpc.py:152-160).
struct CemArgs {
    int mode, iter, H, N, P, T, A, K, Kx;
    float* X; size_t x_stride;          // X_t a-columns hold the candidate actions
    const float* value;                 // [B*T]
    const float* rlast;                 // [B*T]
    float* mean; float* stdv;           // [B][Hmax][A]
    int Hmax;
    const float* eps; long eps_env; long eps_cem_off; long eps_iter; long eps_act_off;
    const double* u;
    float* prev_mean; int warm, eval_mode;
    float temperature, momentum, omm, std_floor;
    float* action; float* metrics;
    float* elite_ws; float* score_ws;
    float* elite_out; float* score_out; float* mean_out; float* std_out; int I;
};

__global__ void __launch_bounds__(1024) cem_kernel(const CemArgs a) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int e = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
    const int H = a.H, A = a.A, K = a.K, T = a.T, N = a.N;
    const int HA = H * A;
    float* vals = sm;                         // [T]
    float* EA = vals + rup(T, 4);             // [H][K][A]
    float* sc = EA + (size_t)H * K * A;       // [K]
    float* smean = sc + rup(K, 4);            // [HA]
    float* sstd = smean + rup(HA, 4);         // [HA]
    int* eidx = (int*)(sstd + rup(HA, 4));    // [K]
    float* red = (float*)(eidx + rup(K, 4));  // [4]
    int* jsel_p = (int*)(red + 2);
    float* gmean = a.mean + (size_t)e * a.Hmax * A;
    float* gstd = a.stdv + (size_t)e * a.Hmax * A;

    if (a.mode == 0) {
        for (int i = tid; i < HA; i += nt) {
            const int t = i / A, c = i % A;
            float mv = 0.f;
            if (a.warm && t < H - 1) mv = a.prev_mean[(size_t)e * H * A + (t + 1) * A + c];
            smean[i] = mv; sstd[i] = 2.f;
            gmean[i] = mv; gstd[i] = 2.f;
        }
    } else {
        for (int i = tid; i < T; i += nt) vals[i] = a.value[(size_t)e * T + i];
        __syncthreads();
        // top-k by rank: rank_i = #{v_j > v_i} + #{j < i : v_j == v_i}; sorted descending like torch.topk.
        for (int i = tid; i < T; i += nt) {
            const float vi = vals[i];
            int rank = 0;
            for (int j = 0; j < T; ++j) {
                const float vj = vals[j];
                rank += (vj > vi) || (vj == vi && j < i);
            }
            if (rank < K) eidx[rank] = i;
        }
        __syncthreads();
        for (int i = tid; i < H * K * A; i += nt) {
            const int t = i / (K * A), k = (i / A) % K, c = i % A;
            EA[i] = a.X[(size_t)t * a.x_stride + ((size_t)e * T + eidx[k]) * a.Kx + c];
        }
        if (tid < K) {
            const float ev = vals[eidx[tid]], vmax = vals[eidx[0]];
            sc[tid] = expf(fmul(a.temperature, ev - vmax));
        }
        __syncthreads();
        if (tid == 0) {
            float s = 0.f;
            for (int k = 0; k < K; ++k) s += sc[k];
            red[0] = s;
        }
        __syncthreads();
        if (tid < K) sc[tid] = __fdiv_rn(sc[tid], red[0]);
        __syncthreads();
        if (tid == 0) {
            float s = 0.f;
            for (int k = 0; k < K; ++k) s += sc[k];
            red[1] = fadd(s, 1e-9f);
        }
        __syncthreads();
        const float den = red[1];
        for (int i = tid; i < HA; i += nt) {
            const int t = i / A, c = i % A;
            const float* ea = EA + (size_t)t * K * A + c;
            float s = 0.f;
            for (int k = 0; k < K; ++k) s = fadd(s, fmul(sc[k], ea[(size_t)k * A]));
            const float mu = __fdiv_rn(s, den);
            float v = 0.f;
            for (int k = 0; k < K; ++k) {
                const float dd = ea[(size_t)k * A] - mu;
                v = fadd(v, fmul(sc[k], fmul(dd, dd)));
            }
            float sd = sqrtf(__fdiv_rn(v, den));
            sd = tclamp(sd, a.std_floor, 2.f);
            const float nm = fadd(fmul(a.momentum, gmean[i]), fmul(a.omm, mu));
            smean[i] = nm; sstd[i] = sd;
            gmean[i] = nm; gstd[i] = sd;
            if (a.mean_out) a.mean_out[((size_t)e * a.I + a.iter) * HA + i] = nm;
            if (a.std_out) a.std_out[((size_t)e * a.I + a.iter) * HA + i] = sd;
        }
        if (a.mode == 2) {
            for (int i = tid; i < H * K * A; i += nt) {
                a.elite_ws[(size_t)e * H * K * A + i] = EA[i];
                if (a.elite_out) a.elite_out[(size_t)e * H * K * A + i] = EA[i];
            }
            if (tid < K) {
                a.score_ws[(size_t)e * K + tid] = sc[tid];
                if (a.score_out) a.score_out[(size_t)e * K + tid] = sc[tid];
            }
        }
    }
    __syncthreads();

    if (a.mode != 2) {
        // actions = clamp(mean + std * randn(H,N,A), -1, 1) for the next iteration's rollout rows
        const int it = a.mode == 0 ? 0 : a.iter + 1;
        const float* ep = a.eps + (size_t)e * a.eps_env + a.eps_cem_off + (size_t)it * a.eps_iter;
        const int total = H * N * A;
        for (int i = tid; i < total; i += nt) {
            const int t = i / (N * A), n = (i / A) % N, c = i % A;
            const int hc = t * A + c;
            const float v = tclamp(fadd(smean[hc], fmul(sstd[hc], ep[i])), -1.f, 1.f);
            a.X[(size_t)t * a.x_stride + ((size_t)e * T + n) * a.Kx + c] = v;
        }
        return;
    }
    // final pick: j = np.random.choice(K, p=score) -> cdf in float64 (numpy legacy), searchsorted right
    if (tid == 0) {
        double last = 0.0;
        for (int k = 0; k < K; ++k) last += (double)sc[k];
        const double u = a.u[e];
        double acc = 0.0;
        int j = K - 1;
        for (int k = 0; k < K; ++k) {
            acc += (double)sc[k];
            if (acc / last > u) { j = k; break; }
        }
        *jsel_p = j;
        float rs = 0.f;
        for (int i = 0; i < T; ++i) rs += a.rlast[(size_t)e * T + i];
        float cs = 0.f;
        for (int c = 0; c < A; ++c) cs += sstd[c];
        a.metrics[(size_t)e * 2 + 0] = rs / (float)T;
        a.metrics[(size_t)e * 2 + 1] = cs / (float)A;
    }
    __syncthreads();
    const int j = *jsel_p;
    for (int c = tid; c < A; c += nt) {
        float v = EA[(size_t)j * A + c];
        if (!a.eval_mode) v = fadd(v, fmul(sstd[c], a.eps[(size_t)e * a.eps_env + a.eps_act_off + c]));
        a.action[(size_t)e * A + c] = v;
    }
    for (int i = tid; i < HA; i += nt) a.prev_mean[(size_t)e * H * A + i] = smean[i];
}

// ------------------------------------------------------------------------------------------------ encoder
// helper.enc, state modality: Linear(obs->E) ELU Linear(E->L) (helper.py:130-132). One wave per output
// neuron; the workgroup then broadcasts z0 into X_0's latent columns for its slice of the env's T rows.
struct EncArgs {
    const float* obs; long obs_stride; int obs_dim, E, L, Lp, Kx, Ap, T, rows_per_blk;
    const float* w1; const float* b1; const float* w2; const float* b2;
    float* z0; float* X0;
};

__global__ void __launch_bounds__(256) encode_state_kernel(const EncArgs a) {
    extern __shared__ __attribute__((aligned(16))) float es[];
    const int e = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
    float* x = es;                      // [obs_dim] or [flat]
    float* hh = x + rup(a.obs_dim, 4);  // [E]
    float* z = hh + rup(a.E, 4);        // [L]
    const float* src = a.obs + (size_t)e * a.obs_stride;
    for (int i = tid; i < a.obs_dim; i += blockDim.x) x[i] = src[i];
    __syncthreads();
    if (a.w1) {
        for (int j = wave; j < a.E; j += nw) {
            const float* wr = a.w1 + (size_t)j * a.obs_dim;
            float s = 0.f;
            for (int k = lane; k < a.obs_dim; k += 64) s += wr[k] * x[k];
            for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
            if (lane == 0) hh[j] = elu1(s + a.b1[j]);
        }
        __syncthreads();
    } else {
        for (int i = tid; i < a.E; i += blockDim.x) hh[i] = x[i];  // pixel path: flat conv features
        __syncthreads();
    }
    for (int j = wave; j < a.L; j += nw) {
        const float* wr = a.w2 + (size_t)j * a.E;
        float s = 0.f;
        for (int k = lane; k < a.E; k += 64) s += wr[k] * hh[k];
        for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
        if (lane == 0) z[j] = s + a.b2[j];
    }
    __syncthreads();
    if (blockIdx.y == 0)
        for (int i = tid; i < a.L; i += blockDim.x) a.z0[(size_t)e * a.Lp + i] = z[i];
    const int r0 = blockIdx.y * a.rows_per_blk, r1 = min(r0 + a.rows_per_blk, a.T);
    for (int i = tid; i < (r1 - r0) * a.L; i += blockDim.x) {
        const int rr = r0 + i / a.L, c = i % a.L;
        a.X0[((size_t)e * a.T + rr) * a.Kx + a.Ap + c] = z[c];
    }
}

// Direct 2-D convolution, stride 2, no padding, ReLU; input optionally uint8 scaled by 1/255
// (NormalizeImg, helper.py:99-106, then nn.Conv2d + nn.ReLU, helper.py:123-127).
__global__ void __launch_bounds__(256) conv_relu_kernel(const void* in, int in_u8, long in_bstride, int cin,
                                                        int hin, float* out, long out_bstride, int cout,
                                                        int hout, int ks, const float* w, const float* b) {
    const int e = blockIdx.y;
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    const int total = cout * hout * hout;
    if (idx >= total) return;
    const int co = idx / (hout * hout), oy = (idx / hout) % hout, ox = idx % hout;
    float s = 0.f;
    const float* wr = w + (size_t)co * cin * ks * ks;
    for (int ci = 0; ci < cin; ++ci) {
        for (int ky = 0; ky < ks; ++ky) {
            const long base = (long)e * in_bstride + ((long)ci * hin + (2 * oy + ky)) * hin + 2 * ox;
            for (int kx = 0; kx < ks; ++kx) {
                float v;
                if (in_u8) v = __fdiv_rn((float)((const uint8_t*)in)[base + kx], 255.f);
                else v = ((const float*)in)[base + kx];
                s += wr[(ci * ks + ky) * ks + kx] * v;
            }
        }
    }
    out[(size_t)e * out_bstride + idx] = fmaxf(s + b[co], 0.f);
}

// Actions [B][H][T][A] -> X_t a-columns (tdmpc_estimate_value entry).
__global__ void scatter_actions_kernel(const float* act, float* X, size_t x_stride, int H, int T, int A, int Kx,
                                       int B) {
    const size_t total = (size_t)B * H * T * A;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const int c = i % A;
        const size_t r = (i / A) % T;
        const int t = (i / ((size_t)A * T)) % H;
        const size_t e = i / ((size_t)A * T * H);
        X[(size_t)t * x_stride + (e * T + r) * Kx + c] = act[i];
    }
}

__global__ void bcast_z_kernel(const float* z0, int L, float* X0, int Kx, int Ap, int T, int B) {
    const size_t total = (size_t)B * T * L;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const size_t r = i / L;
        X0[r * Kx + Ap + i % L] = z0[(r / T) * L + i % L];
    }
}

__global__ void gather_z_kernel(const float* X, int Kx, int Ap, int L, int rows, float* out) {
    const size_t total = (size_t)rows * L;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x)
        out[i] = X[(i / L) * Kx + Ap + i % L];
}

// ------------------------------------------------------------------------------------------------ host side
#define HIPCHK(x)                                                                          \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            snprintf(g_err, sizeof g_err, "%s:%d %s", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return TDMPC_E_HIP;                                                            \
        }                                                                                  \
    } while (0)

template <int WN, int PRO, int KCH>
int set_lds_attr() {
    HIPCHK(hipFuncSetAttribute((const void*)linear_kernel<WN, PRO, KCH>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    return 0;
}

int init_attrs() {
    static int done = 0;
    if (done) return 0;
    int rc = 0;
    rc |= set_lds_attr<1, 0, 32>(); rc |= set_lds_attr<1, 0, 64>(); rc |= set_lds_attr<1, 0, 128>();
    rc |= set_lds_attr<2, 0, 32>(); rc |= set_lds_attr<2, 0, 64>(); rc |= set_lds_attr<2, 0, 128>();
    rc |= set_lds_attr<1, 1, 32>(); rc |= set_lds_attr<1, 1, 64>(); rc |= set_lds_attr<1, 1, 128>();
    rc |= set_lds_attr<2, 1, 32>(); rc |= set_lds_attr<2, 1, 64>(); rc |= set_lds_attr<2, 1, 128>();
    HIPCHK(hipFuncSetAttribute((const void*)cem_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    if (rc) return TDMPC_E_HIP;
    done = 1;
    return 0;
}

// Diagnostic kernel timer (tdmpc_profile_*): when armed on this thread, every linear_kernel launch whose
// (WN, PRO, KCH) instance matches is bracketed by HIP events on its stream, and its algorithmic FLOPs
// (2*M*N*K per problem) are recorded. Used by bench.py for the live roofline of the dominant kernel.
struct Profiler {
    int armed = 0, wn = 0, pro = 0, kch = 0, n = 0, cap = 0, kdim = 0;
    hipEvent_t* ev = nullptr;
    double flops = 0.0;
};
thread_local Profiler g_prof;

template <int WN, int PRO, int KCH>
int launch_lin_t(const LinArgs& a, int nprob, int nmax, hipStream_t s) {
    const int nw = (a.K + KCH - 1) / KCH;
    LinArgs b = a;
    b.kch = KCH;
    dim3 grid((a.M + 31) / 32, (nmax + 32 * WN - 1) / (32 * WN), nprob);
    dim3 block(64 * nw);
    const size_t lds = (size_t)nw * 32 * (32 * WN + 4) * 4;
    Profiler& pf = g_prof;
    const bool prof = pf.armed && pf.wn == WN && pf.pro == PRO && pf.kch == KCH && pf.n + 2 <= pf.cap &&
                      (pf.kdim == 0 || (a.K == pf.kdim && nmax == pf.kdim));
    if (prof) HIPCHK(hipEventRecord(pf.ev[pf.n], s));
    hipLaunchKernelGGL((linear_kernel<WN, PRO, KCH>), grid, block, lds, s, b);
    HIPCHK(hipGetLastError());
    if (prof) {
        HIPCHK(hipEventRecord(pf.ev[pf.n + 1], s));
        pf.n += 2;
        for (int q = 0; q < nprob; ++q) pf.flops += 2.0 * a.M * std::min(a.p[q].N, nmax) * a.K;
    }
    return 0;
}

// Picks the per-wave K chunk so that a workgroup has at most 8 waves (16 for very wide K).
int launch_lin(const LinArgs& a, int nprob, int nmax, int wn, int pro, hipStream_t s) {
    if (a.M <= 0) return 0;
    int kch = 32;
    if ((a.K + 31) / 32 > 8) kch = 64;
    if ((a.K + 63) / 64 > 8) kch = 128;
    if ((a.K + kch - 1) / kch > 8 || a.K % 8) { snprintf(g_err, sizeof g_err, "bad K %d", a.K); return TDMPC_E_DIMS; }
#define DISPATCH(WN_, PRO_, KCH_) \
    if (wn == WN_ && pro == PRO_ && kch == KCH_) return launch_lin_t<WN_, PRO_, KCH_>(a, nprob, nmax, s);
    DISPATCH(1, 0, 32) DISPATCH(1, 0, 64) DISPATCH(1, 0, 128)
    DISPATCH(2, 0, 32) DISPATCH(2, 0, 64) DISPATCH(2, 0, 128)
    DISPATCH(1, 1, 32) DISPATCH(1, 1, 64) DISPATCH(1, 1, 128)
    DISPATCH(2, 1, 32) DISPATCH(2, 1, 64) DISPATCH(2, 1, 128)
#undef DISPATCH
    return TDMPC_E_DIMS;
}

LinProb prob0() { LinProb p; memset(&p, 0, sizeof p); return p; }
LinArgs args0() { LinArgs a; memset(&a, 0, sizeof a); a.amap = {1 << 30, 0, 0}; a.cmap = {1 << 30, 0, 0}; return a; }

// The planner's per-call context.
struct Ctx {
    const tdmpc_dims* d; Layout w; Work k; const float* pw; hipStream_t s;
    int B, N, P, T, H, A, M, Kx;
    long eps_env, eps_cem_off, eps_iter, eps_term_off, eps_act_off;
};

float* Xt(const Ctx& c, int t) { return c.k.X + (size_t)t * c.k.x_stride; }

// One TOLD.next step for `rows` logical rows mapped onto X rows (tdmpc.py:34-37 + the G update of :88-90).
int step_next(const Ctx& c, int t, int rows, RowMap map, float disc, int first, int last) {
    const Layout& w = c.w;
    const float* pw = c.pw;
    int rc;
    {   // h1 = ELU(W1[d;r] [a|z] + b)   (dynamics.0 and reward.0 fused: N = 2M)
        LinArgs a = args0();
        a.M = rows; a.K = c.Kx; a.a_mapped = 1; a.amap = map;
        LinProb& p = a.p[0];
        p.A = Xt(c, t); p.lda = c.Kx; p.W = pw + w.w1x; p.ldw = c.Kx; p.bias = pw + w.b1x;
        p.C = c.k.H1; p.ldc = 2 * c.M; p.N = 2 * c.M; p.epi = EPI_ELU;
        if ((rc = launch_lin(a, 1, 2 * c.M, 2, PRO_PLAIN, c.s))) return rc;
    }
    {   // h2_d = ELU(W2d h1_d + b); reward partial dots of ELU(W2r h1_r + b) with reward.4.weight
        LinArgs a = args0();
        a.M = rows; a.K = c.M;
        LinProb& p0 = a.p[0];
        p0.A = c.k.H1; p0.lda = 2 * c.M; p0.W = pw + w.w2d; p0.ldw = c.M; p0.bias = pw + w.b2d;
        p0.C = c.k.H2; p0.ldc = 2 * c.M; p0.N = c.M; p0.epi = EPI_ELU;
        LinProb& p1 = a.p[1];
        p1.A = c.k.H1 + c.M; p1.lda = 2 * c.M; p1.W = pw + w.w2r; p1.ldw = c.M; p1.bias = pw + w.b2r;
        p1.N = c.M; p1.epi = EPI_ELU_DOT; p1.dotw = pw + w.w3r; p1.dot_out = c.k.rpart; p1.dot_ld = c.M / 32;
        if ((rc = launch_lin(a, 2, c.M, 1, PRO_PLAIN, c.s))) return rc;
    }
    {   // z' = W3d h2_d + b -> X_{t+1} latent columns; reward = sum(partials) + b; G update
        LinArgs a = args0();
        a.M = rows; a.K = c.M; a.c_mapped = 1; a.cmap = map;
        LinProb& p = a.p[0];
        p.A = c.k.H2; p.lda = 2 * c.M; p.W = pw + w.w3d; p.ldw = c.M; p.bias = pw + w.b3d;
        p.C = Xt(c, t + 1) + w.Ap; p.ldc = c.Kx; p.N = w.L; p.epi = EPI_LIN_Z;
        a.rpart = c.k.rpart; a.rpart_nt = c.M / 32; a.b3r = pw + w.b3r;
        a.G = c.k.G; a.rlast = c.k.rlast; a.disc = disc; a.first = first; a.last = last;
        if ((rc = launch_lin(a, 1, w.L, 1, PRO_PLAIN, c.s))) return rc;
    }
    return 0;
}

// pi(z_t) with TruncatedNormal noise for `rows` rows of X_t -> X_t action columns (tdmpc.py:39-45).
int policy(const Ctx& c, int t, int rows, RowMap map, const float* eps, long eps_env, int eps_G, long eps_off,
           float min_std) {
    const Layout& w = c.w;
    const float* pw = c.pw;
    int rc;
    {
        LinArgs a = args0();
        a.M = rows; a.K = w.Lp; a.a_mapped = 1; a.amap = map;
        LinProb& p = a.p[0];
        p.A = Xt(c, t) + w.Ap; p.lda = c.Kx; p.W = pw + w.wp1; p.ldw = w.Lp; p.bias = pw + w.bp1;
        p.C = c.k.H1; p.ldc = 2 * c.M; p.N = c.M; p.epi = EPI_ELU;
        if ((rc = launch_lin(a, 1, c.M, 2, PRO_PLAIN, c.s))) return rc;
    }
    {
        LinArgs a = args0();
        a.M = rows; a.K = c.M;
        LinProb& p = a.p[0];
        p.A = c.k.H1; p.lda = 2 * c.M; p.W = pw + w.wp2; p.ldw = c.M; p.bias = pw + w.bp2;
        p.C = c.k.H2; p.ldc = 2 * c.M; p.N = c.M; p.epi = EPI_ELU;
        if ((rc = launch_lin(a, 1, c.M, 1, PRO_PLAIN, c.s))) return rc;
    }
    {
        LinArgs a = args0();
        a.M = rows; a.K = c.M; a.c_mapped = 1; a.cmap = map;
        LinProb& p = a.p[0];
        p.A = c.k.H2; p.lda = 2 * c.M; p.W = pw + w.wp3; p.ldw = c.M; p.bias = pw + w.bp3;
        p.C = Xt(c, t); p.ldc = c.Kx; p.N = w.A; p.epi = EPI_PI;
        a.eps = eps; a.eps_G = eps_G; a.eps_env = eps_env; a.eps_off = eps_off; a.A = w.A;
        a.min_std = min_std;
        a.lo = (float)(-1.0 + 1e-6); a.hi = (float)(1.0 - 1e-6);
        return launch_lin(a, 1, w.A, 1, PRO_PLAIN, c.s);
    }
}

// Terminal value: Q(z_H, pi(z_H)) for all T rows of every env (tdmpc.py:91-92).
int terminal_q(const Ctx& c, float discH, float* value_out, int I, int iter) {
    const Layout& w = c.w;
    const float* pw = c.pw;
    const int rows = c.B * c.T;
    int rc;
    {   // y1 = Wq1[Q1;Q2] [a|z] + b, with LayerNorm partial moments per 64 columns
        LinArgs a = args0();
        a.M = rows; a.K = c.Kx;
        LinProb& p = a.p[0];
        p.A = Xt(c, c.H); p.lda = c.Kx; p.W = pw + w.wq1x; p.ldw = c.Kx; p.bias = pw + w.bq1x;
        p.C = c.k.H1; p.ldc = 2 * c.M; p.N = 2 * c.M; p.epi = EPI_LNSTATS;
        p.st_out = c.k.st1; p.st_ld = 2 * c.M / 64;
        if ((rc = launch_lin(a, 1, 2 * c.M, 2, PRO_PLAIN, c.s))) return rc;
    }
    {   // y2_p = Wq2_p tanh(LN(y1_p)) + b, moments again
        LinArgs a = args0();
        a.M = rows; a.K = c.M;
        for (int q = 0; q < 2; ++q) {
            LinProb& p = a.p[q];
            p.A = c.k.H1 + q * c.M; p.lda = 2 * c.M; p.W = pw + w.wq2 + (size_t)q * c.M * c.M; p.ldw = c.M;
            p.bias = pw + w.bq2 + q * c.M; p.C = c.k.H2 + q * c.M; p.ldc = 2 * c.M; p.N = c.M;
            p.epi = EPI_LNSTATS; p.st_out = c.k.st2 + q * (c.M / 64); p.st_ld = 2 * c.M / 64;
            p.ln_stats = c.k.st1; p.ln_ld = 2 * c.M / 64; p.ln_t0 = q * (c.M / 64); p.ln_nt = c.M / 64;
            p.ln_g = pw + w.g1 + q * c.M; p.ln_b = pw + w.be1 + q * c.M;
        }
        if ((rc = launch_lin(a, 2, c.M, 2, PRO_LN_TANH, c.s))) return rc;
    }
    {
        ValueArgs v;
        v.Y = c.k.H2; v.ldy = 2 * c.M; v.st = c.k.st2; v.st_ld = 2 * c.M / 64; v.M_ = c.M;
        v.g2 = pw + w.g2; v.be2 = pw + w.be2; v.w3 = pw + w.wq3; v.b3 = pw + w.bq3;
        v.G = c.k.G; v.disc = discH; v.value = c.k.value; v.value_out = value_out; v.rows = rows;
        v.T = c.T; v.I = I; v.iter = iter;
        hipLaunchKernelGGL(value_kernel, dim3((rows + 3) / 4), dim3(256), 0, c.s, v);
        HIPCHK(hipGetLastError());
    }
    return 0;
}

int encode(const Ctx& c, const void* obs, int obs_is_u8, int batch, float* z0_out, int T, float* X0) {
    const Layout& w = c.w;
    const float* pw = c.pw;
    EncArgs a;
    memset(&a, 0, sizeof a);
    a.L = w.L; a.Lp = w.Lp; a.Kx = w.Kx; a.Ap = w.Ap; a.T = T;
    a.z0 = z0_out; a.X0 = X0;
    if (w.modality == 0) {
        a.obs = (const float*)obs; a.obs_dim = w.obs_dim; a.obs_stride = w.obs_dim; a.E = w.E;
        a.w1 = pw + w.enc_w1; a.b1 = pw + w.enc_b1; a.w2 = pw + w.enc_w2; a.b2 = pw + w.enc_b2;
    } else {
        static const int ks[4] = {7, 5, 3, 3};
        const size_t act = pixel_act_floats(w) / 2;
        float* bufs[2] = {c.k.enc_tmp, c.k.enc_tmp + (size_t)batch * act};
        const void* in = obs;
        int in_u8 = obs_is_u8;
        long in_bs = (long)w.img_c * w.img_hw * w.img_hw;
        int cin = w.img_c;
        for (int i = 0; i < 4; ++i) {
            const int ho = w.conv_hw[i + 1];
            const int total = w.nch * ho * ho;
            float* out = bufs[i & 1];
            hipLaunchKernelGGL(conv_relu_kernel, dim3((total + 255) / 256, batch), dim3(256), 0, c.s, in, in_u8,
                               in_bs, cin, w.conv_hw[i], out, (long)act, w.nch, ho, ks[i], pw + w.cw[i], pw + w.cb[i]);
            HIPCHK(hipGetLastError());
            in = out; in_u8 = 0; in_bs = (long)act; cin = w.nch;
        }
        a.obs = (const float*)in; a.obs_dim = w.flat; a.obs_stride = (long)act;
        a.E = w.flat; a.w1 = nullptr; a.w2 = pw + w.pl_w; a.b2 = pw + w.pl_b;
    }
    const int rpb = 64;
    a.rows_per_blk = rpb;
    const int chunks = X0 ? (T + rpb - 1) / rpb : 1;
    if (!X0) a.T = 0;
    const size_t lds = (rup(a.obs_dim, 4) + rup(a.E, 4) + rup(a.L, 4)) * 4;
    hipLaunchKernelGGL(encode_state_kernel, dim3(batch, chunks), dim3(256), lds, c.s, a);
    HIPCHK(hipGetLastError());
    return 0;
}

int setup_ctx(Ctx& c, const tdmpc_dims* d, const void* packed, void* ws, size_t ws_bytes, int batch, int H,
              int I, hipStream_t s) {
    if (!check_dims(d)) { snprintf(g_err, sizeof g_err, "bad dims"); return TDMPC_E_DIMS; }
    c.d = d;
    make_layout(d, &c.w);
    Work probe;
    make_work(d, c.w, nullptr, &probe);
    if (ws_bytes < probe.total) { snprintf(g_err, sizeof g_err, "workspace too small"); return TDMPC_E_SIZE; }
    make_work(d, c.w, (char*)ws, &c.k);
    c.pw = (const float*)packed; c.s = s;
    c.B = batch; c.N = d->num_samples; c.P = d->num_pi; c.T = c.N + c.P; c.H = H;
    c.A = c.w.A; c.M = c.w.M; c.Kx = c.w.Kx;
    const long A = c.A;
    c.eps_cem_off = (long)H * c.P * A;
    c.eps_iter = (long)H * c.N * A + (long)c.T * A;
    c.eps_term_off = (long)H * c.N * A;
    c.eps_act_off = c.eps_cem_off + (long)I * c.eps_iter;
    c.eps_env = c.eps_act_off + A;
    if (batch <= 0 || batch > d->max_batch || H <= 0 || H > d->max_horizon || I <= 0 || I > d->max_iterations) {
        snprintf(g_err, sizeof g_err, "bad call params");
        return TDMPC_E_DIMS;
    }
    return init_attrs();
}

}  // namespace

// ================================================================================================ C ABI
extern "C" {

int tdmpc_abi_version(void) { return TDMPC_ABI_VERSION; }

const char* tdmpc_last_error(void) { return g_err; }

int tdmpc_sizes_for(const tdmpc_dims* d, tdmpc_sizes* out) {
    if (!d || !out) return TDMPC_E_NULL;
    if (!check_dims(d)) return TDMPC_E_DIMS;
    Layout w;
    make_layout(d, &w);
    Work k;
    make_work(d, w, nullptr, &k);
    out->packed_weight_bytes = rup(w.total * 4, 256);
    out->workspace_bytes = k.total;
    out->noise_floats_per_env = tdmpc_noise_floats(d, d->max_horizon, d->max_iterations);
    return 0;
}

size_t tdmpc_noise_floats(const tdmpc_dims* d, int32_t H, int32_t I) {
    if (!d) return 0;
    const size_t A = d->action_dim, N = d->num_samples, P = d->num_pi, T = N + P;
    return (size_t)H * P * A + (size_t)I * ((size_t)H * N * A + T * A) + A;
}

int tdmpc_num_param_tensors(const tdmpc_dims* d) {
    if (!d) return TDMPC_E_NULL;
    return (d->modality ? 10 : 4) + 6 + 6 + 6 + 10 + 10;
}

int tdmpc_pack_weights(const tdmpc_dims* d, const float* const* t, int32_t n, void* packed, size_t bytes,
                       void* stream) {
    if (!d || !t || !packed) return TDMPC_E_NULL;
    if (!check_dims(d)) return TDMPC_E_DIMS;
    Layout w;
    make_layout(d, &w);
    if (n != tdmpc_num_param_tensors(d)) return TDMPC_E_DIMS;
    if (bytes < w.total * 4) return TDMPC_E_SIZE;
    if (init_attrs()) return TDMPC_E_HIP;
    hipStream_t s = (hipStream_t)stream;
    float* pw = (float*)packed;
    const size_t M = w.M, L = w.L, A = w.A, F = 4;
    HIPCHK(hipMemsetAsync(packed, 0, w.total * 4, s));
    auto cp = [&](size_t dst, const float* src, size_t nfl) {
        return hipMemcpyAsync(pw + dst, src, nfl * F, hipMemcpyDeviceToDevice, s);
    };
    // 2-D copy: rows x cols floats from src (row pitch spitch floats) to dst (pitch dpitch floats)
    auto cp2 = [&](size_t dst, size_t dpitch, const float* src, size_t spitch, size_t cols, size_t rows) {
        return hipMemcpy2DAsync(pw + dst, dpitch * F, src, spitch * F, cols * F, rows, hipMemcpyDeviceToDevice, s);
    };
    int i = 0;
    if (w.modality == 0) {
        HIPCHK(cp(w.enc_w1, t[i++], (size_t)w.E * w.obs_dim)); HIPCHK(cp(w.enc_b1, t[i++], w.E));
        HIPCHK(cp(w.enc_w2, t[i++], L * w.E)); HIPCHK(cp(w.enc_b2, t[i++], L));
    } else {
        static const int ks[4] = {7, 5, 3, 3};
        int cin = w.img_c;
        for (int c = 0; c < 4; ++c) {
            HIPCHK(cp(w.cw[c], t[i++], (size_t)w.nch * cin * ks[c] * ks[c]));
            HIPCHK(cp(w.cb[c], t[i++], w.nch));
            cin = w.nch;
        }
        HIPCHK(cp(w.pl_w, t[i++], L * w.flat)); HIPCHK(cp(w.pl_b, t[i++], L));
    }
    const size_t KI = L + A;  // reference input width of cat[z, a]
    // permuted first layer: dst [a | 0 | z | 0]  <-  src [z | a]
    auto cp_first = [&](size_t dst, const float* src) -> hipError_t {
        hipError_t e = cp2(dst, w.Kx, src + L, KI, A, M);
        if (e != hipSuccess) return e;
        return cp2(dst + w.Ap, w.Kx, src, KI, L, M);
    };
    // dynamics: 0.w 0.b 2.w 2.b 4.w 4.b
    HIPCHK(cp_first(w.w1x, t[i++])); HIPCHK(cp(w.b1x, t[i++], M));
    HIPCHK(cp(w.w2d, t[i++], M * M)); HIPCHK(cp(w.b2d, t[i++], M));
    HIPCHK(cp(w.w3d, t[i++], L * M)); HIPCHK(cp(w.b3d, t[i++], L));
    // reward
    HIPCHK(cp_first(w.w1x + M * w.Kx, t[i++])); HIPCHK(cp(w.b1x + M, t[i++], M));
    HIPCHK(cp(w.w2r, t[i++], M * M)); HIPCHK(cp(w.b2r, t[i++], M));
    HIPCHK(cp(w.w3r, t[i++], M)); HIPCHK(cp(w.b3r, t[i++], 1));
    // pi
    HIPCHK(cp2(w.wp1, w.Lp, t[i++], L, L, M)); HIPCHK(cp(w.bp1, t[i++], M));
    HIPCHK(cp(w.wp2, t[i++], M * M)); HIPCHK(cp(w.bp2, t[i++], M));
    HIPCHK(cp(w.wp3, t[i++], A * M)); HIPCHK(cp(w.bp3, t[i++], A));
    // Q1, Q2: 0.w 0.b 1.w 1.b 3.w 3.b 4.w 4.b 6.w 6.b
    for (int q = 0; q < 2; ++q) {
        HIPCHK(cp_first(w.wq1x + q * M * w.Kx, t[i++])); HIPCHK(cp(w.bq1x + q * M, t[i++], M));
        HIPCHK(cp(w.g1 + q * M, t[i++], M)); HIPCHK(cp(w.be1 + q * M, t[i++], M));
        HIPCHK(cp(w.wq2 + q * M * M, t[i++], M * M)); HIPCHK(cp(w.bq2 + q * M, t[i++], M));
        HIPCHK(cp(w.g2 + q * M, t[i++], M)); HIPCHK(cp(w.be2 + q * M, t[i++], M));
        HIPCHK(cp(w.wq3 + q * M, t[i++], M)); HIPCHK(cp(w.bq3 + q, t[i++], 1));
    }
    return 0;
}

int tdmpc_encode(const tdmpc_dims* d, const void* packed, const void* obs, int32_t obs_is_u8, int32_t batch,
                 void* workspace, float* z0, void* stream) {
    if (!d || !packed || !obs || !z0 || !workspace) return TDMPC_E_NULL;
    Ctx c;
    tdmpc_sizes sz;
    int rc = tdmpc_sizes_for(d, &sz);
    if (rc) return rc;
    if ((rc = setup_ctx(c, d, packed, workspace, sz.workspace_bytes, batch, 1, 1, (hipStream_t)stream))) return rc;
    // z0 written with row stride Lp inside encode; use a compact copy for the caller
    if ((rc = encode(c, obs, obs_is_u8, batch, c.k.z0, 0, nullptr))) return rc;
    HIPCHK(hipMemcpy2DAsync(z0, c.w.L * 4, c.k.z0, c.w.Lp * 4, c.w.L * 4, batch, hipMemcpyDeviceToDevice, c.s));
    return 0;
}

int tdmpc_plan(const tdmpc_dims* d, const tdmpc_plan_params* prm, const void* packed, const void* obs,
               int32_t obs_is_u8, const float* noise, const double* u, float* prev_mean, float* action,
               float* metrics, float* elite_out, float* score_out, float* value_out, float* mean_out,
               float* std_out, void* workspace, size_t ws_bytes, void* stream) {
    if (!d || !prm || !packed || !obs || !noise || !u || !prev_mean || !action || !metrics || !workspace)
        return TDMPC_E_NULL;
    Ctx c;
    int rc;
    const int H = prm->horizon, I = prm->iterations, B = prm->batch;
    if ((rc = setup_ctx(c, d, packed, workspace, ws_bytes, B, H, I, (hipStream_t)stream))) return rc;
    const int N = c.N, P = c.P, T = c.T;
    // X holds [a|0|z|0] rows; zero the padding once per call (kernels only write real columns)
    HIPCHK(hipMemsetAsync(c.k.X, 0, (size_t)(H + 1) * c.k.x_stride * 4, c.s));
    if ((rc = encode(c, obs, obs_is_u8, B, c.k.z0, T, Xt(c, 0)))) return rc;

    CemArgs ca;
    memset(&ca, 0, sizeof ca);
    ca.H = H; ca.N = N; ca.P = P; ca.T = T; ca.A = c.A; ca.K = d->num_elites; ca.Kx = c.Kx;
    ca.X = c.k.X; ca.x_stride = c.k.x_stride; ca.value = c.k.value; ca.rlast = c.k.rlast;
    ca.mean = c.k.mean; ca.stdv = c.k.stdv; ca.Hmax = d->max_horizon;
    ca.eps = noise; ca.eps_env = c.eps_env; ca.eps_cem_off = c.eps_cem_off; ca.eps_iter = c.eps_iter;
    ca.eps_act_off = c.eps_act_off; ca.u = u; ca.prev_mean = prev_mean; ca.warm = prm->warm_start;
    ca.eval_mode = prm->eval_mode; ca.temperature = prm->temperature; ca.momentum = prm->momentum;
    ca.omm = prm->one_minus_momentum; ca.std_floor = prm->std_floor; ca.action = action; ca.metrics = metrics;
    ca.elite_ws = c.k.elite; ca.score_ws = c.k.score; ca.elite_out = elite_out; ca.score_out = score_out;
    ca.mean_out = mean_out; ca.std_out = std_out; ca.I = I;
    const size_t cem_lds = (rup(T, 4) + (size_t)H * ca.K * c.A + 2 * rup(ca.K, 4) + 2 * rup(H * c.A, 4) + 4) * 4;
    const int cem_thr = 1024;

    ca.mode = 0;
    hipLaunchKernelGGL(cem_kernel, dim3(B), dim3(cem_thr), cem_lds, c.s, ca);
    HIPCHK(hipGetLastError());

    // pi pre-rollout on the P policy rows of every env (tdmpc.py:113-118); their H-step rollout, reward
    // prefix and z_H are identical in every CEM iteration (same z0, same pi_actions), so they are computed
    // once here and reused (rows N..T-1 of X_t, G and rlast).
    if (P > 0) {
        const RowMap pm = {P, T, N};
        for (int t = 0; t < H; ++t) {
            // pi(z_t) -> X_t action cols of pi rows, eps_pi[t]
            if ((rc = policy(c, t, B * P, pm, noise, c.eps_env, P, (long)t * P * c.A, prm->min_std))) return rc;
            if ((rc = step_next(c, t, B * P, pm, prm->discount_pow[t], t == 0, t == H - 1))) return rc;
        }
    }
    const RowMap rm = {N, T, 0};
    const RowMap all = {T, T, 0};
    for (int i = 0; i < I; ++i) {
        for (int t = 0; t < H; ++t)
            if ((rc = step_next(c, t, B * N, rm, prm->discount_pow[t], t == 0, t == H - 1))) return rc;
        if ((rc = policy(c, H, B * T, all, noise, c.eps_env, T, c.eps_cem_off + (long)i * c.eps_iter + c.eps_term_off,
                         prm->min_std)))
            return rc;
        if ((rc = terminal_q(c, prm->discount_pow[H], value_out, I, i))) return rc;
        ca.mode = (i == I - 1) ? 2 : 1;
        ca.iter = i;
        hipLaunchKernelGGL(cem_kernel, dim3(B), dim3(cem_thr), cem_lds, c.s, ca);
        HIPCHK(hipGetLastError());
    }
    return 0;
}

int tdmpc_estimate_value(const tdmpc_dims* d, const tdmpc_plan_params* prm, const void* packed, const float* z0,
                         const float* actions, const float* eps_term, int32_t rows, float* value, float* reward_last,
                         float* z_last, void* workspace, size_t ws_bytes, void* stream) {
    if (!d || !prm || !packed || !z0 || !actions || !eps_term || !value || !reward_last || !workspace)
        return TDMPC_E_NULL;
    Ctx c;
    int rc;
    const int H = prm->horizon, B = prm->batch;
    if ((rc = setup_ctx(c, d, packed, workspace, ws_bytes, B, H, 1, (hipStream_t)stream))) return rc;
    if (rows != c.T) { snprintf(g_err, sizeof g_err, "rows must equal N+P"); return TDMPC_E_DIMS; }
    const int T = c.T, L = c.w.L;
    HIPCHK(hipMemsetAsync(c.k.X, 0, (size_t)(H + 1) * c.k.x_stride * 4, c.s));
    hipLaunchKernelGGL(bcast_z_kernel, dim3(256), dim3(256), 0, c.s, z0, L, Xt(c, 0), c.Kx, c.w.Ap, T, B);
    HIPCHK(hipGetLastError());
    hipLaunchKernelGGL(scatter_actions_kernel, dim3(512), dim3(256), 0, c.s, actions, c.k.X, c.k.x_stride, H, T,
                       c.A, c.Kx, B);
    HIPCHK(hipGetLastError());
    const RowMap all = {T, T, 0};
    for (int t = 0; t < H; ++t)
        if ((rc = step_next(c, t, B * T, all, prm->discount_pow[t], t == 0, t == H - 1))) return rc;
    if (z_last) {
        hipLaunchKernelGGL(gather_z_kernel, dim3(256), dim3(256), 0, c.s, Xt(c, H), c.Kx, c.w.Ap, L, B * T, z_last);
        HIPCHK(hipGetLastError());
    }
    if ((rc = policy(c, H, B * T, all, eps_term, (long)T * c.A, T, 0, prm->min_std))) return rc;
    if ((rc = terminal_q(c, prm->discount_pow[H], nullptr, 1, 0))) return rc;
    HIPCHK(hipMemcpyAsync(value, c.k.value, (size_t)B * T * 4, hipMemcpyDeviceToDevice, c.s));
    HIPCHK(hipMemcpyAsync(reward_last, c.k.rlast, (size_t)B * T * 4, hipMemcpyDeviceToDevice, c.s));
    return 0;
}

int tdmpc_profile_begin(int32_t wn, int32_t pro, int32_t kch, int32_t kdim, int32_t max_launches) {
    Profiler& pf = g_prof;
    if (pf.ev) {
        for (int i = 0; i < pf.cap; ++i) (void)hipEventDestroy(pf.ev[i]);
        free(pf.ev);
    }
    pf = Profiler();
    pf.cap = 2 * std::max(1, (int)max_launches);
    pf.ev = (hipEvent_t*)calloc(pf.cap, sizeof(hipEvent_t));
    for (int i = 0; i < pf.cap; ++i) HIPCHK(hipEventCreate(&pf.ev[i]));
    pf.wn = wn; pf.pro = pro; pf.kch = kch; pf.kdim = kdim; pf.armed = 1;
    return 0;
}

int tdmpc_profile_end(int32_t* launches, double* total_ms, double* flops) {
    Profiler& pf = g_prof;
    pf.armed = 0;
    double tot = 0.0;
    for (int i = 0; i + 1 < pf.n; i += 2) {
        HIPCHK(hipEventSynchronize(pf.ev[i + 1]));
        float ms = 0.f;
        HIPCHK(hipEventElapsedTime(&ms, pf.ev[i], pf.ev[i + 1]));
        tot += ms;
    }
    if (launches) *launches = pf.n / 2;
    if (total_ms) *total_ms = tot;
    if (flops) *flops = pf.flops;
    return 0;
}

}  // extern "C"
