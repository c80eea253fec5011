// tdmpc_kernels.hip -- MI355X (gfx950 / CDNA4) kernels for TD-MPC planning (TDMPC.plan + TOLD rollout).
//
// Reference behaviour: /root/reference/src/algorithm/tdmpc.py:83-163 (plan, estimate_value) and the TOLD
// heads tdmpc.py:30-50 built from helper.py:119-133 (enc), 169-176 (mlp), 197-201 (q), 71-96
// (TruncatedNormal). See DESIGN.md for the decomposition, data layout and rooflines.
//
// Data layout. Every matrix an MFMA reads (weights and activations) is stored in the "panel" layout
//   [rows/32][cols/4][32][4]   element (r, c) at (r>>5)*(cols*32) + (c>>2)*128 + (r&31)*4 + (c&3)
// so that the A or B operand of v_mfma_f32_32x32x2_f32 for one 8-deep k group is ONE contiguous 1 KiB
// wave load (lanes 0-31 read k-quad q of 32 rows, lanes 32-63 quad q+1). The k order inside an 8-group is
// permuted identically for A and B, which leaves the dot product unchanged.
//
// Kernel families
//   linear_kernel<WN,PRO,KCH>  one fused nn.Linear on f32 MFMA: a workgroup owns a 32-row x (32*WN)-col
//       output tile, its waves split K (KCH each) and reduce through LDS; fused epilogues: bias + ELU /
//       TruncatedNormal policy sample / LayerNorm partial moments / reward-head dot / discounted return.
//       Fused prologues: LayerNorm+tanh of A; CEM action sampling clamp(mean+std*eps) for the action
//       columns; broadcast of the encoder output z0 for the latent columns at t = 0.
//   value_kernel   Q heads' LayerNorm+ELU+Linear(M->1), min(Q1,Q2), G + gamma^H Q, nan_to_num.
//   cem_kernel     one workgroup per env: bitonic top-k, softmax, weighted mean/std refit, momentum, and
//                  on the last iteration the elite choice (np.random.choice cdf) and the output action.
//   encode_kernel / conv_relu_kernel   TOLD.h (state MLP or pixel conv stack) + CEM mean/std init.
#include <hip/hip_runtime.h>
#include <hiprand/hiprand_kernel.h>

#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <mutex>
#include <type_traits>
#include <vector>

#include "../../include/tdmpc_hip.h"

typedef float floatx16 __attribute__((ext_vector_type(16)));

#define DEVI __device__ __forceinline__

// Diagnostic build only (tools/mb, -DTDMPC_STAMPS): per-workgroup phase timestamps of linear_kernel.
#ifdef TDMPC_STAMPS
__device__ unsigned long long* g_stamps;   // null unless the diagnostic host sets it
__device__ unsigned int g_stamp_n;
__device__ unsigned int g_stamp_cap;
#define STAMP(slot)                                                                                   \
    do {                                                                                              \
        __builtin_amdgcn_sched_barrier(0);                                                            \
        unsigned long long t_;                                                                        \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");                     \
        __builtin_amdgcn_sched_barrier(0);                                                            \
        st_[slot] = t_;                                                                               \
    } while (0)
// Record of one workgroup: [realtime start, 5 phase stamps (shader clock), block ids, xcc | realtime span << 8]
#define STAMP_RECORD()                                                                                \
    do {                                                                                              \
        if (threadIdx.x == 0 && g_stamps) {                                                           \
            const unsigned long long rt1_ = __builtin_amdgcn_s_memrealtime();                         \
            const unsigned int slot = atomicAdd(&g_stamp_n, 1u);                                      \
            if (slot < g_stamp_cap) {                                                                 \
                unsigned long long* o = g_stamps + (size_t)slot * 8;                                  \
                o[0] = rt0_; o[1] = st_[0]; o[2] = st_[1]; o[3] = st_[2]; o[4] = st_[3]; o[5] = st_[4]; \
                o[6] = blockIdx.x | (blockIdx.y << 16) | ((unsigned long long)blockIdx.z << 32);      \
                unsigned int xcc_;                                                                    \
                asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc_));                   \
                o[7] = (xcc_ & 0xff) | ((rt1_ - rt0_) << 8);                                          \
            }                                                                                         \
        }                                                                                             \
    } while (0)
#else
#define STAMP(slot) do {} while (0)
#endif

namespace {

thread_local char g_err[512] = "";

__host__ __device__ inline size_t rup(size_t x, size_t a) { return (x + a - 1) / a * a; }

// ------------------------------------------------------------------------------------------------ layout
// Packed parameter buffer (float offsets, each tensor 64-float aligned). First-layer inputs are
// x = [a | 0 | z | 0] (action columns first, each part padded to a multiple of 8) so that every 8-deep
// k group is all-action or all-latent.
struct Layout {
    int A, L, M, E, Ap, Lp, Kx, Ar, Lr;
    int modality, obs_dim, img_c, img_hw, nch, conv_hw[5], flat;
    size_t enc_w1t, enc_b1, enc_w2t, enc_b2;         // state encoder, weights transposed [in][out]
    size_t enc_lng, enc_lnb; int enc_norm;           // its LayerNorm (enc_norm), [E] each
    size_t cw[4], cb[4], pl_wt, pl_b;                // pixel encoder (conv dense, linear transposed)
    size_t cwt[4];                                   // conv weights again as [ci][ky][kx][co] (conv_tile_kernel)
    size_t w1x, b1x;                                 // panel [2M][Kx]: dynamics.0 rows then reward.0 rows
    size_t w2d, b2d, w2r, b2r;                       // panel [M][M]
    size_t w3d, b3d, w3r, b3r;                       // panel [Lr][M]; reward.4 dense [M]
    size_t wp1, bp1, wp2, bp2, wp3, bp3;             // pi: panel [M][Lp], [M][M], [Ar][M]
    size_t wq1x, bq1x, g1, be1;                      // panel [2M][Kx]; LN1 gamma/beta [2M]
    size_t wq2, bq2, g2, be2;                        // 2 panels [M][M]; LN2 [2M]
    size_t wq3, bq3;                                 // [2][M], [2]
    // the chain kernels' weight panels again as three bf16 planes (x6 layout, X6_* below, pack_fused_kernel)
    size_t x6[9];
    // the wide step kernel's copies of X6_W1X .. X6_W3D in the x6q layout: block (nb, g) of 16 rows x 32 k is
    // [3 planes][64 lanes][8 bf16]: lane l (m = l & 15, q = l >> 4) element j holds row 16 nb + m,
    // k = 32 g + 16 (j >> 2) + 4 q + (j & 3) -- the v_mfma_f32_16x16x32_bf16 A fragment, in the k order in which a
    // 16x16 accumulator tile pair (a lane holding features 16t + 4q + i of its row) is the next layer's B fragment
    size_t x6q[9];   // (X6_N: every x6 matrix; the wide kernels read W1X .. W3D and WQ1X, WQ2)
    size_t jobtab;   // the fused pack's header (PackHdr: table nonce, sticky status) + job table (launch_pack):
                     // caller-owned, lives and dies with the packed buffer
    // helper.q's LayerNorm-1 statistics block (wide_heads.inc; written by qstat_*_kernel after every pack) for planners
    // whose batches reach the wide kernels: nqs = the first layer's real columns + its bias (A + L + 1), 0 = none
    int nqs, nsr;          // columns of the Cholesky factor; statistics rows per Q head (16 x 8 or 16 x 16)
    size_t x6qs, bqs;      // x6q [2][nsr][rup(Kx, 32)]; bias [2][nsr]
    size_t x6qf, bqf;      // the folded first layer diag(g1) (W1 - 1 wbar^T): x6q [2][M][rup(Kx, 32)]; g1 (b1 - bbar) [2][M]
    size_t qs_gram;        // fp64 scratch [2][nqs][nqs] (the Gram matrices)
    // the folded first layer of TOLD.next for latent_dim == mlp_dim (pack_fold; wide_step.inc WS_OUTH): both heads'
    // [W1a | W1z W3] in x6q [2M][rup(Kx, 32)] and b1 + W1z b3 [2M] -- the first layer of a step whose input latent
    // columns hold the previous step's h2 instead of z (fold = 0: none)
    int fold;
    size_t x6qw, bfw;
    size_t fold_w;         // fp32 scratch [2M][M]: W1z W3 (fp64 sums, rounded once)
    // ... and the terminal heads' first layers for the chain kernels (x6 layout), so the last step stores h2 too:
    // pi [Wp1 W3] (M x Lp) with bp1 + Wp1 b3, Q1|Q2 [Wq1a | Wq1z W3] (2M x Kx) with bq1 + Wq1z b3
    size_t fpi_x6, fpi_b, fq_x6, fq_b, fold_p, fold_q;
    size_t fw1_x6;         // ... and TOLD.next's folded first layer again in the chain x6 layout (the policy rows)
    size_t total;
};
constexpr int PACK_MAX_JOBS = 96;              // job-table capacity (pack_jobs emits ~40-60)
constexpr int PACK_JOB_BYTES = 192;            // >= sizeof(PackJob) (static_assert at its definition)
constexpr int PACK_HDR_BYTES = 256;            // PackHdr slot ahead of the job table
// The header of the packed buffer's job table. `nonce` names the table last uploaded into the buffer; every pack
// launch carries the nonce of the table its host record says is there and checks it on the device, so a pack that
// would read another table (a re-allocated or re-zeroed buffer, a captured graph whose buffer was re-keyed) poisons
// the weights and raises `status` instead of packing from stale pointers. `status` is sticky until the next upload;
// every plan ORs it into the caller's status word (TDMPC_STATUS_PACK_STALE).
struct PackHdr {
    unsigned long long nonce;
    int status, njobs;
};

// Matrices kept in the x6 layout: fp32 = hi + mid + lo, three bf16 planes. Block (nb, g) of 32 rows x 16 k is
// [3 planes][64 lanes][8 bf16]: lane l (r = l & 31, h = l >> 5) element j holds row 32 nb + r,
// k = 16 g + 8 (j >> 2) + 4 h + (j & 3) -- the v_mfma_f32_32x32x16_bf16 A fragment, with the k order the chain
// kernel's fp32 activation panel gives its B fragment (two ds_read_b128 of quads 4g + h and 4g + 2 + h).
enum { X6_W1X, X6_W2D, X6_W2R, X6_W3D, X6_WP1, X6_WP2, X6_WP3, X6_WQ1X, X6_WQ2, X6_N };
// rows / k of x6 matrix i (the source panel's rows and columns)
__host__ __device__ inline void x6_shape(const Layout& w, int i, int* rows, int* k) {
    const int M = w.M;
    switch (i) {
        case X6_W1X: *rows = 2 * M; *k = w.Kx; break;
        case X6_W2D: case X6_W2R: case X6_WP2: *rows = M; *k = M; break;
        case X6_W3D: *rows = w.Lr; *k = M; break;
        case X6_WP1: *rows = M; *k = w.Lp; break;
        case X6_WP3: *rows = w.Ar; *k = M; break;
        case X6_WQ1X: *rows = 2 * M; *k = w.Kx; break;
        default: *rows = 2 * M; *k = M; break;   // X6_WQ2: the two Q heads' panels stacked
    }
}
inline size_t x6_src(const Layout& w, int i) {
    const size_t src[X6_N] = {w.w1x, w.w2d, w.w2r, w.w3d, w.wp1, w.wp2, w.wp3, w.wq1x, w.wq2};
    return src[i];
}

bool make_layout(const tdmpc_dims* d, Layout* w) {
    if (!d || d->action_dim <= 0 || d->latent_dim <= 0 || d->mlp_dim <= 0 || d->mlp_dim % 64) return false;
    w->A = d->action_dim; w->L = d->latent_dim; w->M = d->mlp_dim; w->E = d->enc_dim;
    w->Ap = (int)rup(w->A, 8); w->Lp = (int)rup(w->L, 8); w->Kx = w->Ap + w->Lp;
    w->Ar = (int)rup(w->A, 32); w->Lr = (int)rup(w->L, 32);
    w->modality = d->modality; w->obs_dim = d->obs_dim;
    w->img_c = d->img_c; w->img_hw = d->img_hw; w->nch = d->num_channels;
    size_t o = 0;
    auto take = [&](size_t n) { size_t r = o; o += rup(n, 64); return r; };
    if (d->modality == 0) {
        if (d->obs_dim <= 0 || d->enc_dim <= 0) return false;
        w->enc_w1t = take((size_t)w->E * d->obs_dim); w->enc_b1 = take(w->E);
        w->enc_norm = d->enc_norm != 0;
        w->enc_lng = take(w->E); w->enc_lnb = take(w->E);
        w->enc_w2t = take((size_t)w->L * w->E); w->enc_b2 = take(w->L);
        w->flat = 0;
    } else {
        if (d->img_c <= 0 || d->img_hw <= 0 || d->num_channels <= 0 || d->enc_norm) return false;
        w->enc_norm = 0;
        static const int ks[4] = {7, 5, 3, 3};
        int s = d->img_hw, cin = d->img_c;
        w->conv_hw[0] = s;
        for (int i = 0; i < 4; ++i) {
            w->cw[i] = take((size_t)w->nch * cin * ks[i] * ks[i]);
            w->cwt[i] = take((size_t)w->nch * cin * ks[i] * ks[i]);
            w->cb[i] = take(w->nch);
            s = (s - ks[i]) / 2 + 1; cin = w->nch;
            w->conv_hw[i + 1] = s;
            if (s <= 0) return false;
        }
        w->flat = w->nch * s * s;
        w->pl_wt = take((size_t)w->L * w->flat); w->pl_b = take(w->L);
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
    for (int i = 0; i < X6_N; ++i) {
        int r, k;
        x6_shape(*w, i, &r, &k);
        w->x6[i] = take(rup(r, 32) * rup(k, 16) * 3 / 2);   // bf16 elements / 2 = floats
    }
    for (int i = 0; i < X6_N; ++i) {
        int r, k;
        x6_shape(*w, i, &r, &k);
        w->x6q[i] = take(rup(r, 16) * rup(k, 32) * 3 / 2);
    }
    w->jobtab = take((size_t)(PACK_HDR_BYTES + PACK_MAX_JOBS * PACK_JOB_BYTES) / 4);
    // the statistics block: only where the wide heads may run (B N >= 4096 rows, M = 512) and the Cholesky's
    // upper-packed fp64 factor fits one workgroup's LDS
    w->nqs = w->nsr = 0;
    w->x6qs = w->bqs = w->x6qf = w->bqf = w->qs_gram = 0;
    {
        const int n = w->A + w->L + 1;
        if (w->M == 512 && (long)d->max_batch * d->num_samples >= 4096 && n + 1 <= 256 &&
            ((size_t)n * (n + 1) / 2 + n) * 8 <= 150 * 1024) {
            w->nqs = n;
            w->nsr = n + 1 <= 128 ? 128 : 256;
            w->x6qs = take((size_t)2 * w->nsr * rup(w->Kx, 32) * 3 / 2);
            w->bqs = take((size_t)2 * w->nsr);
            w->x6qf = take((size_t)2 * w->M * rup(w->Kx, 32) * 3 / 2);
            w->bqf = take((size_t)2 * w->M);
            w->qs_gram = take((size_t)2 * n * n * 2);
        }
    }
    w->fold = 0;
    w->x6qw = w->bfw = w->fold_w = 0;
    w->fpi_x6 = w->fpi_b = w->fq_x6 = w->fq_b = w->fold_p = w->fold_q = w->fw1_x6 = 0;
    if (w->M == 512 && w->Lp == w->M && w->Lr == w->M) {
        w->fold = 1;
        w->x6qw = take((size_t)2 * w->M * rup(w->Kx, 32) * 3 / 2);
        w->bfw = take((size_t)2 * w->M);
        w->fold_w = take((size_t)2 * w->M * w->M);
        int r, k;
        x6_shape(*w, X6_WP1, &r, &k);
        w->fpi_x6 = take(rup(r, 32) * rup(k, 16) * 3 / 2);
        w->fpi_b = take((size_t)w->M);
        x6_shape(*w, X6_WQ1X, &r, &k);
        w->fq_x6 = take(rup(r, 32) * rup(k, 16) * 3 / 2);
        w->fq_b = take((size_t)2 * w->M);
        w->fold_p = take((size_t)w->M * w->M);
        w->fold_q = take((size_t)2 * w->M * w->M);
        x6_shape(*w, X6_W1X, &r, &k);
        w->fw1_x6 = take(rup(r, 32) * rup(k, 16) * 3 / 2);
    }
    w->total = o;
    return true;
}

// ------------------------------------------------------------------------------------------------ workspace
// split_step_kernel: the M-wide second layer is split over SPLIT_S column slices (one workgroup each) for launches
// of at most SPLIT_MAX_ROWS rows.
constexpr int SPLIT_S = 4;
constexpr int SPLIT_MAX_ROWS = 4096;

struct Work {
    float* X;        // (Hmax+1) panels [Xrows][Kx]: step inputs [a|z]; X_H is the terminal input
    float* H1;       // panel [Xrows][2M]
    float* H2;       // panel [Xrows][2M]
    float2* st1;     // [B*T][2M/64] LayerNorm partial moments of Q layer 0
    float2* st2;     // [B*T][2M/64] of Q layer 1
    float* rpart;    // [B*T][M/32] reward-head partial dots
    float* G;        // [B*T] discounted return so far
    float* rlast;    // [B*T] reward at t = H-1
    float* value;    // [B*T]
    float* qv;       // [2][xrows] Q-head outputs of the chain path
    float* z0c;      // [B][2][M] TOLD.next first layer's z0 share + bias per env (t = 0 steps of the chain kernel)
    float* pimu;     // [xrows][Ap] tanh(pi(z_H)) per X row: the pi rows' terminal means, reused by CEM iterations >= 1
    float* zpart;    // [2][SPLIT_S][split_rows][max(Lr, Ar)] split-step partial z' / pi outputs, two parities
    float* rpart_s;  // [2][SPLIT_S][split_rows] split-step partial reward dots
    int split_rows;  // rows the split partial buffers hold (min(xrows, SPLIT_MAX_ROWS))
    float* z0;       // [B][Lp] dense
    float* mean;     // [B][Hmax][A]
    float* stdv;     // [B][Hmax][A]
    float* enc_tmp;  // pixel conv activations
    size_t x_stride; // floats per X_t
    int xrows;       // rup(B*T, 32)
    char* p1;        // exchange region of the persistent one-env plan (plan1.inc), p1_bytes (0: not eligible)
    size_t p1_bytes;
    size_t total;
};

size_t pixel_act_floats(const Layout& w) {
    size_t m = 0;
    for (int i = 1; i <= 4; ++i) m = std::max(m, (size_t)w.nch * w.conv_hw[i] * w.conv_hw[i]);
    return m;
}

// ---- persistent one-env plan (plan1.inc): its exchange region and shape limits
constexpr int P1_NG = 8;      // row groups
constexpr int P1_WPG = 32;    // workgroups per group: 2 heads x 16 column slices
constexpr int P1_RTM = 3;     // 32-row tiles per group at most
constexpr int P1_ROWS = 32 * P1_RTM;
// hidden-activation exchange row stride (floats): 512 + 32, so the 16 rows a wave reads per k-step do not all map to
// one L2 channel (a 2 KB stride puts every row's 128 B line of a k-step on the same channel)
constexpr int P1_H1LD = 544;
constexpr unsigned P1_XCC_TAB = P1_NG * 256 + 256;   // sync block: per-workgroup XCD ids (placement census)
constexpr unsigned P1_SPIN_MAX = 400000;   // ~0.3-0.5 s of polling before a workgroup gives up

// exchange region bytes (all offsets 256-aligned) for dims; 0 = not eligible
struct P1Region {
    unsigned o_sync, o_xb, o_h1, o_zp, o_rp, o_pp, o_qm, o_qp, o_val, o_rl, o_mu, o_y2, xb_t, xb_g, total;
};

// the first layer's 32-k steps the kernel instantiation runs (4 or 6; steps past K meet zero activations)
inline int p1_ks(const Layout& w) { return (w.Kx + 31) / 32 <= 4 ? 4 : 6; }
// XB row floats: [a | 0 | z | 0] zero-padded past both first layers' KS 32-k steps (the policy's starts at Ap)
inline int p1_kxs(const Layout& w) { return (int)rup(w.Ap + 32 * p1_ks(w), 16); }

inline P1Region p1_region(const tdmpc_dims* d, const Layout& w) {
    P1Region r;
    memset(&r, 0, sizeof r);
    const size_t T = d->num_samples + d->num_pi, Hm = d->max_horizon;
    size_t o = 0;
    auto take = [&](size_t b) { size_t x = o; o += rup(b, 256); return (unsigned)x; };
    r.o_sync = take(P1_NG * 256 + 256 + 4 * P1_NG * P1_WPG);   // counters, error word, XCD census
    r.xb_t = (unsigned)((size_t)P1_ROWS * p1_kxs(w) * 4);
    r.xb_g = (unsigned)((Hm + 1) * r.xb_t);
    r.o_xb = take((size_t)P1_NG * r.xb_g);
    r.o_h1 = take((size_t)P1_NG * 2 * P1_ROWS * P1_H1LD * 4);
    r.o_zp = take((size_t)P1_NG * 16 * P1_ROWS * w.Lr * 4);
    r.o_rp = take((size_t)P1_NG * 16 * P1_ROWS * 4);
    r.o_pp = take((size_t)P1_NG * 16 * P1_ROWS * w.Ar * 4);
    r.o_qm = take((size_t)P1_NG * 2 * 16 * P1_ROWS * 8);
    r.o_qp = take((size_t)P1_NG * 2 * 16 * P1_ROWS * 4);
    r.o_val = take(2 * T * 4);
    r.o_rl = take(T * 4);
    r.o_mu = take((size_t)P1_NG * P1_ROWS * w.Ap * 4);   // the pi rows' cached terminal means
    r.o_y2 = take((size_t)P1_NG * 2 * P1_ROWS * P1_H1LD * 4);   // the Q heads' raw second-layer rows
    r.total = (unsigned)o;
    return r;
}

// LDS of plan1_kernel: the hidden-layer weight slice (96 KB), a layer's 32-column slice of the group's rows (+ per-row
// LayerNorm scalars), the CEM step's top-k keys and elite actions, mean / std / scores / bias slices
__host__ __device__ inline size_t p1_cem_floats(int H, int K, int A, int T) {
    // CEM step: top-k keys + elites | phases: K-half partials (8 KB) + every wave's dynamics W3 fragment (8 x 3 KB)
    const size_t c = (size_t)(T + 63) / 64 * 64 * 2 + rup((size_t)H * K * A, 4);
    return c > 8192 ? c : 8192;
}
inline size_t p1_lds_bytes(int H, int K, int A, int T) {
    const size_t HA = (size_t)H * A;
    return ((size_t)32 * 3 * 64 * 4 + (size_t)P1_ROWS * 36 + 2 * P1_ROWS + p1_cem_floats(H, K, A, T) +
            3 * rup(HA, 4) + 64 + 64 + 16 + 32 + 648) * 4;
}

// plan1_kernel's shape limits (dims only; the call adds batch == 1 and >= 256 CUs): mlp_dim 512, at most 96 rows
// (three 32-row tiles) per row group, first-layer K <= 192 and latent K <= 192 (three 16-k groups per wave), latent
// and action heads <= 128 / 64 columns, LDS within 160 KB.
inline bool p1_dims_ok(const tdmpc_dims* d, const Layout& w) {
    if (w.M != 512 || d->num_elites > 64) return false;
    const int N = d->num_samples, P = d->num_pi, T = N + P;
    const int sr = (N + P1_NG - 1) / P1_NG, pr = (P + P1_NG - 1) / P1_NG;
    if (sr + pr > P1_ROWS || T > 1024) return false;
    if ((w.Kx + 15) / 16 > 12 || (w.Lp + 15) / 16 > 12 || w.Lr > 128 || w.Ar > 128) return false;
    return p1_lds_bytes(d->max_horizon, d->num_elites, w.A, T) <= 160 * 1024;
}

// extra: rows per env beyond N + P (the iCEM planner keeps up to K reused elite trajectories per env)
void make_work(const tdmpc_dims* d, const Layout& w, char* base, Work* k, int extra = 0) {
    const size_t B = d->max_batch, N = d->num_samples, P = d->num_pi, T = N + P + extra, H = d->max_horizon;
    const size_t M = w.M;
    size_t o = 0;
    auto take = [&](size_t bytes) { size_t r = o; o += rup(bytes, 256); return base ? base + r : nullptr; };
    k->xrows = (int)rup(B * T, 32);
    k->x_stride = (size_t)k->xrows * w.Kx;
    k->X = (float*)take((H + 1) * k->x_stride * 4);
    k->H1 = (float*)take((size_t)k->xrows * 2 * M * 4);
    k->H2 = (float*)take((size_t)k->xrows * 2 * M * 4);
    k->st1 = (float2*)take(B * T * (2 * M / 64) * 8);
    k->st2 = (float2*)take(B * T * (2 * M / 64) * 8);
    k->rpart = (float*)take(B * T * (M / 32) * 4);
    k->G = (float*)take(B * T * 4);
    k->rlast = (float*)take(B * T * 4);
    k->value = (float*)take(B * T * 4);
    k->qv = (float*)take(2 * (size_t)k->xrows * 4);
    k->pimu = (float*)take((size_t)k->xrows * w.Ap * 4);
    k->z0c = (float*)take(B * 2 * M * 4);
    k->split_rows = std::min(k->xrows, SPLIT_MAX_ROWS);
    k->zpart = (float*)take((size_t)2 * SPLIT_S * k->split_rows * std::max(w.Lr, w.Ar) * 4);
    k->rpart_s = (float*)take((size_t)2 * SPLIT_S * k->split_rows * 4);
    k->z0 = (float*)take(B * w.Lp * 4);
    k->mean = (float*)take(B * H * w.A * 4);
    k->stdv = (float*)take(B * H * w.A * 4);
    k->enc_tmp = (float*)take(d->modality ? 2 * B * pixel_act_floats(w) * 4 : 256);
    k->p1_bytes = p1_dims_ok(d, w) && !extra ? p1_region(d, w).total : 0;
    k->p1 = k->p1_bytes ? (char*)take(k->p1_bytes) : nullptr;
    k->total = o;
}

size_t cem_lds_bytes(int T, int H, int K, int A) {
    const size_t nl = (T + 63) / 64;
    return nl * 64 * 8 + ((size_t)H * K * A + 64 + 4 * rup((size_t)H * A, 4) + 64 + 32) * 4;
}

bool check_dims(const tdmpc_dims* d) {
    if (!d) return false;
    if (d->num_samples <= 0 || d->num_pi < 0 || d->num_elites <= 0 || d->max_horizon <= 0 ||
        d->max_horizon > 16 || d->max_iterations <= 0 || d->max_batch <= 0) return false;
    const int T = d->num_samples + d->num_pi;
    if (d->num_elites > T || d->num_elites > 64 || T > 4096) return false;
    Layout w;
    if (!make_layout(d, &w)) return false;
    if (w.Kx > 1024 || w.M > 1024 || w.L > 1024 || w.A > 256 || w.E > 1024) return false;
    if (cem_lds_bytes(T, d->max_horizon, d->num_elites, w.A) > 160 * 1024) return false;
    return true;
}

// ------------------------------------------------------------------------------------------------ device math
DEVI float elu1(float x) { return x > 0.f ? x : expm1f(x); }
DEVI float fmul(float a, float b) { return __fmul_rn(a, b); }
DEVI float fadd(float a, float b) { return __fadd_rn(a, b); }
// torch.clamp propagates NaN; plain fminf/fmaxf would drop it.
DEVI float tclamp(float x, float lo, float hi) { return x != x ? x : fminf(fmaxf(x, lo), hi); }
DEVI float nan_to_num(float x) {
    if (x != x) return 0.f;
    if (isinf(x)) return x > 0 ? 3.402823466e38f : -3.402823466e38f;
    return x;
}
__host__ __device__ inline size_t pidx(size_t r, size_t c, size_t cols) {
    return (r >> 5) * (cols * 32) + (c >> 2) * 128 + (r & 31) * 4 + (c & 3);
}

struct RowMap {  // logical row m -> physical row (m / G) * S + O + m % G
    int G, S, O;
};
DEVI int map_row(const RowMap& r, int m) { return (m / r.G) * r.S + r.O + (m % r.G); }

// Panel operand: element (r, k) at p + (r>>5)*ts + (q0 + (k>>2))*128 + (r&31)*4 + (k&3)
struct Opnd {
    const float* p; long ts; int q0;
};
struct Outp {
    float* p; long ts; int q0;
};

// ------------------------------------------------------------------------------------------------ linear
enum { PRO_PLAIN = 0, PRO_LN_TANH = 1 };
enum { EPI_ELU = 0, EPI_LIN_Z = 1, EPI_PI = 2, EPI_LNSTATS = 3, EPI_ELU_DOT = 4 };

// Cheap activations for the hot loops: |error| < 2e-7 against libm over the value range here, well inside
// the parity tolerance (tests/test_gpu_plan.py). ELU uses exp(x) - 1 like ATen's scalar path.
DEVI float elu_f(float x) { return x > 0.f ? x : __expf(x) - 1.f; }
DEVI float tanh_f(float x) {
    const float e = __expf(-2.f * fabsf(x));
    return copysignf(__fdividef(1.f - e, 1.f + e), x);
}

struct LinProb {
    Opnd A; Opnd W;
    const float* bias;            // [>= grid columns]
    Outp C;
    int N;                        // output columns covered by the grid (tiles beyond return early)
    int nvalid;                   // real output columns; columns >= nvalid are written as 0
    int nstore;                   // stored columns (multiple of 4)
    int epi;
    const float2* ln_stats; int ln_ld; int ln_t0; int ln_nt;   // PRO_LN_TANH: per-64-col (mean, M2)
    const float* ln_g; const float* ln_b;                      // LN affine for this problem's K columns
    float2* st_out; int st_ld;                                 // EPI_LNSTATS: per-64-col moments out
    const float* dotw; float* dot_out; int dot_ld;             // EPI_ELU_DOT: per-block partial dots
};

struct LinArgs {
    LinProb p[2];
    int M, K, kch;
    int a_mapped, c_mapped;
    RowMap amap, cmap;
    int A;                        // action dim (EPI_PI noise rows)
    // EPI_LIN_Z: reward head + return
    const float* rpart; int rpart_nt; const float* b3r;
    float* G; float* rlast; float disc; int first, last;
    // EPI_PI
    const float* eps; int eps_G; long eps_env; long eps_off; float min_std, lo, hi;
};

// Shared epilogue of the linear kernels. smem holds KS partial tiles [KS][R][C+4] (summed here), sbias /
// sdotw the bias and reward-head weights of this tile's columns, srp the reward partial dots of its rows.
template <int R, int C>
DEVI void lin_epilogue(const LinArgs& args, const LinProb& P, float* smem, int KS, int m0, int n0,
                       const float* sbias, const float* sdotw, const float* srp) {
    constexpr int LDC = C + 4;
    constexpr int BW = C >= 64 ? 64 : C;     // row-reduction block width
    constexpr int NB = C / BW;
    const int nthr = blockDim.x;
    const int epi = P.epi;
    // ---- epilogue phase A: thread -> (row, column quads); 32 consecutive lanes own 32 consecutive rows,
    // so one quad stored by them is 512 contiguous bytes of the panel layout.
    const bool need_red = epi == EPI_LNSTATS || epi == EPI_ELU_DOT;
    {
        const int rows_blk = R / 32;
        const int row = (threadIdx.x & 31) + 32 * ((threadIdx.x >> 5) % rows_blk);
        const int cq0 = (threadIdx.x >> 5) / rows_blk, cqs = nthr / R;
        const int lm = m0 + row;
        // threads past the last full row sweep (nthr % R) idle in this phase
        const bool active = (int)threadIdx.x < cqs * R;
        const bool rval = lm < args.M;
        const int crow = rval ? (args.c_mapped ? map_row(args.cmap, lm) : lm) : 0;
        float* Cbase = P.C.p ? P.C.p + (size_t)(crow >> 5) * P.C.ts + (crow & 31) * 4 : nullptr;
        for (int cq = active ? cq0 : C / 4; cq < C / 4; cq += cqs) {
            const int c = 4 * cq;
            float4 v = *(const float4*)(smem + (size_t)row * LDC + c);
            for (int w = 1; w < KS; ++w) {
                const float4 u = *(const float4*)(smem + ((size_t)w * R + row) * LDC + c);
                v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
            }
            const int n = n0 + c;
            const float4 bb = *(const float4*)(sbias + c);
            float o[4] = {v.x + bb.x, v.y + bb.y, v.z + bb.z, v.w + bb.w};
            if (epi == EPI_ELU || epi == EPI_ELU_DOT) {
#pragma unroll
                for (int i = 0; i < 4; ++i) o[i] = elu_f(o[i]);
            }
            if (epi == EPI_PI) {
                // TOLD.pi + TruncatedNormal.sample(clip=0.3) (tdmpc.py:39-45, helper.py:86-96)
                const int e = lm / args.eps_G, rr = lm % args.eps_G;
                const float* ep = args.eps + (size_t)e * args.eps_env + args.eps_off + (size_t)rr * args.A;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    float x = 0.f;
                    if (n + i < P.nvalid && rval) {
                        const float muv = tanhf(o[i]);
                        x = muv;
                        if (args.min_std > 0.f) {
                            const float ee = tclamp(fmul(ep[n + i], args.min_std), -0.3f, 0.3f);
                            x = tclamp(fadd(muv, ee), args.lo, args.hi);
                        }
                    }
                    o[i] = x;
                }
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if (n + i >= P.nvalid) o[i] = 0.f;
            }
            if (need_red) *(float4*)(smem + (size_t)row * LDC + c) = make_float4(o[0], o[1], o[2], o[3]);
            if (rval && n < P.nstore)
                *(float4*)(Cbase + (size_t)(P.C.q0 + (n >> 2)) * 128) = make_float4(o[0], o[1], o[2], o[3]);
        }
    }
    // ---- epilogue phase B: one thread per (row, BW-column block) for the row reductions
    if (need_red) {
        __syncthreads();
        for (int t = threadIdx.x; t < R * NB; t += nthr) {
            const int row = t % R, blk = t / R;
            const int lm = m0 + row;
            if (lm >= args.M) continue;
            const float* v = smem + (size_t)row * LDC + blk * BW;
            if (epi == EPI_LNSTATS) {
                // LayerNorm partial moments of this 64-column slice: (mean, sum of squared deviations)
                float s = 0.f;
                for (int c = 0; c < BW; c += 4) {
                    const float4 x = *(const float4*)(v + c);
                    s += (x.x + x.y) + (x.z + x.w);
                }
                const float mean = s / (float)BW;
                float m2 = 0.f;
                for (int c = 0; c < BW; c += 4) {
                    const float4 x = *(const float4*)(v + c);
                    const float d0 = x.x - mean, d1 = x.y - mean, d2 = x.z - mean, d3 = x.w - mean;
                    m2 += (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3);
                }
                P.st_out[(size_t)lm * P.st_ld + (n0 / 64) + blk] = make_float2(mean, m2);
            } else {
                const float* wv = sdotw + blk * BW;
                float s = 0.f;
                for (int c = 0; c < BW; c += 4) {
                    const float4 x = *(const float4*)(v + c), w4 = *(const float4*)(wv + c);
                    s += (x.x * w4.x + x.y * w4.y) + (x.z * w4.z + x.w * w4.w);
                }
                P.dot_out[(size_t)lm * P.dot_ld + (n0 / BW) + blk] = s;
            }
        }
    }
    if (epi == EPI_LIN_Z && blockIdx.y == 0) {
        // reward head (helper.mlp last Linear, M -> 1) from the partial dots, then
        // G += discount * reward (tdmpc.py:89) with float32(discount) like ATen's scalar mul.
        for (int row = threadIdx.x; row < R; row += nthr) {
            const int lm = m0 + row;
            if (lm >= args.M) continue;
            const int crow = args.c_mapped ? map_row(args.cmap, lm) : lm;
            float s = 0.f;
            for (int i = 0; i < args.rpart_nt; ++i) s += srp[row * args.rpart_nt + i];
            const float rew = s + args.b3r[0];
            const float dr = fmul(args.disc, rew);
            args.G[crow] = args.first ? dr : fadd(args.G[crow], dr);
            if (args.last) args.rlast[crow] = rew;
        }
    }
}

// Fused nn.Linear on v_mfma_f32_32x32x2_f32.
//   Workgroup tile: R = 32*TM*WGM rows x C = 32*TN*WGN columns; waves = WGM*WGN*KS where KS (runtime,
//   blockDim / (64*WGM*WGN)) splits K into chunks of KCH. Each wave owns a (32*TM) x (32*TN) register tile.
//   ROLL = false: a wave preloads its whole K chunk (<= KCH/8 groups) -- the latency configuration for
//   small row counts. ROLL = true: KS = 1 and a 4-deep prefetch ring walks the full K -- the throughput
//   configuration for large row counts.
template <int TM, int TN, int WGM, int WGN, int PRO, int KCH, bool ROLL>
__global__ void __launch_bounds__(512) linear_kernel(const LinArgs args) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int R = 32 * TM * WGM, C = 32 * TN * WGN, LDC = C + 4;
    const LinProb& P = args.p[blockIdx.z];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nthr = blockDim.x;
    const int r = lane & 31, h = lane >> 5;
    const int m0 = blockIdx.x * R, n0 = blockIdx.y * C;
    if (n0 >= P.N) return;  // uniform over the workgroup
#ifdef TDMPC_STAMPS
    unsigned long long st_[6];
    unsigned long long rt0_ = __builtin_amdgcn_s_memrealtime();
    STAMP(0);
#endif
    const int KS = nthr / (64 * WGM * WGN);
    const int wm = wave % WGM, wn = (wave / WGM) % WGN, ks = wave / (WGM * WGN);
    const int epi = P.epi;

    // LDS: partial tiles [KS][R][LDC] | bias [C] | dotw [C] | rpart [R][rpart_nt]
    float* sbias = smem + (size_t)KS * R * LDC;
    float* sdotw = sbias + C;
    float* srp = sdotw + C;
    // prefetch the epilogue's operands now; the loads land while the MFMAs run
    for (int i = threadIdx.x; i < C / 4; i += nthr) {
        const int n = n0 + 4 * i;
        *(float4*)(sbias + 4 * i) = *(const float4*)(P.bias + n);
        if (epi == EPI_ELU_DOT) *(float4*)(sdotw + 4 * i) = *(const float4*)(P.dotw + n);
    }
    if (epi == EPI_LIN_Z && blockIdx.y == 0)
        for (int i = threadIdx.x; i < R * args.rpart_nt; i += nthr) {
            const int lm = m0 + i / args.rpart_nt;
            srp[i] = lm < args.M ? args.rpart[(size_t)lm * args.rpart_nt + i % args.rpart_nt] : 0.f;
        }

    // this lane's A rows (TM of them) and W rows (TN)
    const float* Abase[TM];
    int arow[TM];
    float mu[TM], rs[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const int m = m0 + (wm * TM + i) * 32 + r;
        const int mm = m < args.M ? m : 0;
        arow[i] = args.a_mapped ? map_row(args.amap, mm) : mm;
        Abase[i] = P.A.p + (size_t)(arow[i] >> 5) * P.A.ts + (arow[i] & 31) * 4;
        mu[i] = 0.f; rs[i] = 1.f;
        if (PRO == PRO_LN_TANH) {
            // Chan-combine the producer's per-64-column (mean, M2) into mean and 1/sqrt(var + 1e-5)
            const float2* st = P.ln_stats + (size_t)mm * P.ln_ld + P.ln_t0;
            float n = 0.f, mean = 0.f, m2 = 0.f;
            for (int q = 0; q < P.ln_nt; ++q) {
                const float2 s = st[q];
                const float nn = n + 64.f, delta = s.x - mean;
                mean += delta * 64.f / nn;
                m2 += s.y + delta * delta * n * 64.f / nn;
                n = nn;
            }
            mu[i] = mean;
            rs[i] = 1.0f / sqrtf(fmaxf(m2 / n, 0.f) + 1e-5f);
        }
    }
    const float* Wbase = P.W.p + (size_t)((n0 >> 5) + wn * TN) * P.W.ts + r * 4;

    floatx16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

    auto mfma_group = [&](float4 (&a)[TM], const float4 (&b)[TN], int k) {
        if (PRO == PRO_LN_TANH) {
            // helper.q: LayerNorm -> Tanh, as ATen computes it: (x * rstd + (-rstd * mean)) * g + b
            const float4 gg = *(const float4*)(P.ln_g + k);
            const float4 bb = *(const float4*)(P.ln_b + k);
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const float sh = -rs[i] * mu[i];
                a[i].x = tanh_f(fadd(fmul(fadd(fmul(a[i].x, rs[i]), sh), gg.x), bb.x));
                a[i].y = tanh_f(fadd(fmul(fadd(fmul(a[i].y, rs[i]), sh), gg.y), bb.y));
                a[i].z = tanh_f(fadd(fmul(fadd(fmul(a[i].z, rs[i]), sh), gg.z), bb.z));
                a[i].w = tanh_f(fadd(fmul(fadd(fmul(a[i].w, rs[i]), sh), gg.w), bb.w));
            }
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].x, b[j].x, acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].y, b[j].y, acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].z, b[j].z, acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].w, b[j].w, acc[i][j], 0, 0, 0);
            }
    };
    auto load_group = [&](int g, float4 (&a)[TM], float4 (&b)[TN]) {
        const int kq = 2 * g + h;  // quad of this lane half within K
#pragma unroll
        for (int j = 0; j < TN; ++j) b[j] = *(const float4*)(Wbase + (size_t)j * P.W.ts + kq * 128);
#pragma unroll
        for (int i = 0; i < TM; ++i) a[i] = *(const float4*)(Abase[i] + (size_t)(P.A.q0 + kq) * 128);
    };

    if constexpr (!ROLL) {
        constexpr int NG = KCH / 8;
        const int g0 = (ks * args.kch) >> 3;
        const int ng = min(args.kch, args.K - ks * args.kch) >> 3;
        float4 av[NG][TM], bv[NG][TN];
#pragma unroll
        for (int g = 0; g < NG; ++g)
            if (g < ng) load_group(g0 + g, av[g], bv[g]);
#ifdef TDMPC_STAMPS
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        STAMP(1);
#endif
#pragma unroll
        for (int g = 0; g < NG; ++g)
            if (g < ng) mfma_group(av[g], bv[g], 8 * (g0 + g) + 4 * h);
    } else {
        constexpr int D = 4;
        const int gbase = (ks * args.kch) >> 3;
        const int ng = min(args.kch, args.K - ks * args.kch) >> 3;
        float4 ra[D][TM], rb[D][TN];
#pragma unroll
        for (int d = 0; d < D; ++d)
            if (d < ng) load_group(gbase + d, ra[d], rb[d]);
#ifdef TDMPC_STAMPS
        STAMP(1);
#endif
        for (int gb = 0; gb < ng; gb += D) {
#pragma unroll
            for (int d = 0; d < D; ++d) {
                const int g = gb + d;
                if (g < ng) {
                    float4 ta[TM], tb[TN];
#pragma unroll
                    for (int i = 0; i < TM; ++i) ta[i] = ra[d][i];
#pragma unroll
                    for (int j = 0; j < TN; ++j) tb[j] = rb[d][j];
                    if (g + D < ng) load_group(gbase + g + D, ra[d], rb[d]);
                    mfma_group(ta, tb, 8 * (gbase + g) + 4 * h);
                }
            }
        }
    }

    // partial tiles -> LDS [ks][row][col]; C/D map: col = lane&31, row = (e&3) + 8*(e>>2) + 4*(lane>>5)
    {
        float* base = smem + (size_t)ks * R * LDC + (size_t)(wm * TM * 32) * LDC + wn * TN * 32;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int e = 0; e < 16; ++e)
                    base[(size_t)(i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h) * LDC + j * 32 + r] = acc[i][j][e];
    }
#ifdef TDMPC_STAMPS
    STAMP(2);
#endif
    __syncthreads();
#ifdef TDMPC_STAMPS
    STAMP(3);
#endif

    lin_epilogue<R, C>(args, P, smem, KS, m0, n0, sbias, sdotw, srp);
#ifdef TDMPC_STAMPS
    __syncthreads();
    STAMP(4);
    STAMP_RECORD();
#endif
}

DEVI float f4c(const float4& v, int k) { return k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w; }

// Throughput configuration for large row counts: LDS-staged (three stage buffers) output tile of
// R = 32*TM*WGM rows x C = 32*TN*WGN columns over K tiles of KT. WGM x WGN waves (2x2 or 2x4), each owning a (32*TM) x (32*TN)
// register tile. With the panel layout one K tile of one 32-row block is a contiguous 4 KiB, so staging is
// 1 KiB wave loads and every fragment read is a conflict-free ds_read_b128; global traffic per MFMA is
// shared by the whole workgroup.
template <int TM, int TN, int WGM, int WGN, int KT, bool FK>
__global__ void __launch_bounds__(64 * WGM * WGN) linear_lds_kernel(const LinArgs args) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int R = 32 * TM * WGM, C = 32 * TN * WGN, NT = 64 * WGM * WGN;
    constexpr int RB = R / 32, CB = C / 32;            // 32-row / 32-col blocks
    constexpr int KQ = KT / 4;                         // k quads per stage
    constexpr int SA = RB * KQ * 128, SW = CB * KQ * 128;   // floats per stage (KQ quads x 32 x 4 per block)
    constexpr int CA = RB * KQ * 32 / NT, CW = CB * KQ * 32 / NT;   // 16-B chunks per thread per stage
    static_assert(CA * NT == RB * KQ * 32 && CW * NT == CB * KQ * 32, "stage does not split over the threads");
    const LinProb& P = args.p[blockIdx.z];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int wm = wave % WGM, wn = wave / WGM;
    const int m0 = blockIdx.x * R, n0 = blockIdx.y * C;
    if (n0 >= P.N) return;
#ifdef TDMPC_STAMPS
    unsigned long long st_[5];
    const unsigned long long rt0_ = __builtin_amdgcn_s_memrealtime();
    STAMP(0);
#endif
    const int epi = P.epi;
    // LDS: stage buffers [3][SA + SW]; bias [C]; dotw [C]; per-row 32-column partials [R][C/32] (float2)
    constexpr int BUF = SA + SW;
    constexpr int BODY = 3 * BUF;
    float* sbias = smem + BODY;
    float* sdotw = sbias + C;
    float2* spart = (float2*)(sdotw + C);
    for (int i = tid; i < C / 4; i += NT) {
        const int n = n0 + 4 * i;
        *(float4*)(sbias + 4 * i) = *(const float4*)(P.bias + n);
        if (epi == EPI_ELU_DOT) *(float4*)(sdotw + 4 * i) = *(const float4*)(P.dotw + n);
    }

    // staging slots: chunk c = tid + i*NT of a stage -> block c / (32*KQ), quad (c>>5) % KQ, row c&31
    const float* Asrc[CA];
#pragma unroll
    for (int i = 0; i < CA; ++i) {
        const int cidx = tid + i * NT;
        const int m = m0 + (cidx / (32 * KQ)) * 32 + (cidx & 31);
        const int mm = m < args.M ? m : 0;
        const int arow = args.a_mapped ? map_row(args.amap, mm) : mm;
        Asrc[i] = P.A.p + (size_t)(arow >> 5) * P.A.ts + (arow & 31) * 4 + (size_t)P.A.q0 * 128;
    }
    // per-chunk W pointers (chunk c: column block c / (32*KQ), quad (c>>5) % KQ, column c&31 of the block)
    const float* Wsrc[CW];
#pragma unroll
    for (int i = 0; i < CW; ++i) {
        const int cidx = tid + i * NT;
        Wsrc[i] = P.W.p + (size_t)((n0 >> 5) + cidx / (32 * KQ)) * P.W.ts + ((cidx >> 5) % KQ) * 128 + (cidx & 31) * 4;
    }
    const int kq_total = args.K >> 2;
    auto stage_load = [&](int kt, float4 (&ra)[CA], float4 (&rw)[CW]) {
        // FK (K a multiple of KT): every chunk is in range, no guards
#pragma unroll
        for (int i = 0; i < CA; ++i) {
            const int cidx = tid + i * NT;
            const int kq = kt * KQ + ((cidx >> 5) % KQ);
            ra[i] = (FK || kq < kq_total) ? *(const float4*)(Asrc[i] + (size_t)kq * 128) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int i = 0; i < CW; ++i) {
            const int kq = kt * KQ + (((tid + i * NT) >> 5) % KQ);
            rw[i] = (FK || kq < kq_total) ? *(const float4*)(Wsrc[i] + (size_t)kt * KQ * 128) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    auto stage_store = [&](int buf, const float4 (&ra)[CA], const float4 (&rw)[CW]) {
        float* sA = smem + buf * BUF;
        float* sW = sA + SA;
#pragma unroll
        for (int i = 0; i < CA; ++i) *(float4*)(sA + (tid + i * NT) * 4) = ra[i];
#pragma unroll
        for (int i = 0; i < CW; ++i) *(float4*)(sW + (tid + i * NT) * 4) = rw[i];
    };

    floatx16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

    // Three LDS stage buffers: while the MFMAs of stage st run, the fragments of stage st+1 (complete since
    // the previous barrier) are already being read into registers and stage st+2 is in flight from global
    // memory; it lands in the buffer stage st-1 used. One barrier per stage, and no MFMA ever waits on an
    // LDS read issued after a barrier. A partial last K tile is zero-filled, so every stage runs all KT/8
    // fragment groups (adding exact zero products).
    constexpr int NG = KT / 8;
    float4 fa0[NG][TM], fb0[NG][TN], fa1[NG][TM], fb1[NG][TN];
    auto frag_load = [&](int buf, float4 (&fa)[NG][TM], float4 (&fb)[NG][TN]) {
        const float* sA = smem + buf * BUF;
        const float* sW = sA + SA;
#pragma unroll
        for (int g = 0; g < NG; ++g) {
#pragma unroll
            for (int i = 0; i < TM; ++i) fa[g][i] = *(const float4*)(sA + (((wm * TM + i) * KQ + 2 * g + h) * 32 + r) * 4);
#pragma unroll
            for (int j = 0; j < TN; ++j) fb[g][j] = *(const float4*)(sW + (((wn * TN + j) * KQ + 2 * g + h) * 32 + r) * 4);
        }
    };
    auto mfma_stage = [&](const float4 (&fa)[NG][TM], const float4 (&fb)[NG][TN]) {
#pragma unroll
        for (int g = 0; g < NG; ++g)
#pragma unroll
            for (int kk = 0; kk < 4; ++kk)
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(f4c(fb[g][j], kk), f4c(fa[g][i], kk), acc[i][j], 0, 0, 0);
    };
    // Global loads run two stages ahead of their LDS store: stage st+3 is requested during stage st into one
    // register set while the other set (stage st+2, requested a stage earlier) is written to LDS at its end,
    // so each load has ~2 stages (~4 us) to arrive from HBM.
    const int nst = (args.K + KT - 1) / KT;
    float4 ra0[CA], rw0[CW], ra1[CA], rw1[CW];
    stage_load(0, ra0, rw0);
    if (nst > 1) stage_load(1, ra1, rw1);
    stage_store(0, ra0, rw0);
    if (nst > 1) stage_store(1, ra1, rw1);
    if (nst > 2) stage_load(2, ra0, rw0);
    __syncthreads();
#ifdef TDMPC_STAMPS
    STAMP(1);
#endif
    frag_load(0, fa0, fb0);
    // drain the LDS counter here: otherwise the loop header merges these reads' pending state and the
    // waitcnt pass makes the first MFMAs of every iteration wait on the next stage's fragment reads
    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0), vmcnt/expcnt unconstrained
    int bnext = 1, bfill = 2;   // buffers of stages st+1 and st+2
    auto iter = [&](int st, const float4 (&fac)[NG][TM], const float4 (&fbc)[NG][TN], float4 (&fan)[NG][TM],
                    float4 (&fbn)[NG][TN], float4 (&ral)[CA], float4 (&rwl)[CW], const float4 (&ras)[CA],
                    const float4 (&rws)[CW]) {
        // unconditional (past the end: the last stage again, never stored) so that the vmcnt wait before
        // the store below can leave exactly this stage's loads in flight
        stage_load(min(st + 3, nst - 1), ral, rwl);
        if (st + 1 < nst) frag_load(bnext, fan, fbn);
        mfma_stage(fac, fbc);
        if (st + 2 < nst) stage_store(bfill, ras, rws);
        __syncthreads();
        bnext = bfill;
        bfill = bfill == 2 ? 0 : bfill + 1;
    };
    int st = 0;
    for (; st + 1 < nst; st += 2) {
        iter(st, fa0, fb0, fa1, fb1, ra1, rw1, ra0, rw0);
        iter(st + 1, fa1, fb1, fa0, fb0, ra0, rw0, ra1, rw1);
    }
    if (st < nst) iter(st, fa0, fb0, fa1, fb1, ra1, rw1, ra0, rw0);
#ifdef TDMPC_STAMPS
    STAMP(2);
#endif
    // Register epilogue. The MFMA operands are swapped (W fragment first), so acc[i][j] holds the transposed
    // 32x32 block: lane (r, h) owns activation row (wm*TM + i)*32 + r and, for q = 0..3, the four consecutive
    // output columns (wn*TN + j)*32 + 8q + 4h + 0..3 -- one float4 panel quad per q, and 32 lanes store one
    // quad of 32 consecutive rows = 512 contiguous bytes. Row reductions (reward-head dot, LayerNorm moments)
    // meet the other half-wave through a lane swap and the other 32-column block through LDS.
#ifdef TDMPC_STAMPS
    STAMP(3);
#endif
    {
        const int cq0 = n0 >> 2;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const int lrow = (wm * TM + i) * 32 + r;
            const int lm = m0 + lrow;
            const bool rval = lm < args.M;
            const int crow = rval ? (args.c_mapped ? map_row(args.cmap, lm) : lm) : 0;
            float* Cbase = P.C.p ? P.C.p + (size_t)(crow >> 5) * P.C.ts + (crow & 31) * 4 : nullptr;
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int cb = (wn * TN + j) * 32;        // column block within the tile
                float v[16];
                float s1 = 0.f;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int c = cb + 8 * q + 4 * h;
                    const float4 bb = *(const float4*)(sbias + c);
                    float o[4] = {acc[i][j][4 * q] + bb.x, acc[i][j][4 * q + 1] + bb.y, acc[i][j][4 * q + 2] + bb.z,
                                  acc[i][j][4 * q + 3] + bb.w};
                    if (epi == EPI_ELU || epi == EPI_ELU_DOT) {
#pragma unroll
                        for (int k = 0; k < 4; ++k) o[k] = elu_f(o[k]);
                    }
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        if (n0 + c + k >= P.nvalid) o[k] = 0.f;
                        v[4 * q + k] = o[k];
                    }
                    if (rval && n0 + c < P.nstore)
                        *(float4*)(Cbase + (size_t)(P.C.q0 + cq0 + (c >> 2)) * 128) = make_float4(o[0], o[1], o[2], o[3]);
                    if (epi == EPI_ELU_DOT) {
                        const float4 w4 = *(const float4*)(sdotw + c);
                        s1 += (o[0] * w4.x + o[1] * w4.y) + (o[2] * w4.z + o[3] * w4.w);
                    } else if (epi == EPI_LNSTATS) {
                        s1 += (o[0] + o[1]) + (o[2] + o[3]);
                    }
                }
                if (epi == EPI_ELU_DOT) {
                    const float tot = s1 + __shfl_xor(s1, 32);
                    if (h == 0) spart[lrow * (C / 32) + (wn * TN + j)] = make_float2(tot, 0.f);
                } else if (epi == EPI_LNSTATS) {
                    // (mean, M2) of the 32 columns of this block
                    const float mean = (s1 + __shfl_xor(s1, 32)) * (1.f / 32.f);
                    float m2 = 0.f;
#pragma unroll
                    for (int k = 0; k < 16; ++k) {
                        const float d = v[k] - mean;
                        m2 += d * d;
                    }
                    m2 += __shfl_xor(m2, 32);
                    if (h == 0) spart[lrow * (C / 32) + (wn * TN + j)] = make_float2(mean, m2);
                }
            }
        }
        if (epi == EPI_ELU_DOT || epi == EPI_LNSTATS) {
            // pairs of 32-column blocks -> the per-64-column outputs (dot partials / Chan-combined moments)
            __syncthreads();
            for (int t = tid; t < R * (C / 64); t += NT) {
                const int row = t % R, b = t / R;
                const int lm = m0 + row;
                if (lm >= args.M) continue;
                const float2 x = spart[row * (C / 32) + 2 * b], y = spart[row * (C / 32) + 2 * b + 1];
                if (epi == EPI_ELU_DOT) {
                    P.dot_out[(size_t)lm * P.dot_ld + (n0 / 64) + b] = x.x + y.x;
                } else {
                    const float delta = y.x - x.x;
                    P.st_out[(size_t)lm * P.st_ld + (n0 / 64) + b] =
                        make_float2(x.x + 0.5f * delta, x.y + y.y + delta * delta * 16.f);
                }
            }
        }
    }
#ifdef TDMPC_STAMPS
    __syncthreads();
    STAMP(4);
    STAMP_RECORD();
#endif
}

// ------------------------------------------------------------------------------------------------ chain
// Row-block MLP chain: one workgroup carries 32 candidate rows through a whole TOLD head -- Linear(K1 -> M)
// + activation, Linear(M -> M) + activation and the head's last layer -- with the hidden activations held in
// LDS ([M/4][32][4], the panel layout of one 32-row block) and never written to HBM. 8 waves; in the two
// M-wide layers wave w owns output columns [w*32*TN, (w+1)*32*TN) and streams its own weight-panel columns
// from L2 straight into registers (a D-deep ring of 1 KiB wave loads; the 1-3 MB of a head's weights are
// read by every workgroup and stay L2-resident), while the A fragments -- the block's activations -- are
// conflict-free ds_read_b128 shared by all waves. Per FLOP this reads as many bytes as a 128x128-tiled GEMM
// (32 rows reuse each weight fragment), but a rollout step is one launch instead of three and the
// 2 x 16 MB of hidden activations per step never leave the CU.
//   CH_STEP  TOLD.next (tdmpc.py:34-37) + the return update (:88-90); blockIdx.y = 0 dynamics (z' into
//            X_{t+1}), 1 reward (reward-head dot, G += gamma^t r).
//   CH_PI    TOLD.pi + TruncatedNormal sample (tdmpc.py:39-45, helper.py:86-96) -> X_t action columns.
//   CH_Q     helper.q (helper.py:197-201): Linear, LayerNorm, Tanh, Linear, LayerNorm, ELU, Linear(M -> 1);
//            blockIdx.y = Q head; writes q_p per row (min, gamma^H and nan_to_num: qvalue()).
enum { CH_STEP = 0, CH_PI = 1, CH_Q = 2 };

struct ChainProb {
    const float* W1; const float* b1;    // panel [M][K1], bias [M]
    const float* W2; const float* b2;    // panel [M][M], bias [M]
    const float* g1; const float* be1; const float* g2; const float* be2;  // CH_Q LayerNorm affines [M]
    const float* w3v; const float* b3v;  // reward / Q last layer: dense [M] + bias [1]
    const unsigned short* X1; const unsigned short* X2;   // W1 / W2 in the x6 layout (chain_kernel<..., X6>)
};

struct ChainArgs {
    ChainProb p[2];
    int rows, M, K1, q1;                 // logical rows; hidden width; first-layer K and its X quad offset
    int k1_alg;                          // the first layer's real input width (L + A or L), for the profiler's FLOPs
    int rb;                              // row block: 32 (chain_kernel) or 16 (chain16_kernel)
    int nw;                              // waves per workgroup of chain_kernel: 8 or 16
    int hfl;                             // floats of the LDS activation block (max(K1, M) * rb, K1 to 16)
    int il;                              // (retired: 0, the problems along blockIdx.y)
    int x6;                              // chain_kernel<..., X6 = true>: fp32 products from split bf16
    RowMap amap;                         // logical row -> X row (input and output)
    const float* X; long x_ts;           // X_t panel (input)
    // last layer of dynamics / pi: panel [n3][M] + bias -> Xo quads [out_q0, out_q0 + nstore/4)
    const float* W3; const float* b3; int n3, nvalid, nstore;
    const unsigned short* X3;            // W3 in the x6 layout
    float* Xo; int out_q0;
    // CH_STEP reward: G update (EPI_LIN_Z of the layered path)
    float* G; float* rlast; float disc; int first, last;
    // CH_PI: TruncatedNormal noise
    const float* eps; int eps_G; long eps_env; long eps_off; float min_std, lo, hi; int A;
    float* mu_out;                       // CH_PI, non-null: tanh(mu) of row x also to mu_out[x * nstore + col]
    // CH_STEP at t = 0 (every row's latent is its env's z0): non-null, layer 1 runs over the first k1c columns only
    // and its bias is z0c[env][head] = b1 + W1[:, k1c:] X_0[k1c:] (z0c_kernel), env = logical row / z0_G
    const float* z0c; int z0_G, k1c;
    // CH_Q: q_p of row x at q[p * q_ld + x]
    float* q; int q_ld;
    // CH_STEP (chain_kernel, latent_dim == mlp_dim): store h2 = ELU(W2 h1 + b2) into Xo's latent columns instead of
    // running layer 3 -- the next step / the terminal heads read it through folded first layers (Layout::fold)
    int outh;
};

// Weight ring: D k groups x TN 1-KiB wave loads of the weight panel in flight. ring_fill issues the first D
// groups (callers issue it early: before the input staging or the previous layer's epilogue, so that the
// ~1 us L2 latency under load hides behind that work); ring_run then walks groups [g0, g1):
// acc[j] += W(block j) . A, A from the LDS block [K/4][32][4] one group ahead, W refilled D groups ahead.
// Wp is the wave's first weight-panel block, already offset by the lane's (h, r); blocks wbs floats apart.
template <int TN, int D>
DEVI void ring_fill(float4 (&wr)[D][TN], const float* Wp, long wbs, int g0, int g1) {
    const int gl = g1 - 1;
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
        for (int j = 0; j < TN; ++j) wr[d][j] = *(const float4*)(Wp + j * wbs + (size_t)min(g0 + d, gl) * 256);
}

template <int TN, int D>
DEVI void ring_run(floatx16 (&acc)[TN], float4 (&wr)[D][TN], const float* sA, const float* Wp, long wbs, int g0,
                   int g1, int r, int h) {
    // Every refill is issued unconditionally (past the end: the last group again, never used) so that the
    // number of loads in flight is the same at every MFMA and the wait before group g's MFMAs is
    // vmcnt((D-1)*TN), not a drain.
    const int gl = g1 - 1;
    const float* ap = sA + (h * 32 + r) * 4;
    float4 an = *(const float4*)(ap + (size_t)g0 * 256);
    int gb = g0;
    for (; gb + D <= g1; gb += D) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const int g = gb + d;
            const float4 av = an;
            an = *(const float4*)(ap + (size_t)min(g + 1, gl) * 256);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int kk = 0; kk < 4; ++kk)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(f4c(wr[d][j], kk), f4c(av, kk), acc[j], 0, 0, 0);
#pragma unroll
            for (int j = 0; j < TN; ++j) wr[d][j] = *(const float4*)(Wp + j * wbs + (size_t)min(g + D, gl) * 256);
            // keep each group's refill right behind its MFMAs (the scheduler would otherwise cluster the
            // chunk's loads at its end and shrink the prefetch distance to one group)
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    // tail (< D groups): their weights are already in the ring
#pragma unroll
    for (int d = 0; d < D - 1; ++d) {
        if (gb + d < g1) {
            const float4 av = an;
            an = *(const float4*)(ap + (size_t)min(gb + d + 1, gl) * 256);
#pragma unroll
            for (int kk = 0; kk < 4; ++kk)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(f4c(wr[d][j], kk), f4c(av, kk), acc[j], 0, 0, 0);
        }
    }
}

// ---- x6: fp32 products from a three-way bf16 split on v_mfma_f32_32x32x16_bf16 (16x the f32 MFMA rate). Each
// operand x = hi + mid + lo (bf16 each, the residuals exact in fp32); a product keeps the six terms down to
// 2^-16 relative (hi.hi, hi.mid, mid.hi, hi.lo, lo.hi, mid.mid), dropping mid.lo, lo.mid, lo.lo (<= 2^-24
// relative, the size of one fp32 rounding), and accumulates in fp32: the accuracy of an fp32 GEMM, at 6/16 of
// the f32 MFMA cycles. Weights come pre-split (Layout::x6, pack_fused_kernel); the activations stay fp32 in LDS
// and are split as they are read.
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
#ifndef X6_D3
#define X6_D3 2   // weight-ring depth of the x6 chain kernel's last layer (k groups of 16)
#endif
DEVI bf16x8_t as_bf16x8(const uint4& v) { return __builtin_bit_cast(bf16x8_t, v); }

// Weights (pack time, pack_fused_kernel): x = hi + mid + lo exactly, each part round-to-nearest (the smallest dropped
// terms). A finite weight beyond bf16's largest value (whose rounding would be inf) takes its truncated top half as hi,
// and a non-finite one passes through whole in hi (mid = lo = 0).
DEVI void split3(float x, __bf16& hi, __bf16& mid, __bf16& lo) {
    float h = (float)(__bf16)x;
    const bool xfin = __builtin_isfinite(x);
    if (!__builtin_isfinite(h)) h = xfin ? __uint_as_float(__float_as_uint(x) & 0xffff0000u) : x;
    hi = (__bf16)h;
    const float r1 = xfin ? __fsub_rn(x, h) : 0.f;
    mid = (__bf16)r1;
    lo = (__bf16)__fsub_rn(r1, (float)mid);
}

// Activations (in the hot loop, once per MFMA k group). Finite x: hi = the truncated top half of x (one AND; finite for
// every finite x, beyond bf16's largest value included), then mid / lo round-to-nearest: x = hi + mid + lo exactly (the
// residual keeps <= 16 significant bits). The dropped terms (w_mid x_lo + w_lo x_mid + w_lo x_lo) are <= 1.5 * 2^-23
// of |w x|, the size of an fp32 product rounding.
// Non-finite x (+-inf, NaN): only the w_hi.x_hi term sees it (`h`: x's own top half -- arithmetic NaNs keep their
// payload there); the w_mid.x_hi and w_lo.x_hi terms take `s` = 0 and mid = lo = 0, so the x6 product is w_hi * x:
// +-inf or NaN exactly where fp32's w * x is (w_hi is 0 only for w = 0, or |w| under bf16's smallest subnormal).
// With one hi operand for all three weight planes, an infinite activation met 0 * inf = NaN in every weight whose mid
// or lo part is zero, and a +inf hidden unit that fp32 carries to G = +FLT_MAX came out as G = 0
// (tests/test_gpu_configs.py::test_estimate_value_nonfinite, cases inf_hidden*). A non-finite WEIGHT is not handled
// (its w_hi.x_mid / w_hi.x_lo terms meet zero activation parts): planning weights are finite.
struct X6B {
    bf16x8_t h;   // hi of x (w_hi term)
    bf16x8_t s;   // hi of x, 0 where x is not finite (w_mid / w_lo terms)
    bf16x8_t m, l;
};
DEVI void split3_act(float x, __bf16& hi, __bf16& hs, __bf16& mid, __bf16& lo) {
    const uint32_t u = __float_as_uint(x);
    const float xs = __builtin_isfinite(x) ? x : 0.f;
    const uint32_t us = __float_as_uint(xs);
    const float h = __uint_as_float(us & 0xffff0000u);
    hi = __builtin_bit_cast(__bf16, (unsigned short)(u >> 16));
    hs = __builtin_bit_cast(__bf16, (unsigned short)(us >> 16));
    const float r1 = __fsub_rn(xs, h);
    mid = (__bf16)r1;
    lo = (__bf16)__fsub_rn(r1, (float)mid);
}

DEVI X6B split8(const float4& a0, const float4& a1) {
    const float x[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
    X6B b;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        __bf16 h, hs, m, l;
        split3_act(x[e], h, hs, m, l);
        b.h[e] = h; b.s[e] = hs; b.m[e] = m; b.l[e] = l;
    }
    return b;
}

// The x6 B operand as dwords (two bf16 per dword, the fragment's k order), THREE planes: x = h + m + l for finite x
// (h its upper 16 bits, m = bf16(x - h), l = bf16(x - h - m)), and h = m = 0, l = x (inf, or a quiet bf16 NaN) for
// non-finite x, so that of the six products only w_hi l = w_hi x carries it -- the fp32 product's inf / NaN, and
// nothing from the w_mid / w_lo terms (split3_act's separate finite-zeroed hi plane does the same with a fourth
// plane). Finite operands give the products of ws_x6 bit for bit. Built a PAIR of elements at a time and packed at
// once (an element-wise bf16 build keeps every half in a register of its own until the vector is assembled).
struct X6U { uint4 h, m, l; };
typedef float w2f2 __attribute__((ext_vector_type(2)));
typedef __bf16 w2b2 __attribute__((ext_vector_type(2)));
DEVI unsigned w2_pk(float a, float b) {   // round-to-nearest-even bf16 pair {a, b}
    return __builtin_bit_cast(unsigned, __builtin_convertvector((w2f2){a, b}, w2b2));
}
DEVI void w2_split_pair(X6U& b, int d, float x0, float x1) {
    const bool f0 = __builtin_isfinite(x0), f1 = __builtin_isfinite(x1);
    const unsigned us0 = f0 ? __float_as_uint(x0) : 0u, us1 = f1 ? __float_as_uint(x1) : 0u;
    const unsigned h = __builtin_amdgcn_perm(us1, us0, 0x07060302u);
    const float r0 = __fsub_rn(__uint_as_float(us0), __uint_as_float(us0 & 0xffff0000u));
    const float r1 = __fsub_rn(__uint_as_float(us1), __uint_as_float(us1 & 0xffff0000u));
    const unsigned m = w2_pk(r0, r1);
    unsigned l = w2_pk(__fsub_rn(r0, __uint_as_float(m << 16)), __fsub_rn(r1, __uint_as_float(m & 0xffff0000u)));
    if (!f0) l = (l & 0xffff0000u) | (x0 != x0 ? 0x7fc0u : __float_as_uint(x0) >> 16);
    if (!f1) l = (l & 0x0000ffffu) | (x1 != x1 ? 0x7fc00000u : __float_as_uint(x1) & 0xffff0000u);
    if (d == 0) { b.h.x = h; b.m.x = m; b.l.x = l; }
    else if (d == 1) { b.h.y = h; b.m.y = m; b.l.y = l; }
    else if (d == 2) { b.h.z = h; b.m.z = m; b.l.z = l; }
    else { b.h.w = h; b.m.w = m; b.l.w = l; }
}
DEVI X6U w2_split8(const float4& a0, const float4& a1) {
    X6U b;
    w2_split_pair(b, 0, a0.x, a0.y);
    w2_split_pair(b, 1, a0.z, a0.w);
    w2_split_pair(b, 2, a1.x, a1.y);
    w2_split_pair(b, 3, a1.z, a1.w);
    return b;
}
// w2_split_pair for operands known finite (the caller checked the whole wave's values): 48 instead of 106 VALU per
// eight elements (split8's four-plane form: 74)
DEVI void w2_split_pair_fin(X6U& b, int d, float x0, float x1) {
    const unsigned us0 = __float_as_uint(x0), us1 = __float_as_uint(x1);
    const unsigned h = __builtin_amdgcn_perm(us1, us0, 0x07060302u);
    const float r0 = __fsub_rn(x0, __uint_as_float(us0 & 0xffff0000u));
    const float r1 = __fsub_rn(x1, __uint_as_float(us1 & 0xffff0000u));
    const unsigned m = w2_pk(r0, r1);
    const unsigned l = w2_pk(__fsub_rn(r0, __uint_as_float(m << 16)), __fsub_rn(r1, __uint_as_float(m & 0xffff0000u)));
    if (d == 0) { b.h.x = h; b.m.x = m; b.l.x = l; }
    else if (d == 1) { b.h.y = h; b.m.y = m; b.l.y = l; }
    else if (d == 2) { b.h.z = h; b.m.z = m; b.l.z = l; }
    else { b.h.w = h; b.m.w = m; b.l.w = l; }
}
// true when a value every lane of the wave computed is finite (a sum of a lane's elements is non-finite when one of
// them is; an overflowing sum only sends the wave down the general path)
DEVI bool ws_wave_finite(float s) { return __builtin_amdgcn_ballot_w64(!__builtin_isfinite(s)) == 0; }
DEVI float ws_sum8(const float4& a0, const float4& a1) {
    return ((a0.x + a0.y) + (a0.z + a0.w)) + ((a1.x + a1.y) + (a1.z + a1.w));
}
// The activation operand in three planes for finite values (the wave-uniform fast path of the chain and wide
// kernels' splits; x6_group / x6_group16 and ws_opnd)
DEVI X6U w2_split8_fin(const float4& a0, const float4& a1) {
    X6U b;
    w2_split_pair_fin(b, 0, a0.x, a0.y);
    w2_split_pair_fin(b, 1, a0.z, a0.w);
    w2_split_pair_fin(b, 2, a1.x, a1.y);
    w2_split_pair_fin(b, 3, a1.z, a1.w);
    return b;
}

// Weight ring of the x6 form: D k groups (16 k each) x TN blocks x 3 planes of 1 KiB wave loads. Wp is the wave's
// first block already offset by the lane (lane * 8 bf16); blocks wbs bf16 apart.
template <int TN, int D>
DEVI void ring6_fill(uint4 (&wr)[D][TN][3], const unsigned short* Wp, long wbs, int g0, int g1) {
    const int gl = g1 - 1;
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int p = 0; p < 3; ++p)
                wr[d][j][p] = *(const uint4*)(Wp + j * wbs + ((size_t)min(g0 + d, gl) * 3 + p) * 512);
}

DEVI X6B ch_split(const float4& a0, const float4& a1) { return split8(a0, a1); }

template <int TN>
DEVI void x6_group(floatx16 (&acc)[TN], const uint4 (&w)[TN][3], const float4& a0, const float4& a1) {
    const auto b = ch_split(a0, a1);
    // small terms first, the hi.hi term last
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(w[j][1]), b.m, acc[j], 0, 0, 0);
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(w[j][2]), b.s, acc[j], 0, 0, 0);
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(w[j][0]), b.l, acc[j], 0, 0, 0);
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(w[j][1]), b.s, acc[j], 0, 0, 0);
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(w[j][0]), b.m, acc[j], 0, 0, 0);
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(w[j][0]), b.h, acc[j], 0, 0, 0);
}

// acc[j] += W(block j) . A over k groups [g0, g1); A from the fp32 LDS block [K/4][32][4] (quads 4g + h and
// 4g + 2 + h of row r: the x6 k order), one group ahead; W refilled D groups ahead, as ring_run.
template <int TN, int D>
DEVI void ring6_run(floatx16 (&acc)[TN], uint4 (&wr)[D][TN][3], const float* sA, const unsigned short* Wp, long wbs,
                    int g0, int g1, int r, int h) {
    const int gl = g1 - 1;
    const float* ap = sA + (h * 32 + r) * 4;
    float4 n0 = *(const float4*)(ap + (size_t)g0 * 512), n1 = *(const float4*)(ap + (size_t)g0 * 512 + 256);
    int gb = g0;
    for (; gb + D <= g1; gb += D) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const int g = gb + d;
            const float4 a0 = n0, a1 = n1;
            const size_t gn = (size_t)min(g + 1, gl) * 512;
            n0 = *(const float4*)(ap + gn);
            n1 = *(const float4*)(ap + gn + 256);
#ifndef TDMPC_X6_FREE_SCHED
            __builtin_amdgcn_sched_barrier(0);
#endif
            x6_group<TN>(acc, wr[d], a0, a1);
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int p = 0; p < 3; ++p)
                    wr[d][j][p] = *(const uint4*)(Wp + j * wbs + ((size_t)min(g + D, gl) * 3 + p) * 512);
#ifndef TDMPC_X6_FREE_SCHED
            __builtin_amdgcn_sched_barrier(0);
#endif
        }
    }
#pragma unroll
    for (int d = 0; d < D - 1; ++d) {
        if (gb + d < g1) {
            const float4 a0 = n0, a1 = n1;
            const size_t gn = (size_t)min(gb + d + 1, gl) * 512;
            n0 = *(const float4*)(ap + gn);
            n1 = *(const float4*)(ap + gn + 256);
            x6_group<TN>(acc, wr[d], a0, a1);
        }
    }
}

// Workgroup barrier for the chain kernels' LDS hand-offs: waits for this wave's LDS traffic only. HIP's
// __syncthreads() carries a fence that drains vmcnt, i.e. it also waits for every global load in flight (the next
// layer's weight ring prefetched before the epilogue, the ring's tail refills). No chain-kernel barrier orders
// global memory between waves. Measured neutral on MI355X (stamps, round-1 run: the layer-boundary cost is
// the MFMA pipe draining before each epilogue, not the load wait), kept as the precise primitive.
DEVI void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Row mean and 1/sqrt(var + 1e-5) over the M columns of the block's rows (biased variance, two passes),
// from each lane's TN*16 values of row r: per-wave partials through red0 / red1 ([NW][32] each).
template <int TN, int NW>
DEVI void chain_row_moments(const float (&v)[TN * 16], float* red0, float* red1, int wave, int r, int h, int M,
                            float& mean, float& rstd) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < TN * 16; ++i) s += v[i];
    s += __shfl_xor(s, 32);
    if (h == 0) red0[wave * 32 + r] = s;
    lds_barrier();
    float tot = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) tot += red0[w * 32 + r];
    mean = tot / (float)M;
    float m2 = 0.f;
#pragma unroll
    for (int i = 0; i < TN * 16; ++i) {
        const float d = v[i] - mean;
        m2 += d * d;
    }
    m2 += __shfl_xor(m2, 32);
    if (h == 0) red1[wave * 32 + r] = m2;
    lds_barrier();
    float tot2 = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) tot2 += red1[w * 32 + r];
    rstd = 1.0f / sqrtf(fmaxf(tot2 / (float)M, 0.f) + 1e-5f);
}

// LDS floats of the chain kernel's per-head parameter vectors (after the activation block and red0/red1).
__host__ __device__ inline int chain_param_floats(int mode, int M, int n3) {
    return mode == CH_Q ? 7 * M : 3 * M + n3;
}

// bias (+ LayerNorm affine + activation) of a layer's register tile, in place: v = act(acc + b)
template <int TN>
DEVI void chain_bias(float (&v)[TN * 16], const floatx16 (&acc)[TN], const float* sb, int cw0, int h) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float4 bb = *(const float4*)(sb + (cw0 + j) * 32 + 8 * q + 4 * h);
            v[j * 16 + 4 * q + 0] = acc[j][4 * q + 0] + bb.x;
            v[j * 16 + 4 * q + 1] = acc[j][4 * q + 1] + bb.y;
            v[j * 16 + 4 * q + 2] = acc[j][4 * q + 2] + bb.z;
            v[j * 16 + 4 * q + 3] = acc[j][4 * q + 3] + bb.w;
        }
}

// ATen LayerNorm on the tile: (x * rstd + (-rstd * mean)) * gamma + beta
template <int TN>
DEVI void chain_ln(float (&v)[TN * 16], float rs, float sh, const float* sg, const float* sbe, int cw0, int h) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int c = (cw0 + j) * 32 + 8 * q + 4 * h;
            const float4 gg = *(const float4*)(sg + c), bb = *(const float4*)(sbe + c);
            float* x = v + j * 16 + 4 * q;
            x[0] = fadd(fmul(fadd(fmul(x[0], rs), sh), gg.x), bb.x);
            x[1] = fadd(fmul(fadd(fmul(x[1], rs), sh), gg.y), bb.y);
            x[2] = fadd(fmul(fadd(fmul(x[2], rs), sh), gg.z), bb.z);
            x[3] = fadd(fmul(fadd(fmul(x[3], rs), sh), gg.w), bb.w);
        }
}

// the tile into the activation block (panel quads; lanes of one quad write 512 contiguous bytes)
template <int TN>
DEVI void chain_store_lds(float* sH, const float (&v)[TN * 16], int cw0, int r, int h) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int cq = (cw0 + j) * 8 + 2 * q + h;
            *(float4*)(sH + (cq * 32 + r) * 4) =
                make_float4(v[j * 16 + 4 * q], v[j * 16 + 4 * q + 1], v[j * 16 + 4 * q + 2], v[j * 16 + 4 * q + 3]);
        }
}

// NW = 8 or 16 waves per workgroup (16: 4 waves per SIMD on one 32-row block, TN = M / 512).
// X6: 0 = f32 MFMA; 1 = x6 with the activations kept fp32 in LDS and split as read (a split-planes form in LDS
// measured 2-3 % slower and was retired in round 3).
template <int MODE, int TN, int NW = 8, int D = 4, int D3 = 8, int X6 = 0>
__global__ void __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(X6 == 1 && NW == 8 ? 4 : X6 == 1 && NW == 4 ? 2 : 1))) chain_kernel(const ChainArgs a) {
    constexpr int NTH = 64 * NW;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 31, h = lane >> 5;
    // il > 0: heads interleaved along x; il < 0: XCD-grouped heads (blocks b, b + 8, ... share an XCD: dispatch
    // groups 0-3 run head 0, 4-7 head 1, so each XCD's L2 holds one head's weights); else head = blockIdx.y
    const int bx = blockIdx.x;
    const int pb = blockIdx.y;
    const ChainProb& P = a.p[pb];
    const int M = a.M;
    const int m0 = bx * 32;
    if (m0 >= a.rows) return;   // (XCD-grouped grids are padded to a multiple of 4 blocks per head)
    float* sH = smem;                       // activation block [max(K1, M)/4][32][4]
    float* red0 = smem + a.hfl;             // [NW][32]
    float* red1 = red0 + 32 * NW;           // [NW][32]
    float* sp = red1 + 32 * NW;                // parameter vectors (chain_param_floats)
    float* sb1 = sp;
    float* sb2 = sp + M;
    float* sw3 = sp + 2 * M;                // reward / Q head weights
    float* sb3 = sp + 3 * M;                // dynamics / pi last-layer bias [n3]
    float* sg1 = sp + 3 * M;                // CH_Q LayerNorm affines
    float* sbe1 = sp + 4 * M;
    float* sg2 = sp + 5 * M;
    float* sbe2 = sp + 6 * M;
    const int lo = h * 128 + r * 4;         // lane offset inside a weight-panel k group
    // x6: k groups of 16, blocks of 32 rows x K16 x 3 planes (bf16 elements)
    const int g1n = X6 ? (int)(rup(a.K1, 16) >> 4) : a.K1 >> 3, g2n = X6 ? M >> 4 : M >> 3;
    const long wb1 = (long)g1n * 1536, wb2 = (long)g2n * 1536;
    // layer-1 k groups run here: all, or with z0c only the first k1c columns (the rest is in the per-env bias)
    const bool zc = MODE == CH_STEP && a.z0c != nullptr;
    const int g1e = zc ? (X6 ? a.k1c >> 4 : a.k1c >> 3) : g1n;
    const int cw0 = wave * TN;              // first 32-column block of this wave in the M-wide layers
    const bool head_dot = MODE == CH_Q || (MODE == CH_STEP && pb == 1);
#ifdef TDMPC_STAMPS
    unsigned long long st_[5];
    const unsigned long long rt0_ = __builtin_amdgcn_s_memrealtime();
    STAMP(0);
#endif

    // ---- layer-1 weights in flight first, then the block's input rows (X quads [q1, q1 + K1/4); 32
    // consecutive lanes = 32 rows of one quad) and the parameter vectors
    float4 wr[X6 ? 1 : D][TN];
    uint4 wx[X6 ? D : 1][TN][3];
    if constexpr (X6) ring6_fill<TN, D>(wx, P.X1 + (size_t)cw0 * wb1 + lane * 8, wb1, 0, g1e);
    else ring_fill<TN, D>(wr, P.W1 + (size_t)cw0 * a.K1 * 32 + lo, (long)a.K1 * 32, 0, g1e);
    // (x6: K1 rounded to 16 with zero quads)
    const int q1n = zc ? a.k1c >> 2 : X6 ? g1n * 4 : a.K1 >> 2;
    for (int i = tid; i < q1n * 32; i += NTH) {
        const int row = i & 31, q = i >> 5;
        const int lm = m0 + row;
        const int xr = map_row(a.amap, lm < a.rows ? lm : 0);
        const float4 x = q < (a.K1 >> 2)
            ? *(const float4*)(a.X + (size_t)(xr >> 5) * a.x_ts + (size_t)(a.q1 + q) * 128 + (xr & 31) * 4)
            : make_float4(0.f, 0.f, 0.f, 0.f);
        ((float4*)sH)[i] = x;
    }
    const float* b1src = zc ? a.z0c + ((size_t)(m0 / a.z0_G) * 2 + pb) * M : P.b1;
    for (int i = tid; i < M / 4; i += NTH) {
        ((float4*)sb1)[i] = ((const float4*)b1src)[i];
        ((float4*)sb2)[i] = ((const float4*)P.b2)[i];
        if (head_dot) ((float4*)sw3)[i] = ((const float4*)P.w3v)[i];
        if (MODE == CH_Q) {
            ((float4*)sg1)[i] = ((const float4*)P.g1)[i];
            ((float4*)sbe1)[i] = ((const float4*)P.be1)[i];
            ((float4*)sg2)[i] = ((const float4*)P.g2)[i];
            ((float4*)sbe2)[i] = ((const float4*)P.be2)[i];
        }
    }
    if (!head_dot)
        for (int i = tid; i < a.n3 / 4; i += NTH) ((float4*)sb3)[i] = ((const float4*)a.b3)[i];
    // early operands of the last stage: the running return (reward WG) / the policy noise (pi)
    float g_old = 0.f;
    if (MODE == CH_STEP && pb == 1 && tid < 32 && !a.first && m0 + tid < a.rows)
        g_old = a.G[map_row(a.amap, m0 + tid)];
    // (one output quad per thread and pass: NIT passes cover nstore/4 * 32 <= 512 quads)
    constexpr int NIT = NTH >= 512 ? 1 : 512 / NTH;
    float eps4[NIT][4];
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
#pragma unroll
        for (int k = 0; k < 4; ++k) eps4[it][k] = 0.f;
        const int iq = tid + it * NTH;
        if (MODE == CH_PI && iq < (a.nstore >> 2) * 32 && m0 + (iq & 31) < a.rows) {
            const int lm = m0 + (iq & 31), c = 4 * (iq >> 5);
            const int e = lm / a.eps_G, rr = lm % a.eps_G;
            const float* ep = a.eps + (size_t)e * a.eps_env + a.eps_off + (size_t)rr * a.A;
#pragma unroll
            for (int k = 0; k < 4; ++k) eps4[it][k] = c + k < a.nvalid ? ep[c + k] : 0.f;
        }
    }
    lds_barrier();
#if defined(TDMPC_STAMPS) && defined(TDMPC_STAMPS_STAGE)
    STAMP(1);   // diagnostic variant: phase 0 = staging only, phase 1 = layer 1 + its epilogue
#endif

    // ---- layer 1: [32 x K1] . W1^T -> [32 x M]
    floatx16 acc[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[j][e] = 0.f;
    if constexpr (X6 == 1) ring6_run<TN, D>(acc, wx, sH, P.X1 + (size_t)cw0 * wb1 + lane * 8, wb1, 0, g1e, r, h);
    else ring_run<TN, D>(acc, wr, sH, P.W1 + (size_t)cw0 * a.K1 * 32 + lo, (long)a.K1 * 32, 0, g1e, r, h);
    // layer-2 weights in flight during the epilogue
    if constexpr (X6) ring6_fill<TN, D>(wx, P.X2 + (size_t)cw0 * wb2 + lane * 8, wb2, 0, g2n);
    else ring_fill<TN, D>(wr, P.W2 + (size_t)cw0 * M * 32 + lo, (long)M * 32, 0, M >> 3);
    lds_barrier();   // every wave is done with the input tile: sH becomes h1
#if defined(TDMPC_STAMPS) && !defined(TDMPC_STAMPS_STAGE)
    STAMP(1);
#endif
    {
        float v[TN * 16];
        chain_bias<TN>(v, acc, sb1, cw0, h);
        if (MODE == CH_Q) {
            float mean, rs;
            chain_row_moments<TN, NW>(v, red0, red1, wave, r, h, M, mean, rs);
            chain_ln<TN>(v, rs, -rs * mean, sg1, sbe1, cw0, h);
#pragma unroll
            for (int i = 0; i < TN * 16; ++i) v[i] = tanh_f(v[i]);
        } else {
#pragma unroll
            for (int i = 0; i < TN * 16; ++i) v[i] = elu_f(v[i]);
        }
        chain_store_lds<TN>(sH, v, cw0, r, h);
    }
    lds_barrier();
#ifdef TDMPC_STAMPS
    STAMP(2);
#endif

    // ---- layer 2: [32 x M] . W2^T -> [32 x M]
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[j][e] = 0.f;
    if constexpr (X6 == 1) ring6_run<TN, D>(acc, wx, sH, P.X2 + (size_t)cw0 * wb2 + lane * 8, wb2, 0, g2n, r, h);
    else ring_run<TN, D>(acc, wr, sH, P.W2 + (size_t)cw0 * M * 32 + lo, (long)M * 32, 0, M >> 3, r, h);
#ifdef TDMPC_STAMPS
    STAMP(3);
#endif
    // layer-3 work items (32-column block, K part): narrow heads split K over all NW waves
    const int nb3 = a.n3 >> 5;
    const int ks = nb3 >= NW ? 1 : NW / nb3;
    const int items = nb3 * ks;
    const int gper = g2n / ks;
    float4 w3r[X6 ? 1 : D3][1];
    uint4 w3x[X6 ? D3 : 1][1][3];
    if (!head_dot && wave < items) {
        if constexpr (X6)
            ring6_fill<1, D3>(w3x, a.X3 + (size_t)(wave / ks) * wb2 + lane * 8, wb2, (wave % ks) * gper,
                              (wave % ks + 1) * gper);
        else
            ring_fill<1, D3>(w3r, a.W3 + (size_t)(wave / ks) * M * 32 + lo, (long)M * 32, (wave % ks) * gper,
                             (wave % ks + 1) * gper);
    }
    float v[TN * 16];
    chain_bias<TN>(v, acc, sb2, cw0, h);
    if (head_dot) {
        // reward / Q last layer Linear(M -> 1) on the row: per-wave partial dots, then one lane per row
        if (MODE == CH_Q) {
            float mean, rs;
            chain_row_moments<TN, NW>(v, red0, red1, wave, r, h, M, mean, rs);
            chain_ln<TN>(v, rs, -rs * mean, sg2, sbe2, cw0, h);
        }
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float4 w4 = *(const float4*)(sw3 + (cw0 + j) * 32 + 8 * q + 4 * h);
                const float* x = v + j * 16 + 4 * q;
                s += (elu_f(x[0]) * w4.x + elu_f(x[1]) * w4.y) + (elu_f(x[2]) * w4.z + elu_f(x[3]) * w4.w);
            }
        s += __shfl_xor(s, 32);
        if (h == 0) red0[wave * 32 + r] = s;
        lds_barrier();
        if (tid < 32) {
            const int lm = m0 + tid;
            if (lm < a.rows) {
                const int xr = map_row(a.amap, lm);
                float tot = 0.f;
#pragma unroll
                for (int w = 0; w < NW; ++w) tot += red0[w * 32 + tid];
                const float o = tot + P.b3v[0];
                if (MODE == CH_Q) {
                    a.q[(size_t)pb * a.q_ld + xr] = o;
                } else {
                    // G += discount * reward (tdmpc.py:89), float32(discount) like ATen's scalar mul
                    const float dr = fmul(a.disc, o);
                    a.G[xr] = a.first ? dr : fadd(g_old, dr);
                    if (a.last) a.rlast[xr] = o;
                }
            }
        }
#ifdef TDMPC_STAMPS
        lds_barrier();
        STAMP(4);
        STAMP_RECORD();
#endif
        return;
    }
    // dynamics / pi: h2 = ELU(y2) back into the activation block once every wave is done reading h1
#pragma unroll
    for (int i = 0; i < TN * 16; ++i) v[i] = elu_f(v[i]);
    lds_barrier();
    chain_store_lds<TN>(sH, v, cw0, r, h);
    lds_barrier();
    if (MODE == CH_STEP && a.outh) {
        // h2 where z' would go (M = Lp columns from quad out_q0): the folded first layers read it
        for (int i = tid; i < (M >> 2) * 32; i += NTH) {
            const int row = i & 31, cq = i >> 5, lm = m0 + row;
            if (lm >= a.rows) continue;
            const int xr = map_row(a.amap, lm);
            *(float4*)(a.Xo + (size_t)(xr >> 5) * a.x_ts + (size_t)(a.out_q0 + cq) * 128 + (xr & 31) * 4) =
                *(const float4*)(sH + (cq * 32 + row) * 4);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (the layer-3 weight prefetch, unused here)
        return;
    }

    // ---- layer 3: [32 x M] . W3^T -> [32 x n3]; partial tiles meet in the activation block after the reads
    floatx16 a3a[1], a3b[1];
#pragma unroll
    for (int e = 0; e < 16; ++e) { a3a[0][e] = 0.f; a3b[0][e] = 0.f; }
    if (wave < items) {
        const int blk = wave / ks, kp = wave % ks;
        if constexpr (X6 == 1)
            ring6_run<1, D3>(a3a, w3x, sH, a.X3 + (size_t)blk * wb2 + lane * 8, wb2, kp * gper, (kp + 1) * gper, r, h);
        else
            ring_run<1, D3>(a3a, w3r, sH, a.W3 + (size_t)blk * M * 32 + lo, (long)M * 32, kp * gper, (kp + 1) * gper, r, h);
    }
    if (wave + NW < items) {
        const int blk = (wave + NW) / ks, kp = (wave + NW) % ks;
        if constexpr (X6) {
            ring6_fill<1, D3>(w3x, a.X3 + (size_t)blk * wb2 + lane * 8, wb2, kp * gper, (kp + 1) * gper);
            ring6_run<1, D3>(a3b, w3x, sH, a.X3 + (size_t)blk * wb2 + lane * 8, wb2, kp * gper, (kp + 1) * gper, r, h);
        } else {
            ring_fill<1, D3>(w3r, a.W3 + (size_t)blk * M * 32 + lo, (long)M * 32, kp * gper, (kp + 1) * gper);
            ring_run<1, D3>(a3b, w3r, sH, a.W3 + (size_t)blk * M * 32 + lo, (long)M * 32, kp * gper, (kp + 1) * gper, r, h);
        }
    }
    // 4-wave x6 workgroups (mode 3) take up to four last-layer items per wave (L512: 16 blocks)
    constexpr bool IT4 = NW == 4 && X6 == 1;
    floatx16 a3c[1], a3d[1];
#pragma unroll
    for (int e = 0; e < 16; ++e) { a3c[0][e] = 0.f; a3d[0][e] = 0.f; }
    if constexpr (IT4) {
        auto item = [&](floatx16 (&acc)[1], int it) {
            const int blk = it / ks, kp = it % ks;
            ring6_fill<1, D3>(w3x, a.X3 + (size_t)blk * wb2 + lane * 8, wb2, kp * gper, (kp + 1) * gper);
            ring6_run<1, D3>(acc, w3x, sH, a.X3 + (size_t)blk * wb2 + lane * 8, wb2, kp * gper, (kp + 1) * gper, r, h);
        };
        if (wave + 2 * NW < items) item(a3c, wave + 2 * NW);
        if (wave + 3 * NW < items) item(a3d, wave + 3 * NW);
    }
    lds_barrier();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        if (wave < items)
            *(float4*)(sH + (size_t)wave * 1024 + ((2 * q + h) * 32 + r) * 4) =
                make_float4(a3a[0][4 * q], a3a[0][4 * q + 1], a3a[0][4 * q + 2], a3a[0][4 * q + 3]);
        if (wave + NW < items)
            *(float4*)(sH + (size_t)(wave + NW) * 1024 + ((2 * q + h) * 32 + r) * 4) =
                make_float4(a3b[0][4 * q], a3b[0][4 * q + 1], a3b[0][4 * q + 2], a3b[0][4 * q + 3]);
        if (IT4 && wave + 2 * NW < items)
            *(float4*)(sH + (size_t)(wave + 2 * NW) * 1024 + ((2 * q + h) * 32 + r) * 4) =
                make_float4(a3c[0][4 * q], a3c[0][4 * q + 1], a3c[0][4 * q + 2], a3c[0][4 * q + 3]);
        if (IT4 && wave + 3 * NW < items)
            *(float4*)(sH + (size_t)(wave + 3 * NW) * 1024 + ((2 * q + h) * 32 + r) * 4) =
                make_float4(a3d[0][4 * q], a3d[0][4 * q + 1], a3d[0][4 * q + 2], a3d[0][4 * q + 3]);
    }
    lds_barrier();
    for (int i = tid; i < (a.nstore >> 2) * 32; i += NTH) {
        const int row = i & 31, cq = i >> 5;
        const int lm = m0 + row;
        if (lm >= a.rows) continue;
        const int blk = cq >> 3, qi = cq & 7;
        float4 s = *(const float4*)(sH + (size_t)(blk * ks) * 1024 + (qi * 32 + row) * 4);
        for (int kp = 1; kp < ks; ++kp) {
            const float4 u = *(const float4*)(sH + (size_t)(blk * ks + kp) * 1024 + (qi * 32 + row) * 4);
            s.x += u.x; s.y += u.y; s.z += u.z; s.w += u.w;
        }
        const int c = 4 * cq;
        const float4 bb = *(const float4*)(sb3 + c);
        float o[4] = {s.x + bb.x, s.y + bb.y, s.z + bb.z, s.w + bb.w};
        const int xr = map_row(a.amap, lm);
        if (MODE == CH_PI) {
            // TOLD.pi + TruncatedNormal.sample(clip=0.3) (tdmpc.py:39-45, helper.py:86-96); this thread's noise
            // was loaded at kernel start (pass (i - tid) / NTH < NIT: nstore/4 * 32 <= 512 items)
            const bool second = NIT > 1 && i >= tid + NTH;
            float mu4[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                float x = 0.f;
                mu4[k] = 0.f;
                if (c + k < a.nvalid) {
                    const float muv = tanhf(o[k]);
                    x = muv;
                    mu4[k] = muv;
                    if (a.min_std > 0.f) {
                        const float ee = tclamp(fmul(second ? eps4[NIT - 1][k] : eps4[0][k], a.min_std), -0.3f, 0.3f);
                        x = tclamp(fadd(muv, ee), a.lo, a.hi);
                    }
                }
                o[k] = x;
            }
            if (a.mu_out) *(float4*)(a.mu_out + (size_t)xr * a.nstore + c) = make_float4(mu4[0], mu4[1], mu4[2], mu4[3]);
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (c + k >= a.nvalid) o[k] = 0.f;
        }
        *(float4*)(a.Xo + (size_t)(xr >> 5) * a.x_ts + (size_t)(a.out_q0 + cq) * 128 + (xr & 31) * 4) =
            make_float4(o[0], o[1], o[2], o[3]);
    }
#ifdef TDMPC_STAMPS
    lds_barrier();
    STAMP(4);
    STAMP_RECORD();
#endif
}

// ------------------------------------------------------------------------------------------------ chain16
// Row-block chain kernel on 16-row blocks (v_mfma_f32_16x16x4_f32), the same three modes as chain_kernel.
// Why a second block size: a 32-row chain launch of the B = 8 bench shape is exactly one workgroup per CU
// (2 waves per SIMD), which leaves every L2 fetch and layer epilogue exposed, and its 384-workgroup launches
// (6144 rows) take two rounds on half the chip. Halving the row block doubles the workgroups: two co-resident
// per CU (4 waves per SIMD, <= 128 VGPRs each), a dynamics and a reward workgroup side by side, so one's
// epilogue hides under the other's MFMAs. The cost is twice the L2 -> CU weight traffic per FLOP (each 1 KiB
// weight fragment now serves 16 rows): 32 B/clk/CU at the full MFMA rate, within the L1/L2 budget.
//
// Operand maps (swapped like chain_kernel: weights are the A operand, activations B, so the accumulator of
// lane l holds batch row m = l & 15 and output features 4 (l >> 4) + 0..3 of its 16-column tile):
//   k group g = 16 k values; lane l (m = l & 15, h4 = l >> 4) holds quad 4g + h4 of its row, element kk
//   feeding MFMA kk of the group (k = 16g + 4 h4 + kk, the same permutation for both operands).
//   weights: the 32-row panel [n/32][K/4][32][4] as is; tile of columns [n0, n0 + 16) at
//            (n0 >> 5) * K * 32 + (n0 & 31) * 4 + (l & 15) * 4 + (4g + h4) * 128
//   activations in LDS: [K/4][16][4]; lane l of group g at g * 256 + l * 4 (one conflict-free 1 KiB read).
typedef float floatx4 __attribute__((ext_vector_type(4)));

// Tile j of a wave's NT tiles: columns n0 + 16 j with n0 a multiple of 32, i.e. (j >> 1) blocks of the
// 32-row panel (bs floats each) plus 64 floats for an odd tile. Wp is already offset by the lane.
// A K that is not a multiple of 16 ends in a half group: its lanes h4 = 2, 3 clamp their quad to the last
// real one (qmax) and meet zero-filled activation quads, so they add exactly 0.
DEVI size_t wq16(int g, int gl, int h4, int qmax) { return (size_t)min(4 * min(g, gl) + h4, qmax) * 128; }

template <int NT, int D>
DEVI void ring16_fill(float4 (&wr)[D][NT], const float* Wp, long bs, int g0, int g1, int h4, int qmax) {
    const int gl = g1 - 1;
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
        for (int j = 0; j < NT; ++j)
            wr[d][j] = *(const float4*)(Wp + (j >> 1) * bs + (j & 1) * 64 + wq16(g0 + d, gl, h4, qmax));
}

template <int NT, int D>
DEVI void ring16_run(floatx4 (&acc)[NT], float4 (&wr)[D][NT], const float* sA, const float* Wp, long bs, int g0,
                     int g1, int lane, int qmax) {
    const int gl = g1 - 1, h4 = lane >> 4;
    const float* ap = sA + lane * 4;
    float4 an = *(const float4*)(ap + (size_t)g0 * 256);
    int gb = g0;
    for (; gb + D <= g1; gb += D) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const int g = gb + d;
            const float4 av = an;
            an = *(const float4*)(ap + (size_t)min(g + 1, gl) * 256);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int kk = 0; kk < 4; ++kk)
#pragma unroll
                for (int j = 0; j < NT; ++j)
                    acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(f4c(wr[d][j], kk), f4c(av, kk), acc[j], 0, 0, 0);
#pragma unroll
            for (int j = 0; j < NT; ++j)
                wr[d][j] = *(const float4*)(Wp + (j >> 1) * bs + (j & 1) * 64 + wq16(g + D, gl, h4, qmax));
            __builtin_amdgcn_sched_barrier(0);
        }
    }
#pragma unroll
    for (int d = 0; d < D - 1; ++d) {
        if (gb + d < g1) {
            const float4 av = an;
            an = *(const float4*)(ap + (size_t)min(gb + d + 1, gl) * 256);
#pragma unroll
            for (int kk = 0; kk < 4; ++kk)
#pragma unroll
                for (int j = 0; j < NT; ++j)
                    acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(f4c(wr[d][j], kk), f4c(av, kk), acc[j], 0, 0, 0);
        }
    }
}

// ---- x6 on 16-row blocks (v_mfma_f32_16x16x32_bf16), reusing the 32-row x6 weight layout: a 32-k group G of a
// 16-row tile is the two 16-k groups 2G, 2G + 1 of its 32-row block; lane l (m = l & 15, h4 = l >> 4) takes group
// 2G + (h4 >> 1) of slot (h4 & 1) * 32 + 16 * half + m, whose k order is quads 8G + 4 (h4 >> 1) + (h4 & 1) and that
// + 2 -- the activation quads the lane reads from the fp32 [K/4][16][4] LDS block. Groups past the matrix clamp to
// its last one and meet zero activation quads (the staging zero-fills to a multiple of 32 k).
// Tile j of a wave covers features nf0 + 16 j; Wb = the matrix's x6 base, gmax its 16-k groups.
template <int NT, int D>
DEVI void ring16x6_fill(uint4 (&wr)[D][NT][3], const unsigned short* Wb, int nf0, int gmax, int g0, int g1, int lane) {
    const int gl = g1 - 1, m = lane & 15, h4 = lane >> 4;
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
        for (int j = 0; j < NT; ++j) {
            const int nf = nf0 + 16 * j, gi = min(2 * min(g0 + d, gl) + (h4 >> 1), gmax - 1);
            const unsigned short* q = Wb + ((size_t)(nf >> 5) * gmax + gi) * 1536 + ((h4 & 1) * 32 + (nf & 16) + m) * 8;
#pragma unroll
            for (int p = 0; p < 3; ++p) wr[d][j][p] = *(const uint4*)(q + p * 512);
        }
}

template <int NT>
DEVI void x6_group16(floatx4 (&acc)[NT], const uint4 (&w)[NT][3], const float4& a0, const float4& a1) {
    const auto b = ch_split(a0, a1);
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(w[j][1]), b.m, acc[j], 0, 0, 0);
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(w[j][2]), b.s, acc[j], 0, 0, 0);
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(w[j][0]), b.l, acc[j], 0, 0, 0);
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(w[j][1]), b.s, acc[j], 0, 0, 0);
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(w[j][0]), b.m, acc[j], 0, 0, 0);
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(w[j][0]), b.h, acc[j], 0, 0, 0);
}

// acc[j] += W(tile j) . A over 32-k groups [g0, g1); A = the fp32 16-row LDS block (group G at sA + G * 512)
template <int NT, int D>
DEVI void ring16x6_run(floatx4 (&acc)[NT], uint4 (&wr)[D][NT][3], const float* sA, const unsigned short* Wb, int nf0,
                       int gmax, int g0, int g1, int lane) {
    const int gl = g1 - 1, m = lane & 15, h4 = lane >> 4;
    const float* ap = sA + ((4 * (h4 >> 1) + (h4 & 1)) * 16 + m) * 4;   // quad qa of group 0; qb = qa + 2
    float4 n0 = *(const float4*)(ap + (size_t)g0 * 512), n1 = *(const float4*)(ap + (size_t)g0 * 512 + 128);
    int gb = g0;
    for (; gb + D <= g1; gb += D) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const int g = gb + d;
            const float4 a0 = n0, a1 = n1;
            const size_t gn = (size_t)min(g + 1, gl) * 512;
            n0 = *(const float4*)(ap + gn);
            n1 = *(const float4*)(ap + gn + 128);
            __builtin_amdgcn_sched_barrier(0);
            x6_group16<NT>(acc, wr[d], a0, a1);
#pragma unroll
            for (int j = 0; j < NT; ++j) {
                const int nf = nf0 + 16 * j, gi = min(2 * min(g + D, gl) + (h4 >> 1), gmax - 1);
                const unsigned short* q = Wb + ((size_t)(nf >> 5) * gmax + gi) * 1536 + ((h4 & 1) * 32 + (nf & 16) + m) * 8;
#pragma unroll
                for (int p = 0; p < 3; ++p) wr[d][j][p] = *(const uint4*)(q + p * 512);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    }
#pragma unroll
    for (int d = 0; d < D - 1; ++d) {
        if (gb + d < g1) {
            const float4 a0 = n0, a1 = n1;
            const size_t gn = (size_t)min(gb + d + 1, gl) * 512;
            n0 = *(const float4*)(ap + gn);
            n1 = *(const float4*)(ap + gn + 128);
            x6_group16<NT>(acc, wr[d], a0, a1);
        }
    }
}

// sum over the 4 lanes of row m (h4 = 0..3), then over the 8 waves through red ([8][16])
DEVI float row16_sum(float s, float* red, int wave, int lane) {
    s += __shfl_xor(s, 16);
    s += __shfl_xor(s, 32);
    if (lane < 16) red[wave * 16 + lane] = s;
    lds_barrier();
    float tot = 0.f;
#pragma unroll
    for (int w = 0; w < 8; ++w) tot += red[w * 16 + (lane & 15)];
    return tot;
}

template <int NT>
DEVI void chain16_row_moments(const float (&v)[NT * 4], float* red0, float* red1, int wave, int lane, int M,
                              float& mean, float& rstd) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NT * 4; ++i) s += v[i];
    mean = row16_sum(s, red0, wave, lane) / (float)M;
    float m2 = 0.f;
#pragma unroll
    for (int i = 0; i < NT * 4; ++i) {
        const float d = v[i] - mean;
        m2 += d * d;
    }
    rstd = 1.0f / sqrtf(fmaxf(row16_sum(m2, red1, wave, lane) / (float)M, 0.f) + 1e-5f);
}

// features of tile j held by this lane: f0 + 16 j + 0..3 with f0 = 16 NT wave + 4 h4
template <int NT>
DEVI void chain16_bias(float (&v)[NT * 4], const floatx4 (&acc)[NT], const float* sb, int f0) {
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        const float4 bb = *(const float4*)(sb + f0 + 16 * j);
        v[4 * j + 0] = acc[j][0] + bb.x;
        v[4 * j + 1] = acc[j][1] + bb.y;
        v[4 * j + 2] = acc[j][2] + bb.z;
        v[4 * j + 3] = acc[j][3] + bb.w;
    }
}

template <int NT>
DEVI void chain16_ln(float (&v)[NT * 4], float rs, float sh, const float* sg, const float* sbe, int f0) {
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        const float4 gg = *(const float4*)(sg + f0 + 16 * j), bb = *(const float4*)(sbe + f0 + 16 * j);
        float* x = v + 4 * j;
        x[0] = fadd(fmul(fadd(fmul(x[0], rs), sh), gg.x), bb.x);
        x[1] = fadd(fmul(fadd(fmul(x[1], rs), sh), gg.y), bb.y);
        x[2] = fadd(fmul(fadd(fmul(x[2], rs), sh), gg.z), bb.z);
        x[3] = fadd(fmul(fadd(fmul(x[3], rs), sh), gg.w), bb.w);
    }
}

// the lane's quads into the [M/4][16][4] activation block: quad f0/4 + 4 j, row m (64 lanes = 1 KiB)
template <int NT>
DEVI void chain16_store_lds(float* sH, const float (&v)[NT * 4], int f0, int m) {
#pragma unroll
    for (int j = 0; j < NT; ++j)
        *(float4*)(sH + ((f0 / 4 + 4 * j) * 16 + m) * 4) = make_float4(v[4 * j], v[4 * j + 1], v[4 * j + 2], v[4 * j + 3]);
}

// X6 = 1: layers 1 and 2 on v_mfma_f32_16x16x32_bf16 with the x6 split (ring16x6_*, two passes of NT / 2 tiles);
// the last layer stays f32 MFMA.
template <int MODE, int NT, int D = 4, int D3 = 4, int X6 = 0>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4, 4))) chain16_kernel(const ChainArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, m = lane & 15, h4 = lane >> 4;
    const int pb = blockIdx.y;
    const ChainProb& P = a.p[pb];
    const int M = a.M;
    const int m0 = blockIdx.x * 16;
    float* sH = smem;                       // activation block [max(K1, M)/4][16][4]
    float* red0 = smem + a.hfl;             // [8][16]
    float* red1 = red0 + 128;               // [8][16]
    float* sp = red1 + 128;                 // parameter vectors (chain_param_floats)
    float* sb1 = sp;
    float* sb2 = sp + M;
    float* sw3 = sp + 2 * M;
    float* sb3 = sp + 3 * M;
    float* sg1 = sp + 3 * M;
    float* sbe1 = sp + 4 * M;
    float* sg2 = sp + 5 * M;
    float* sbe2 = sp + 6 * M;
    const int lo = m * 4;                   // lane offset inside a weight-panel quad (quad: wq16)
    const int q1max = (a.K1 >> 2) - 1, qMmax = (M >> 2) - 1;
    const int g1n = (a.K1 + 15) >> 4;       // 16-k groups of layer 1 (the last may be half)
    const int f0 = 16 * NT * wave + 4 * h4; // first output feature of this lane in the M-wide layers
    const long wblk = (long)(NT / 2) * wave;  // first 32-row panel block of this wave
    const bool head_dot = MODE == CH_Q || (MODE == CH_STEP && pb == 1);

    const int g1x = (a.K1 + 31) >> 5, gm1 = (a.K1 + 15) >> 4, gmM = M >> 4;   // x6: 32-k groups
    float4 wr[X6 ? 1 : D][NT];
    uint4 wx[X6 ? 2 : 1][X6 ? NT / 2 : 1][3];
    if constexpr (X6) ring16x6_fill<NT / 2, 2>(wx, P.X1, 16 * NT * wave, gm1, 0, g1x, lane);
    else ring16_fill<NT, D>(wr, P.W1 + wblk * a.K1 * 32 + lo, (long)a.K1 * 32, 0, g1n, h4, q1max);
    for (int i = tid; i < (X6 ? g1x * 8 : g1n * 4) * 16; i += 512) {
        const int row = i & 15, q = i >> 4;
        const int lm = m0 + row;
        const int xr = map_row(a.amap, lm < a.rows ? lm : 0);
        ((float4*)sH)[i] = q <= q1max ? *(const float4*)(a.X + (size_t)(xr >> 5) * a.x_ts + (size_t)(a.q1 + q) * 128 + (xr & 31) * 4)
                                      : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    for (int i = tid; i < M / 4; i += 512) {
        ((float4*)sb1)[i] = ((const float4*)P.b1)[i];
        ((float4*)sb2)[i] = ((const float4*)P.b2)[i];
        if (head_dot) ((float4*)sw3)[i] = ((const float4*)P.w3v)[i];
        if (MODE == CH_Q) {
            ((float4*)sg1)[i] = ((const float4*)P.g1)[i];
            ((float4*)sbe1)[i] = ((const float4*)P.be1)[i];
            ((float4*)sg2)[i] = ((const float4*)P.g2)[i];
            ((float4*)sbe2)[i] = ((const float4*)P.be2)[i];
        }
    }
    if (!head_dot)
        for (int i = tid; i < a.n3 / 4; i += 512) ((float4*)sb3)[i] = ((const float4*)a.b3)[i];
    float g_old = 0.f;
    if (MODE == CH_STEP && pb == 1 && tid < 16 && !a.first && m0 + tid < a.rows)
        g_old = a.G[map_row(a.amap, m0 + tid)];
    float eps4[4] = {0.f, 0.f, 0.f, 0.f};
    if (MODE == CH_PI && tid < (a.nstore >> 2) * 16 && m0 + (tid & 15) < a.rows) {
        const int lm = m0 + (tid & 15), c = 4 * (tid >> 4);
        const int e = lm / a.eps_G, rr = lm % a.eps_G;
        const float* ep = a.eps + (size_t)e * a.eps_env + a.eps_off + (size_t)rr * a.A;
#pragma unroll
        for (int k = 0; k < 4; ++k) eps4[k] = c + k < a.nvalid ? ep[c + k] : 0.f;
    }
    lds_barrier();

    // ---- layer 1
    floatx4 acc[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
    // x6: the NT tiles in two passes of NT / 2 (the ring of the second pass fills after the first runs)
    auto x6_layer = [&](const unsigned short* W, int gmax, int gn, const float* sA) {
      if constexpr (X6 != 0) {
        floatx4 ah[NT / 2];
#pragma unroll
        for (int j = 0; j < NT / 2; ++j) ah[j] = floatx4{0.f, 0.f, 0.f, 0.f};
        ring16x6_run<NT / 2, 2>(ah, wx, sA, W, 16 * NT * wave, gmax, 0, gn, lane);
#pragma unroll
        for (int j = 0; j < NT / 2; ++j) { acc[j] = ah[j]; ah[j] = floatx4{0.f, 0.f, 0.f, 0.f}; }
        ring16x6_fill<NT / 2, 2>(wx, W, 16 * NT * wave + 16 * (NT / 2), gmax, 0, gn, lane);
        ring16x6_run<NT / 2, 2>(ah, wx, sA, W, 16 * NT * wave + 16 * (NT / 2), gmax, 0, gn, lane);
#pragma unroll
        for (int j = 0; j < NT / 2; ++j) acc[NT / 2 + j] = ah[j];
      }
    };
    if constexpr (X6) {
        x6_layer(P.X1, gm1, g1x, sH);
        if constexpr (X6 != 0) ring16x6_fill<NT / 2, 2>(wx, P.X2, 16 * NT * wave, gmM, 0, M >> 5, lane);
    } else {
        ring16_run<NT, D>(acc, wr, sH, P.W1 + wblk * a.K1 * 32 + lo, (long)a.K1 * 32, 0, g1n, lane, q1max);
        ring16_fill<NT, D>(wr, P.W2 + wblk * M * 32 + lo, (long)M * 32, 0, M >> 4, h4, qMmax);
    }
    lds_barrier();
    {
        float v[NT * 4];
        chain16_bias<NT>(v, acc, sb1, f0);
        if (MODE == CH_Q) {
            float mean, rs;
            chain16_row_moments<NT>(v, red0, red1, wave, lane, M, mean, rs);
            chain16_ln<NT>(v, rs, -rs * mean, sg1, sbe1, f0);
#pragma unroll
            for (int i = 0; i < NT * 4; ++i) v[i] = tanh_f(v[i]);
        } else {
#pragma unroll
            for (int i = 0; i < NT * 4; ++i) v[i] = elu_f(v[i]);
        }
        chain16_store_lds<NT>(sH, v, f0, m);
    }
    lds_barrier();

    // ---- layer 2
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
    if constexpr (X6) x6_layer(P.X2, gmM, M >> 5, sH);
    else ring16_run<NT, D>(acc, wr, sH, P.W2 + wblk * M * 32 + lo, (long)M * 32, 0, M >> 4, lane, qMmax);

    // layer-3 items (16-column tile, K part): up to 4 per wave (items <= 32)
    const int nb3 = a.n3 >> 4;
    const int ks = nb3 >= 8 ? 1 : 8 / nb3;
    const int items = nb3 * ks;
    const int gper = (M >> 4) / ks;
    float4 w3r[D3][1];
    auto w3p = [&](int it) { const int t = it / ks; return a.W3 + (size_t)(t >> 1) * M * 32 + (t & 1) * 64 + lo; };
    if (!head_dot && wave < items)
        ring16_fill<1, D3>(w3r, w3p(wave), (long)M * 32, (wave % ks) * gper, (wave % ks + 1) * gper, h4, qMmax);
    float v[NT * 4];
    chain16_bias<NT>(v, acc, sb2, f0);
    if (head_dot) {
        if (MODE == CH_Q) {
            float mean, rs;
            chain16_row_moments<NT>(v, red0, red1, wave, lane, M, mean, rs);
            chain16_ln<NT>(v, rs, -rs * mean, sg2, sbe2, f0);
        }
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < NT; ++j) {
            const float4 w4 = *(const float4*)(sw3 + f0 + 16 * j);
            const float* x = v + 4 * j;
            s += (elu_f(x[0]) * w4.x + elu_f(x[1]) * w4.y) + (elu_f(x[2]) * w4.z + elu_f(x[3]) * w4.w);
        }
        s += __shfl_xor(s, 16);
        s += __shfl_xor(s, 32);
        if (lane < 16) red0[wave * 16 + lane] = s;
        lds_barrier();
        if (tid < 16) {
            const int lm = m0 + tid;
            if (lm < a.rows) {
                const int xr = map_row(a.amap, lm);
                float tot = 0.f;
#pragma unroll
                for (int w = 0; w < 8; ++w) tot += red0[w * 16 + tid];
                const float o = tot + P.b3v[0];
                if (MODE == CH_Q) {
                    a.q[(size_t)pb * a.q_ld + xr] = o;
                } else {
                    const float dr = fmul(a.disc, o);
                    a.G[xr] = a.first ? dr : fadd(g_old, dr);
                    if (a.last) a.rlast[xr] = o;
                }
            }
        }
        return;
    }
#pragma unroll
    for (int i = 0; i < NT * 4; ++i) v[i] = elu_f(v[i]);
    lds_barrier();
    chain16_store_lds<NT>(sH, v, f0, m);
    lds_barrier();

    // ---- layer 3: [16 x M] . W3^T -> [16 x n3]; partial tiles meet in the activation block after the reads
    floatx4 a3[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) a3[u] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int it = wave + 8 * u;
        if (it < items) {
            floatx4 t1[1] = {a3[u]};
            if (u > 0) ring16_fill<1, D3>(w3r, w3p(it), (long)M * 32, (it % ks) * gper, (it % ks + 1) * gper, h4, qMmax);
            ring16_run<1, D3>(t1, w3r, sH, w3p(it), (long)M * 32, (it % ks) * gper, (it % ks + 1) * gper, lane, qMmax);
            a3[u] = t1[0];
        }
    }
    lds_barrier();
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int it = wave + 8 * u;
        if (it < items) *(float4*)(sH + (size_t)it * 256 + lane * 4) = make_float4(a3[u][0], a3[u][1], a3[u][2], a3[u][3]);
    }
    lds_barrier();
    for (int i = tid; i < (a.nstore >> 2) * 16; i += 512) {
        const int row = i & 15, cq = i >> 4;
        const int lm = m0 + row;
        if (lm >= a.rows) continue;
        const int t = cq >> 2, qi = cq & 3;
        float4 s = *(const float4*)(sH + (size_t)(t * ks) * 256 + (qi * 16 + row) * 4);
        for (int kp = 1; kp < ks; ++kp) {
            const float4 u = *(const float4*)(sH + (size_t)(t * ks + kp) * 256 + (qi * 16 + row) * 4);
            s.x += u.x; s.y += u.y; s.z += u.z; s.w += u.w;
        }
        const int c = 4 * cq;
        const float4 bb = *(const float4*)(sb3 + c);
        float o[4] = {s.x + bb.x, s.y + bb.y, s.z + bb.z, s.w + bb.w};
        const int xr = map_row(a.amap, lm);
        if (MODE == CH_PI) {
            float mu4[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                float x = 0.f;
                mu4[k] = 0.f;
                if (c + k < a.nvalid) {
                    const float muv = tanhf(o[k]);
                    x = muv;
                    mu4[k] = muv;
                    if (a.min_std > 0.f) {
                        const float ee = tclamp(fmul(eps4[k], a.min_std), -0.3f, 0.3f);
                        x = tclamp(fadd(muv, ee), a.lo, a.hi);
                    }
                }
                o[k] = x;
            }
            if (a.mu_out) *(float4*)(a.mu_out + (size_t)xr * a.nstore + c) = make_float4(mu4[0], mu4[1], mu4[2], mu4[3]);
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (c + k >= a.nvalid) o[k] = 0.f;
        }
        *(float4*)(a.Xo + (size_t)(xr >> 5) * a.x_ts + (size_t)(a.out_q0 + cq) * 128 + (xr & 31) * 4) =
            make_float4(o[0], o[1], o[2], o[3]);
    }
}

// ------------------------------------------------------------------------------------------------ split step
// TOLD.next for narrow launches (one env: 512 / 768 rows), where even 16-row chain workgroups leave most CUs
// idle and the layered path pays three dependent launches per step. Grid (16-row blocks, SPLIT_S slices, 2 heads):
// every workgroup computes the full first layer of its head for its 16 rows (K = L + A: cheap), then only its
// slice of the M x M second layer (M / SPLIT_S columns, one 16-column tile per wave), then the slice's share of
// the last layer: dynamics z' partial = W3[:, slice] . h2[slice] (K = M / SPLIT_S) into zpart[s], reward partial
// dot w3[slice] . ELU(h2[slice]) into rpart_s[s]. split_finish_kernel sums the SPLIT_S partials in slice order
// (+ bias) into X_{t+1}'s latent columns and the return update. Repeating the first layer SPLIT_S times costs
// ~13 % extra MFMA work at humanoid sizes on a chip that one env leaves mostly idle.
struct SplitArgs {
    ChainProb p[2];
    int rows, M, K1, q1;
    RowMap amap;
    const float* X; long x_ts;
    const float* W3; int n3;                 // dynamics last layer: panel [n3][M]
    float* zpart; float* rpart; int prow;    // partial buffers (logical rows, row stride prow)
    // deferred finish of the previous step (zin != null): its partials are summed while staging X_t's latent
    // quads [zq0, zq0 + Lp/4) (written back to X_t by slice 0's dynamics workgroup), and slice 0's reward
    // workgroup applies its return update
    const float* zin; const float* rin; const float* b3d; const float* b3r; int L, Lp, zq0;
    float* Xw; float* G; float disc_in; int first_in;
    const unsigned short* X3;                // x6 form (split_step_kernel<..., X6 = 1>): W3 in the x6 layout
};

__host__ __device__ inline int split_hfl(int K1, int M) { return ((int)rup(K1, 32) > M ? (int)rup(K1, 32) : M) * 16; }
__host__ __device__ inline int split_lds_floats(int K1, int M) {
    return split_hfl(K1, M) + (M / SPLIT_S) * 16 + 128 + M + 2 * (M / SPLIT_S);
}

// X6 = 1: the three layers on v_mfma_f32_16x16x32_bf16 with the x6 split (ring16x6_*), same data flow.
template <int NT, int D = 4, int X6 = 0>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4, 4))) split_step_kernel(const SplitArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, m = lane & 15, h4 = lane >> 4;
    const int sl = blockIdx.y, pb = blockIdx.z;
    const ChainProb& P = a.p[pb];
    const int M = a.M, SW = M / SPLIT_S;     // slice width = 8 waves x 16 columns
    const int m0 = blockIdx.x * 16;
    float* sH = smem;                        // input block, then h1 [M/4][16][4]
    float* sS = smem + split_hfl(a.K1, M);   // h2 slice [SW/4][16][4]
    float* red = sS + SW * 16;               // [8][16]
    float* sb1 = red + 128;                  // [M]
    float* sb2 = sb1 + M;                    // [SW] second-layer bias of the slice
    float* sw3 = sb2 + SW;                   // [SW] reward head weights of the slice
    const int lo = m * 4;
    const int q1max = (a.K1 >> 2) - 1, qMmax = (M >> 2) - 1;
    const int g1n = (a.K1 + 15) >> 4;
    const int f0 = 16 * NT * wave + 4 * h4;
    const long wblk = (long)(NT / 2) * wave;
    // x6: 32-k groups; the x6 matrices' 16-k group counts
    const int g1x = (a.K1 + 31) >> 5, gm1 = (a.K1 + 15) >> 4, gmM = M >> 4;

    float4 wr[X6 ? 1 : D][NT];
    uint4 wx[X6 ? 2 : 1][X6 ? NT / 2 : 1][3];   // x6 layer 1: two passes of NT / 2 tiles, 2 groups deep
    if constexpr (X6) ring16x6_fill<NT / 2, 2>(wx, P.X1, 16 * NT * wave, gm1, 0, g1x, lane);
    else ring16_fill<NT, D>(wr, P.W1 + wblk * a.K1 * 32 + lo, (long)a.K1 * 32, 0, g1n, h4, q1max);
    for (int i = tid; i < (X6 ? g1x * 8 : g1n * 4) * 16; i += 512) {
        const int row = i & 15, q = i >> 4;
        const int lm = m0 + row;
        const int lr = lm < a.rows ? lm : 0;
        const int xr = map_row(a.amap, lr);
        float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
        const size_t xo = (size_t)(xr >> 5) * a.x_ts + (size_t)(a.q1 + q) * 128 + (xr & 31) * 4;
        if (a.zin && q >= a.zq0 && q < a.zq0 + (a.Lp >> 2)) {
            float o[4];
#pragma unroll
            for (int cc = 0; cc < 4; ++cc) {
                const int col = 4 * (q - a.zq0) + cc;
                if (col < a.L) {
                    float sz = a.zin[(size_t)lr * a.n3 + col];
#pragma unroll
                    for (int sl2 = 1; sl2 < SPLIT_S; ++sl2) sz += a.zin[((size_t)sl2 * a.prow + lr) * a.n3 + col];
                    o[cc] = sz + a.b3d[col];
                } else {
                    o[cc] = 0.f;
                }
            }
            x = make_float4(o[0], o[1], o[2], o[3]);
            if (sl == 0 && pb == 0 && lm < a.rows) *(float4*)(a.Xw + xo) = x;
        } else if (q <= q1max) {
            x = *(const float4*)(a.X + xo);
        }
        ((float4*)sH)[i] = x;
    }
    if (a.rin && sl == 0 && pb == 1 && tid < 16 && m0 + tid < a.rows) {
        const int lm = m0 + tid, xr = map_row(a.amap, lm);
        float r = a.rin[lm];
#pragma unroll
        for (int sl2 = 1; sl2 < SPLIT_S; ++sl2) r += a.rin[(size_t)sl2 * a.prow + lm];
        const float dr = fmul(a.disc_in, r + a.b3r[0]);
        a.G[xr] = a.first_in ? dr : fadd(a.G[xr], dr);
    }
    for (int i = tid; i < M / 4; i += 512) ((float4*)sb1)[i] = ((const float4*)P.b1)[i];
    for (int i = tid; i < SW / 4; i += 512) {
        ((float4*)sb2)[i] = ((const float4*)(P.b2 + sl * SW))[i];
        if (pb == 1) ((float4*)sw3)[i] = ((const float4*)(P.w3v + sl * SW))[i];
    }
    lds_barrier();

    // ---- layer 1, all M columns
    floatx4 acc[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
    const int n2 = sl * SW + 16 * wave;
    float4 w2[X6 ? 1 : D][1];
    uint4 w2x[X6 ? D : 1][1][3];
    if constexpr (X6) {
        floatx4 ah[NT / 2];
#pragma unroll
        for (int j = 0; j < NT / 2; ++j) ah[j] = floatx4{0.f, 0.f, 0.f, 0.f};
        ring16x6_run<NT / 2, 2>(ah, wx, sH, P.X1, 16 * NT * wave, gm1, 0, g1x, lane);
#pragma unroll
        for (int j = 0; j < NT / 2; ++j) { acc[j] = ah[j]; ah[j] = floatx4{0.f, 0.f, 0.f, 0.f}; }
        ring16x6_fill<NT / 2, 2>(wx, P.X1, 16 * NT * wave + 16 * (NT / 2), gm1, 0, g1x, lane);
        ring16x6_run<NT / 2, 2>(ah, wx, sH, P.X1, 16 * NT * wave + 16 * (NT / 2), gm1, 0, g1x, lane);
#pragma unroll
        for (int j = 0; j < NT / 2; ++j) acc[NT / 2 + j] = ah[j];
        ring16x6_fill<1, D>(w2x, P.X2, n2, gmM, 0, M >> 5, lane);
    } else {
        ring16_run<NT, D>(acc, wr, sH, P.W1 + wblk * a.K1 * 32 + lo, (long)a.K1 * 32, 0, g1n, lane, q1max);
    }
    // this wave's 16 columns of the slice in the second layer; its weights in flight during the epilogue
    const float* W2p = P.W2 + (size_t)(n2 >> 5) * M * 32 + (n2 & 31) * 4 + lo;
    if constexpr (!X6) ring16_fill<1, D>(w2, W2p, (long)M * 32, 0, M >> 4, h4, qMmax);
    lds_barrier();   // every wave is done with the input block
    {
        float v[NT * 4];
        chain16_bias<NT>(v, acc, sb1, f0);
#pragma unroll
        for (int i = 0; i < NT * 4; ++i) v[i] = elu_f(v[i]);
        chain16_store_lds<NT>(sH, v, f0, m);
    }
    lds_barrier();

    // ---- layer 2, the slice
    floatx4 a2[1] = {floatx4{0.f, 0.f, 0.f, 0.f}};
    if constexpr (X6) ring16x6_run<1, D>(a2, w2x, sH, P.X2, n2, gmM, 0, M >> 5, lane);
    else ring16_run<1, D>(a2, w2, sH, W2p, (long)M * 32, 0, M >> 4, lane, qMmax);
    const int c2 = 16 * wave + 4 * h4;       // slice-local feature of a2[0][0]
    float v2[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v2[k] = elu_f(a2[0][k] + sb2[c2 + k]);
    if (pb == 1) {
        // reward: partial dot of the slice, reduced over the row's 4 lanes and the 8 waves
        float sd = (v2[0] * sw3[c2] + v2[1] * sw3[c2 + 1]) + (v2[2] * sw3[c2 + 2] + v2[3] * sw3[c2 + 3]);
        sd += __shfl_xor(sd, 16);
        sd += __shfl_xor(sd, 32);
        if (lane < 16) red[wave * 16 + lane] = sd;
        lds_barrier();
        if (tid < 16 && m0 + tid < a.rows) {
            float tot = 0.f;
#pragma unroll
            for (int w = 0; w < 8; ++w) tot += red[w * 16 + tid];
            a.rpart[(size_t)sl * a.prow + m0 + tid] = tot;
        }
        return;
    }
    *(float4*)(sS + ((c2 >> 2) * 16 + m) * 4) = make_float4(v2[0], v2[1], v2[2], v2[3]);
    lds_barrier();
    // ---- the slice's share of the last layer: K = the slice's SW columns = 16-k groups [gs0, gs1) of W3
    const int gs0 = sl * (SW >> 4), gs1 = gs0 + (SW >> 4);
    for (int t = wave; t < (a.n3 >> 4); t += 8) {
        floatx4 a3[1] = {floatx4{0.f, 0.f, 0.f, 0.f}};
        if constexpr (X6) {
            const int gx0 = sl * (SW >> 5), gx1 = gx0 + (SW >> 5);
            uint4 w3x[D][1][3];
            ring16x6_fill<1, D>(w3x, a.X3, 16 * t, gmM, gx0, gx1, lane);
            ring16x6_run<1, D>(a3, w3x, sS - (size_t)gx0 * 512, a.X3, 16 * t, gmM, gx0, gx1, lane);
        } else {
            const float* W3p = a.W3 + (size_t)(t >> 1) * M * 32 + (t & 1) * 64 + lo;
            float4 w3[D][1];
            ring16_fill<1, D>(w3, W3p, (long)M * 32, gs0, gs1, h4, qMmax);
            ring16_run<1, D>(a3, w3, sS - (size_t)gs0 * 256, W3p, (long)M * 32, gs0, gs1, lane, qMmax);
        }
        if (m0 + m < a.rows)
            *(float4*)(a.zpart + ((size_t)sl * a.prow + m0 + m) * a.n3 + t * 16 + 4 * h4) =
                make_float4(a3[0][0], a3[0][1], a3[0][2], a3[0][3]);
    }
}

struct SplitFinishArgs {
    int rows; RowMap amap;
    const float* zpart; const float* rpart; int prow, n3, L, Lp;
    const float* b3d; const float* b3r;
    float* Xo; long x_ts; int out_q0;
    float* G; float* rlast; float disc; int first, last;
};

// z' = sum_s zpart[s] + b into X_{t+1}'s latent quads (zero past L); reward = sum_s rpart[s] + b, G += disc * r
// (tdmpc.py:88-90), r_{H-1} kept on the last step. One thread per (row, latent quad | reward).
__global__ void __launch_bounds__(256) split_finish_kernel(const SplitFinishArgs a) {
    const int nq = a.Lp / 4;
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const int row = (int)(i / (nq + 1)), q = (int)(i % (nq + 1));
    if (row >= a.rows) return;
    const int xr = map_row(a.amap, row);
    if (q < nq) {
        float o[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int col = 4 * q + c;
            if (col < a.L) {
                float s = a.zpart[(size_t)row * a.n3 + col];
#pragma unroll
                for (int sl = 1; sl < SPLIT_S; ++sl) s += a.zpart[((size_t)sl * a.prow + row) * a.n3 + col];
                o[c] = s + a.b3d[col];
            } else {
                o[c] = 0.f;
            }
        }
        *(float4*)(a.Xo + (size_t)(xr >> 5) * a.x_ts + (size_t)(a.out_q0 + q) * 128 + (xr & 31) * 4) =
            make_float4(o[0], o[1], o[2], o[3]);
    } else {
        float r = a.rpart[row];
#pragma unroll
        for (int sl = 1; sl < SPLIT_S; ++sl) r += a.rpart[(size_t)sl * a.prow + row];
        const float o = r + a.b3r[0];
        const float dr = fmul(a.disc, o);
        a.G[xr] = a.first ? dr : fadd(a.G[xr], dr);
        if (a.last) a.rlast[xr] = o;
    }
}

struct SplitPiArgs {
    int rows; RowMap amap;
    const float* part; int prow, n3, A, Ap;
    const float* b3;
    float* Xo; long x_ts;
    const float* eps; int eps_G; long eps_env; long eps_off; float min_std, lo, hi;
};

// The split pi head's finish: mu = tanh(sum_s part[s] + b) and the TruncatedNormal sample (tdmpc.py:39-45,
// helper.py:86-96; the chain CH_PI epilogue's exact arithmetic) into X_t's action quads. One thread per
// (row, action quad).
__global__ void __launch_bounds__(256) split_pi_finish_kernel(const SplitPiArgs a) {
    const int nq = a.Ap / 4;
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const int row = (int)(i / nq), q = (int)(i % nq);
    if (row >= a.rows) return;
    const int xr = map_row(a.amap, row);
    const int e = row / a.eps_G, rr = row % a.eps_G;
    const float* ep = a.eps + (size_t)e * a.eps_env + a.eps_off + (size_t)rr * a.A;
    float o[4];
#pragma unroll
    for (int cc = 0; cc < 4; ++cc) {
        const int col = 4 * q + cc;
        float x = 0.f;
        if (col < a.A) {
            float sv = a.part[(size_t)row * a.n3 + col];
#pragma unroll
            for (int sl = 1; sl < SPLIT_S; ++sl) sv += a.part[((size_t)sl * a.prow + row) * a.n3 + col];
            const float muv = tanhf(sv + a.b3[col]);
            x = muv;
            if (a.min_std > 0.f) {
                const float ee = tclamp(fmul(ep[col], a.min_std), -0.3f, 0.3f);
                x = tclamp(fadd(muv, ee), a.lo, a.hi);
            }
        }
        o[cc] = x;
    }
    *(float4*)(a.Xo + (size_t)(xr >> 5) * a.x_ts + (size_t)q * 128 + (xr & 31) * 4) = make_float4(o[0], o[1], o[2], o[3]);
}

// TOLD.next's first layer at t = 0 splits as W1 [a | z0] = W1[:, :k1c] X_0[:k1c] + W1[:, k1c:] X_0[k1c:]: every
// row of an env shares z0, so the second term (plus the bias) is computed once per env and head here and the chain
// kernel's t = 0 steps run layer 1 over the first k1c columns (the actions, rounded up to a k group) only.
// Grid (B, 2 heads, M / 256); one output column per thread, fp32 FMAs in k order; W1 is the fp32 panel.
__global__ void __launch_bounds__(256) z0c_kernel(const float* W1, const float* b1, const float* z0, int Kx, int Ap,
                                                   int Lp, int k1c, int M, float* out) {
    const int e = blockIdx.x, p = blockIdx.y, n = blockIdx.z * 256 + threadIdx.x;
    if (n >= M) return;
    const int nn = p * M + n;
    const float* wrow = W1 + (size_t)(nn >> 5) * Kx * 32 + (nn & 31) * 4;
    float acc = 0.f;
    // one weight quad (4 consecutive k of the panel) per load, k order kept (k1c and Kx are multiples of 4)
#pragma unroll 8
    for (int kq = k1c >> 2; kq < Kx >> 2; ++kq) {
        const float4 w = *(const float4*)(wrow + kq * 128);
        const int zi = 4 * kq - Ap;
        const float* zr = z0 + (size_t)e * Lp;
        acc = fmaf(w.x, zi + 0 < Lp ? zr[zi + 0] : 0.f, acc);
        acc = fmaf(w.y, zi + 1 < Lp ? zr[zi + 1] : 0.f, acc);
        acc = fmaf(w.z, zi + 2 < Lp ? zr[zi + 2] : 0.f, acc);
        acc = fmaf(w.w, zi + 3 < Lp ? zr[zi + 3] : 0.f, acc);
    }
    out[((size_t)e * 2 + p) * M + n] = acc + b1[nn];
}

// The pi rows' terminal action in CEM iterations >= 1 (tdmpc.py:91, pi(z_H, min_std)): their z_H is the same in
// every iteration (same z0, same pi actions), so mu = tanh(pi(z_H)) is the one the first iteration's pi launch
// cached (ChainArgs::mu_out); only the TruncatedNormal sample is redrawn, with the chain epilogue's arithmetic.
// One thread per (row, action quad).
struct PiMuArgs {
    int rows; RowMap amap; RowMap mmap; const float* mu; int Ap, A; float* Xo; long x_ts;   // mu row: map_row(mmap, row)
    const float* eps; int eps_G; long eps_env; long eps_off; float min_std, lo, hi;
};

DEVI void pi_from_mu_item(const PiMuArgs& a, long i) {
    const int nq = a.Ap / 4;
    const int row = (int)(i / nq), q = (int)(i % nq);
    if (row >= a.rows) return;
    const int xr = map_row(a.amap, row);
    const int e = row / a.eps_G, rr = row % a.eps_G;
    const float* ep = a.eps + (size_t)e * a.eps_env + a.eps_off + (size_t)rr * a.A;
    const float4 m = *(const float4*)(a.mu + (size_t)map_row(a.mmap, row) * a.Ap + 4 * q);
    const float mv[4] = {m.x, m.y, m.z, m.w};
    float o[4];
#pragma unroll
    for (int cc = 0; cc < 4; ++cc) {
        const int col = 4 * q + cc;
        float x = 0.f;
        if (col < a.A) {
            x = mv[cc];
            if (a.min_std > 0.f) {
                const float ee = tclamp(fmul(ep[col], a.min_std), -0.3f, 0.3f);
                x = tclamp(fadd(mv[cc], ee), a.lo, a.hi);
            }
        }
        o[cc] = x;
    }
    *(float4*)(a.Xo + (size_t)(xr >> 5) * a.x_ts + (size_t)q * 128 + (xr & 31) * 4) = make_float4(o[0], o[1], o[2], o[3]);
}

__global__ void __launch_bounds__(256) pi_from_mu_kernel(const PiMuArgs a) {
    pi_from_mu_item(a, (long)blockIdx.x * blockDim.x + threadIdx.x);
}


// estimate_value's terminal combination (tdmpc.py:91-92): G + gamma^H min(Q1, Q2), nan_to_num.
DEVI float qvalue(float G, float q1, float q2, float discH) {
    const float qm = (q1 != q1 || q2 != q2) ? NAN : fminf(q1, q2);   // torch.min keeps NaN
    return nan_to_num(fadd(G, fmul(discH, qm)));
}

__global__ void qvalue_kernel(const float* G, const float* q, int q_ld, float discH, float* value, int rows) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < rows) value[i] = qvalue(G[i], q[i], q[q_ld + i], discH);
}

// ------------------------------------------------------------------------------------------------ LN+tanh
// a1 = tanh(LayerNorm(y1)) for both Q heads (helper.q: Linear -> LayerNorm -> Tanh), computed once per
// element from the producer's per-64-column moments, so the next GEMM is a plain one. Grid: (row tiles,
// Q head); 32 consecutive lanes own 32 consecutive rows of one panel quad (512 B contiguous).
struct LnArgs {
    const float* Y; float* O; long ts; const float2* st; int st_ld; int M_; int rows;
    const float* g; const float* b;
};

__global__ void __launch_bounds__(512) ln_tanh_kernel(const LnArgs a) {
    const int r = threadIdx.x & 31, g = threadIdx.x >> 5;   // 16 threads per row
    const int row = blockIdx.x * 32 + r;
    if (row >= a.rows) return;
    const int p = blockIdx.y;                                 // Q head
    const int ntile = a.M_ / 64, nq = a.M_ / 4;
    const float2* st = a.st + (size_t)row * a.st_ld + p * ntile;
    float n = 0.f, mean = 0.f, m2 = 0.f;
    for (int i = 0; i < ntile; ++i) {
        const float2 s = st[i];
        const float nn = n + 64.f, delta = s.x - mean;
        mean += delta * 64.f / nn;
        m2 += s.y + delta * delta * n * 64.f / nn;
        n = nn;
    }
    const float rs = 1.0f / sqrtf(fmaxf(m2 / n, 0.f) + 1e-5f);
    const float sh = -rs * mean;
    const size_t base = (size_t)(row >> 5) * a.ts + (row & 31) * 4;
#pragma unroll 8
    for (int q = g; q < nq; q += 16) {
        const int c = p * a.M_ + 4 * q;
        const float4 y = *(const float4*)(a.Y + base + (size_t)(c >> 2) * 128);
        const float4 gg = *(const float4*)(a.g + c), bb = *(const float4*)(a.b + c);
        float4 o;
        // ATen LayerNorm: (x * rstd + (-rstd * mean)) * gamma + beta
        o.x = tanh_f(fadd(fmul(fadd(fmul(y.x, rs), sh), gg.x), bb.x));
        o.y = tanh_f(fadd(fmul(fadd(fmul(y.y, rs), sh), gg.y), bb.y));
        o.z = tanh_f(fadd(fmul(fadd(fmul(y.z, rs), sh), gg.z), bb.z));
        o.w = tanh_f(fadd(fmul(fadd(fmul(y.w, rs), sh), gg.w), bb.w));
        *(float4*)(a.O + base + (size_t)(c >> 2) * 128) = o;
    }
}

// ------------------------------------------------------------------------------------------------ value
// q_p = w3_p . ELU(LN_p(y_p)) + b3_p (helper.q last layers), G += gamma^H min(q1, q2), nan_to_num
// (tdmpc.py:91-92). One workgroup per 32-row panel tile, 16 threads per row; loads unrolled so each
// thread has all of its operands in flight at once.
struct ValueArgs {
    const float* Y; long yts; const float2* st; int st_ld; int M_;
    const float* g2; const float* be2; const float* w3; const float* b3;
    const float* G; float disc; float* value; int rows;
    RowMap map;                          // logical row -> row of G / value (the Q input rows were gathered)
};

__global__ void __launch_bounds__(512) value_kernel(const ValueArgs a) {
    __shared__ float red[2][16][32];
    const int tid = threadIdx.x, r = tid & 31, g = tid >> 5;
    const int row = blockIdx.x * 32 + r;
    const int rr = row < a.rows ? row : 0;
    const int ntile = a.M_ / 64, nq = a.M_ / 4;
    const float* ybase = a.Y + (size_t)(rr >> 5) * a.yts + (rr & 31) * 4;
    for (int p = 0; p < 2; ++p) {
        const float2* st = a.st + (size_t)rr * a.st_ld + p * ntile;
        float n = 0.f, mean = 0.f, m2 = 0.f;
        for (int i = 0; i < ntile; ++i) {
            const float2 s = st[i];
            const float nn = n + 64.f, delta = s.x - mean;
            mean += delta * 64.f / nn;
            m2 += s.y + delta * delta * n * 64.f / nn;
            n = nn;
        }
        const float rs = 1.0f / sqrtf(fmaxf(m2 / n, 0.f) + 1e-5f);
        const float sh = -rs * mean;
        const float* gp = a.g2 + p * a.M_;
        const float* bp = a.be2 + p * a.M_;
        const float* wp = a.w3 + p * a.M_;
        float s = 0.f;
#pragma unroll 8
        for (int q = g; q < nq; q += 16) {
            const float4 yv = *(const float4*)(ybase + (size_t)(p * nq + q) * 128);
            const float4 gv = *(const float4*)(gp + 4 * q), bv = *(const float4*)(bp + 4 * q);
            const float4 wv = *(const float4*)(wp + 4 * q);
            s += elu_f(fadd(fmul(fadd(fmul(yv.x, rs), sh), gv.x), bv.x)) * wv.x;
            s += elu_f(fadd(fmul(fadd(fmul(yv.y, rs), sh), gv.y), bv.y)) * wv.y;
            s += elu_f(fadd(fmul(fadd(fmul(yv.z, rs), sh), gv.z), bv.z)) * wv.z;
            s += elu_f(fadd(fmul(fadd(fmul(yv.w, rs), sh), gv.w), bv.w)) * wv.w;
        }
        red[p][g][r] = s;
    }
    __syncthreads();
    if (tid < 32 && row < a.rows) {
        float q[2];
        for (int p = 0; p < 2; ++p) {
            float s = 0.f;
            for (int i = 0; i < 16; ++i) s += red[p][i][r];
            q[p] = s + a.b3[p];
        }
        const float qm = (q[0] != q[0] || q[1] != q[1]) ? NAN : fminf(q[0], q[1]);  // torch.min keeps NaN
        const int x = map_row(a.map, row);
        a.value[x] = nan_to_num(fadd(a.G[x], fmul(a.disc, qm)));
    }
}


// ------------------------------------------------------------------------------------------------ prep
// Fills X before a CEM iteration's rollout: the sampled candidates of the N rollout rows for every step,
// actions = clamp(mean + std * randn, -1, 1) (tdmpc.py:130-132, multiply then add like ATen), and -- before
// the first iteration -- the latent columns of X_0 for all T rows with z0 = h(obs) (tdmpc.py:126-127: every
// trajectory starts at the encoded observation). One float4 panel quad per thread, consecutive threads on
// consecutive rows (512-byte runs of the panel layout).
struct PrepArgs {
    float* X; size_t x_stride; int Kx, apq, lpq;
    int B, N, T, H, A;
    const float* mean; const float* stdv; int mstride;   // [B][Hmax][A]
    const float* eps; long eps_env; long eps_off;        // candidate noise [H][N][A] at eps_off per env
    const float* z0;                                     // [B][Lp] or null (no broadcast)
    long n_zq, n_sq;                                     // work items: z quads, sample quads
    PiMuArgs pm; long n_pm;                              // ... and the policy rows' terminal redraw (pi_from_mu)
};

__global__ void __launch_bounds__(256) prep_kernel(const PrepArgs a) {
    const long total = a.n_zq + a.n_sq + a.n_pm;
    for (long it = (long)blockIdx.x * blockDim.x + threadIdx.x; it < total; it += (long)gridDim.x * blockDim.x) {
        if (it >= a.n_zq + a.n_sq) {
            pi_from_mu_item(a.pm, it - a.n_zq - a.n_sq);
        } else if (it < a.n_zq) {
            // (e, q, row) with row fastest: X_0[e*T + row] latent quad q = z0[e][4q..4q+3]
            const int row = (int)(it % a.T);
            const long r2 = it / a.T;
            const int q = (int)(r2 % a.lpq), e = (int)(r2 / a.lpq);
            const int gr = e * a.T + row;
            *(float4*)(a.X + (size_t)(gr >> 5) * a.Kx * 32 + (size_t)(a.apq + q) * 128 + (gr & 31) * 4) =
                *(const float4*)(a.z0 + (size_t)e * a.lpq * 4 + q * 4);
        } else {
            // (e, t, q, n) with n fastest
            long r2 = it - a.n_zq;
            const int n = (int)(r2 % a.N); r2 /= a.N;
            const int q = (int)(r2 % a.apq); r2 /= a.apq;
            const int t = (int)(r2 % a.H);
            const int e = (int)(r2 / a.H);
            const float* mt = a.mean + (size_t)e * a.mstride + (size_t)t * a.A;
            const float* sd = a.stdv + (size_t)e * a.mstride + (size_t)t * a.A;
            const float* ep = a.eps + (size_t)e * a.eps_env + a.eps_off + ((size_t)t * a.N + n) * a.A;
            float v[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int cc = q * 4 + k;
                v[k] = cc < a.A ? tclamp(fadd(mt[cc], fmul(sd[cc], ep[cc])), -1.f, 1.f) : 0.f;
            }
            const int gr = e * a.T + n;
            *(float4*)(a.X + (size_t)t * a.x_stride + (size_t)(gr >> 5) * a.Kx * 32 + (size_t)q * 128 + (gr & 31) * 4) =
                make_float4(v[0], v[1], v[2], v[3]);
        }
    }
}

// ------------------------------------------------------------------------------------------------ iCEM fill
// iCEM candidate rows besides the sampled ones (tdmpc_icem_similarity_mlp.py:213-229), written into X_t's
// action columns of each env's block of Tw rows:
//   reused elites at rows [n0, n0 + E): mode 1 (first iteration, time shift): t < eH - 1 -> the previous
//   plan's elite[t + 1] (`_elite_actions[1:]`), later steps -> clamp(mean + std * coloured noise) of a fresh
//   sequence (`sample_action_sequence(...)[-1:]` / `[-2:]` when the horizon grew); mode 2 (later iterations,
//   keep_previous_elites): the previous iteration's elites;
//   mean_row: the last iteration's sample 0 becomes the CEM mean (icem best-a).
struct FillArgs {
    float* X; size_t x_stride; int Kx, apq, Tw;
    int B, H, A, Hmax, K;
    int n0, E, mode, eH, mean_row;
    const float* mean; const float* stdv;          // [B][Hmax][A]
    const float* elites;                           // [B][Hmax][K][A]
    const float* eps; long eps_env; long reuse_off; // coloured noise [H][E][A] per env
};

__global__ void __launch_bounds__(256) icem_fill_kernel(const FillArgs a) {
    const int rows = a.E + (a.mean_row ? 1 : 0);
    const long total = (long)a.B * a.H * a.apq * rows;
    for (long it = (long)blockIdx.x * blockDim.x + threadIdx.x; it < total; it += (long)gridDim.x * blockDim.x) {
        long r2 = it;
        const int j = (int)(r2 % rows); r2 /= rows;
        const int q = (int)(r2 % a.apq); r2 /= a.apq;
        const int t = (int)(r2 % a.H);
        const int e = (int)(r2 / a.H);
        const float* mt = a.mean + ((size_t)e * a.Hmax + t) * a.A;
        const float* sd = a.stdv + ((size_t)e * a.Hmax + t) * a.A;
        float v[4];
        int row;
        if (j == a.E) {   // icem best-a: sample 0 = mean
            row = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) v[k] = q * 4 + k < a.A ? mt[q * 4 + k] : 0.f;
        } else {
            row = a.n0 + j;
            const float* el = a.elites + (size_t)e * a.Hmax * a.K * a.A;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int cc = q * 4 + k;
                float x = 0.f;
                if (cc < a.A) {
                    if (a.mode == 2) {
                        x = el[((size_t)t * a.K + j) * a.A + cc];
                    } else if (t < a.eH - 1) {
                        x = el[((size_t)(t + 1) * a.K + j) * a.A + cc];
                    } else {
                        const float ep = a.eps[(size_t)e * a.eps_env + a.reuse_off + ((size_t)t * a.E + j) * a.A + cc];
                        x = tclamp(fadd(mt[cc], fmul(sd[cc], ep)), -1.f, 1.f);
                    }
                }
                v[k] = x;
            }
        }
        const int gr = e * a.Tw + row;
        *(float4*)(a.X + (size_t)t * a.x_stride + (size_t)(gr >> 5) * a.Kx * 32 + (size_t)q * 128 + (gr & 31) * 4) =
            make_float4(v[0], v[1], v[2], v[3]);
    }
}

// ------------------------------------------------------------------------------------------------ CEM
// One workgroup (16 waves) per environment, after each iteration's values: top-k (tdmpc.py:138-139),
// softmax refit (:142-149); on the last iteration the output action (:152-160).
struct CemArgs {
    int final_iter, iter, H, N, P, T, A, K, Kx, Hmax, I;
    // candidate c of this iteration lives in row row_of(c) of its env's block of Tw rows: c < NE -> c, else
    // pi_base + (c - NE) (TDMPC.plan: NE = Tw = T, identity; iCEM: [sampled | reused elites] then pi rows)
    int Tw, NE, pi_base;
    float* elite_store;                 // optional [B][Hmax][K][A]: this iteration's elites (iCEM reuse)
    const float* X; size_t x_stride;    // X_t panels: action columns of the pi rows
    const float* value;                 // [B*T] (layered path: value_kernel's output)
    const float* G; const float* qv; int q_ld; float discH;   // chain path: value = qvalue(G, q1, q2)
    float* value_out;                   // optional [B][I][T]
    const float* rlast;                 // [B*T]
    float* mean; float* stdv;           // [B][Hmax][A]
    const float* eps; long eps_env; long eps_cem_off; long eps_iter; long eps_act_off;
    const double* u;
    float* prev_mean; int eval_mode;
    float temperature, momentum, omm, std_floor;
    const float* std_floor_p;           // optional device scalar overriding std_floor (graph-stable self.std)
    float* action; float* metrics;
    float* elite_out; float* score_out; float* mean_out; float* std_out;
    int no_pick; float* reward_out;     // tdmpc_cem_iter: stop after the refit; reward mean -> reward_out [B]
    const int* pstatus; int* status;    // the packed buffer's sticky pack status -> the caller's status word
};

DEVI uint32_t f2ord(float v) {
    const uint32_t u = __float_as_uint(v);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
DEVI float ord2f(uint32_t o) { return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o); }
// sort key: ascending key = descending value, then ascending index (torch.topk order for distinct values)
DEVI unsigned long long topk_key(float v, int i) {
    return ((unsigned long long)(~f2ord(v)) << 32) | (unsigned)i;
}
DEVI float key_value(unsigned long long k) { return ord2f(~(uint32_t)(k >> 32)); }

DEVI unsigned long long shfl_xor_u64(unsigned long long v, int m) {
    const unsigned lo = __shfl_xor((unsigned)v, m, 64), hi = __shfl_xor((unsigned)(v >> 32), m, 64);
    return ((unsigned long long)hi << 32) | lo;
}
// ascending bitonic sort of one key per lane across the 64 lanes of a wave
DEVI unsigned long long wave_sort64(unsigned long long key, int lane) {
    for (int k = 2; k <= 64; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            const unsigned long long o = shfl_xor_u64(key, j);
            const bool up = (lane & k) == 0, lower = (lane & j) == 0;
            key = (lower == up) ? (key < o ? key : o) : (key > o ? key : o);
        }
    return key;
}
// lanes hold a bitonic sequence -> ascending
DEVI unsigned long long wave_clean64(unsigned long long key, int lane) {
    for (int j = 32; j > 0; j >>= 1) {
        const unsigned long long o = shfl_xor_u64(key, j);
        key = ((lane & j) == 0) ? (key < o ? key : o) : (key > o ? key : o);
    }
    return key;
}
DEVI float wave_sum(float v) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

DEVI int cem_row(const CemArgs& a, int c) { return c < a.NE ? c : a.pi_base + (c - a.NE); }

__global__ void __launch_bounds__(1024) cem_kernel(const CemArgs a) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int e = blockIdx.x, tid = threadIdx.x, nt = blockDim.x, lane = tid & 63, wave = tid >> 6;
    const int nwv = nt >> 6;
    const int H = a.H, A = a.A, K = a.K, T = a.T, N = a.N;
    const int HA = H * A, HKA = H * K * A;
    const int NL = (T + 63) / 64;                           // sorted lists of 64
    unsigned long long* key = (unsigned long long*)sm;     // [NL*64]
    float* EA = (float*)(key + (size_t)NL * 64);           // [H][K][A]
    float* sc = EA + HKA;                                  // [64]
    float* omean = sc + 64;                                // [HA] mean before the update
    float* smean = omean + 2 * rup(HA, 4);                 // [HA] (one [HA] slot unused)
    float* sstd = smean + rup(HA, 4);                      // [HA]
    int* eidx = (int*)(sstd + rup(HA, 4));                 // [64]
    float* red = (float*)(eidx + 64);                      // [32]
    float* gmean = a.mean + (size_t)e * a.Hmax * A;
    float* gstd = a.stdv + (size_t)e * a.Hmax * A;
    const float* val = a.value + (size_t)e * a.Tw;

    for (int i = tid; i < HA; i += nt) omean[i] = gmean[i];
    // ---- top-K (K <= 64): each wave sorts 64-key lists, then a merge tree keeps the best 64
    for (int l = wave; l < NL; l += nwv) {
        const int i = l * 64 + lane;
        float v = 0.f;
        if (i < T) {
            const int row = cem_row(a, i);
            if (a.qv) {
                const size_t x = (size_t)e * a.Tw + row;
                v = qvalue(a.G[x], a.qv[x], a.qv[a.q_ld + x], a.discH);
                if (a.value_out) a.value_out[((size_t)e * a.I + a.iter) * a.Tw + i] = v;
            } else {
                v = val[row];
                if (a.value_out) a.value_out[((size_t)e * a.I + a.iter) * a.Tw + i] = v;
            }
        }
        const unsigned long long k = i < T ? topk_key(v, i) : ~0ull;
        key[(size_t)l * 64 + lane] = wave_sort64(k, lane);
    }
    __syncthreads();
    for (int stride = 1; stride < NL; stride <<= 1) {
        for (int l = wave * 2 * stride; l < NL; l += nwv * 2 * stride) {
            if (l + stride < NL) {
                const unsigned long long x = key[(size_t)l * 64 + lane];
                const unsigned long long y = key[(size_t)(l + stride) * 64 + 63 - lane];
                key[(size_t)l * 64 + lane] = wave_clean64(x < y ? x : y, lane);
            }
        }
        __syncthreads();
    }
    if (tid < K) eidx[tid] = (int)(key[tid] & 0xffffffffu);
    __syncthreads();
    // ---- elite actions from X_t (sampled rows: prep_kernel; pi rows: the pi pre-rollout)
    for (int base = 0; base < HKA; base += 8 * nt) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int idx = base + tid + u * nt;
            if (idx < HKA) {
                const int t = idx / (K * A), k = (idx / A) % K, c = idx % A;
                v[u] = a.X[(size_t)t * a.x_stride + pidx((size_t)e * a.Tw + cem_row(a, eidx[k]), c, a.Kx)];
            }
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int idx = base + tid + u * nt;
            if (idx < HKA) EA[idx] = v[u];
        }
    }
    // ---- softmax scores over the elites (one wave)
    if (wave == 0) {
        const float v0 = key_value(key[0]);
        float s = 0.f;
        if (lane < K) s = expf(fmul(a.temperature, key_value(key[lane]) - v0));
        const float tot = wave_sum(s);
        s = lane < K ? __fdiv_rn(s, tot) : 0.f;
        if (lane < 64) sc[lane] = s;
        const float tot2 = wave_sum(s);
        if (lane == 0) red[0] = fadd(tot2, 1e-9f);
    }
    __syncthreads();
    const float den = red[0];
    const float std_floor = a.std_floor_p ? *a.std_floor_p : a.std_floor;
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
        const float sd = tclamp(sqrtf(__fdiv_rn(v, den)), std_floor, 2.f);
        const float nm = fadd(fmul(a.momentum, omean[i]), fmul(a.omm, mu));
        smean[i] = nm; sstd[i] = sd;
        gmean[i] = nm; gstd[i] = sd;
        if (a.mean_out) a.mean_out[((size_t)e * a.I + a.iter) * HA + i] = nm;
        if (a.std_out) a.std_out[((size_t)e * a.I + a.iter) * HA + i] = sd;
    }
    if (a.elite_store)
        for (int i = tid; i < HKA; i += nt) a.elite_store[(size_t)e * a.Hmax * a.K * A + i] = EA[i];
    if (!a.final_iter) return;
    // a stale pack (PackHdr.status) poisoned the weights: raise it into the caller's word, NaN the outputs below
    const int pst = a.pstatus ? *a.pstatus : 0;
    if (pst && tid == 0 && a.status)
        __hip_atomic_fetch_or(a.status, pst, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (a.elite_out)
        for (int i = tid; i < HKA; i += nt) a.elite_out[(size_t)e * HKA + i] = EA[i];
    if (a.score_out && tid < K) a.score_out[(size_t)e * K + tid] = sc[tid];
    // estimate_value's reward.mean() of the last iteration: block reduction over the T rows
    {
        float s = 0.f;
        for (int i = tid; i < T; i += nt) s += a.rlast[(size_t)e * a.Tw + cem_row(a, i)];
        s = wave_sum(s);
        if (lane == 0) red[1 + wave] = s;
    }
    __syncthreads();
    if (a.no_pick) {
        if (tid == 0) {
            float rs = 0.f;
            for (int w = 0; w < nwv; ++w) rs += red[1 + w];
            a.reward_out[e] = rs / (float)T;
        }
        return;
    }
    // np.random.choice(K, p=score): float64 cdf of the float32 scores, cdf /= cdf[-1], searchsorted right
    int* jsel = (int*)(red + 20);
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
        *jsel = j;
        float rs = 0.f;
        for (int w = 0; w < nwv; ++w) rs += red[1 + w];
        float cs = 0.f;
        for (int c = 0; c < A; ++c) cs += sstd[c];
        a.metrics[(size_t)e * 2 + 0] = pst ? __builtin_nanf("") : rs / (float)T;   // estimate_value's reward.mean()
        a.metrics[(size_t)e * 2 + 1] = pst ? __builtin_nanf("") : cs / (float)A;   // _std[0].mean()
    }
    __syncthreads();
    const int j = *jsel;
    for (int c = tid; c < A; c += nt) {
        float v = EA[(size_t)j * A + c];
        if (!a.eval_mode) v = fadd(v, fmul(sstd[c], a.eps[(size_t)e * a.eps_env + a.eps_act_off + c]));
        if (pst) v = __builtin_nanf("");
        a.action[(size_t)e * A + c] = v;
        // the reference adds the action noise in place to a view of its stored elites (`a = actions[0]`,
        // tdmpc_icem_similarity_mlp.py:255-259): the kept elite[0][j] carries it
        if (a.elite_store) a.elite_store[(size_t)e * a.Hmax * a.K * A + (size_t)j * A + c] = v;
    }
    for (int i = tid; i < HA; i += nt) a.prev_mean[(size_t)e * H * A + i] = smean[i];
}

// ------------------------------------------------------------------------------------------------ encoder
// TOLD.h (helper.py:119-133) for one observation per workgroup. Weights are stored transposed ([in][out])
// so output j's column is read coalesced; each output's dot product is split over several threads whose
// partial sums meet in LDS, with the loads unrolled. Then the CEM mean/std initialisation
// (tdmpc.py:122-125).
struct EncArgs {
    const float* x; long x_stride; int xdim;    // state obs [B][obs_dim] or flat conv features
    int E, L, Lp;
    const float* w1t; const float* b1;          // null for pixels (x already the flat features)
    const float* w2t; const float* b2;
    float* z0;
    float* mean; float* stdv; const float* prev_mean; int warm, H, A, Hmax;
    const int* warm_flags;                      // optional device [B]: per-env warm start (overrides warm)
    const float* ln_g; const float* ln_b;       // LayerNorm after the first Linear (or null)
    int warm_keep_last;                         // iCEM warm start: mean[-1] = prev_mean[-1] (else 0)
    float init_std;                             // 2 (TDMPC.plan) / 0.5 (iCEM)
};

// out[j] = sum_k wt[k*nout + j] * in[k] for j < nout, partial sums in part[] (nthr floats)
DEVI void enc_matvec(const float* wt, const float* in, int nin, int nout, float* part, int tid, int nt) {
    const int np = nt / nout > 0 ? nt / nout : 1;
    const int j = tid % nout, p = tid / nout;
    float s = 0.f;
    if (p < np && j < nout) {
#pragma unroll 8
        for (int k = p; k < nin; k += np) s += wt[(size_t)k * nout + j] * in[k];
    }
    if (tid < np * nout) part[tid] = s;
}

__global__ void __launch_bounds__(1024) encode_kernel(const EncArgs a) {
    extern __shared__ __attribute__((aligned(16))) float es[];
    const int e = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
    float* x = es;                       // [xdim]
    float* hh = x + rup(a.xdim, 4);      // [E]
    float* part = hh + rup(a.E, 4);      // [nt]
    const float* src = a.x + (size_t)e * a.x_stride;
    for (int i = tid; i < a.xdim; i += nt) x[i] = src[i];
    __syncthreads();
    const float* hin = x;
    int E = a.xdim;
    if (a.w1t) {
        enc_matvec(a.w1t, x, a.xdim, a.E, part, tid, nt);  // E <= 1024 (check_dims)
        __syncthreads();
        float v = 0.f;
        if (tid < a.E) {
            const int np = nt / a.E > 0 ? nt / a.E : 1;
            float s = 0.f;
            for (int p = 0; p < np; ++p) s += part[p * a.E + tid];
            v = s + a.b1[tid];
        }
        if (a.ln_g) {
            // LayerNorm over the E hidden units (biased variance, eps 1e-5), ATen's (x*rstd + -rstd*mean)*g + b
            __syncthreads();
            part[tid] = tid < a.E ? v : 0.f;
            __syncthreads();
            for (int off = nt / 2; off > 0; off >>= 1) {
                if (tid < off) part[tid] += part[tid + off];
                __syncthreads();
            }
            const float mean = part[0] / (float)a.E;
            __syncthreads();
            const float dv = v - mean;
            part[tid] = tid < a.E ? dv * dv : 0.f;
            __syncthreads();
            for (int off = nt / 2; off > 0; off >>= 1) {
                if (tid < off) part[tid] += part[tid + off];
                __syncthreads();
            }
            const float rs = 1.0f / sqrtf(part[0] / (float)a.E + 1e-5f);
            if (tid < a.E) v = fadd(fmul(fadd(fmul(v, rs), -rs * mean), a.ln_g[tid]), a.ln_b[tid]);
        }
        if (tid < a.E) hh[tid] = elu1(v);
        __syncthreads();
        hin = hh;
        E = a.E;
    }
    enc_matvec(a.w2t, hin, E, a.L, part, tid, nt);
    __syncthreads();
    for (int l = tid; l < a.Lp; l += nt) {
        float z = 0.f;
        if (l < a.L) {
            const int np = nt / a.L > 0 ? nt / a.L : 1;
            float s = 0.f;
            for (int p = 0; p < np; ++p) s += part[p * a.L + l];
            z = s + a.b2[l];
        }
        a.z0[(size_t)e * a.Lp + l] = z;
    }
    if (a.mean) {
        const int HA = a.H * a.A;
        const int warm = a.warm_flags ? a.warm_flags[e] : a.warm;
        for (int i = tid; i < HA; i += nt) {
            const int t = i / a.A;
            float mv = 0.f;
            if (warm && t < a.H - 1) mv = a.prev_mean[(size_t)e * HA + i + a.A];  // mean[:-1] = prev[1:]
            if (warm && t == a.H - 1 && a.warm_keep_last) mv = a.prev_mean[(size_t)e * HA + i];  // mean[-1] = prev[-1]
            a.mean[(size_t)e * a.Hmax * a.A + i] = mv;
            a.stdv[(size_t)e * a.Hmax * a.A + i] = a.init_std;
        }
    }
}

// Direct 2-D convolution, stride 2, no padding, + ReLU; uint8 input scaled by 1/255 (NormalizeImg,
// helper.py:99-106; conv stack helper.py:123-127).
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

// LDS-tiled form of the same convolution (+ ReLU, uint8 / 255 on the first layer): a workgroup computes all cout
// channels of `toy` output rows of one env. It stages in LDS the input rows those outputs read (every input
// element converted once) and the layer's weights (packed a second time as [ci][ky][kx][cout], so staging is a
// straight copy and the 8 output channels of a thread's item come from two broadcast float4 LDS reads); each
// thread then owns items of PX consecutive output pixels x 8 channels: PX input reads + 2 weight reads feed
// 8 PX FMAs. Per output the sum runs in the same (ci, ky, kx) order as conv_relu_kernel. Item pixels past the
// row end read in-bounds LDS (the next row / the weight block) and are not stored.
template <int PX>
__global__ void __launch_bounds__(256) conv_tile_kernel(const void* in, int in_u8, long in_bstride, int cin, int hin,
                                                        float* out, long out_bstride, int cout, int hout, int ks,
                                                        int toy, const float* w, const float* b) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int e = blockIdx.y;
    const int oy0 = blockIdx.x * toy;
    const int ny = min(toy, hout - oy0);
    const int rows = 2 * (ny - 1) + ks;                  // input rows read by this tile
    const int iy0 = 2 * oy0;
    float* sIn = smem;                                   // [cin][rows][hin]
    float* sW = smem + ((size_t)cin * (2 * (toy - 1) + ks) * hin + 3) / 4 * 4;   // [cin][ks][ks][cout]
    const int kk = ks * ks;
    for (int i = threadIdx.x; i < cin * rows * hin; i += 256) {
        const int ci = i / (rows * hin), r = (i / hin) % rows, x = i % hin;
        const long g = (long)e * in_bstride + ((long)ci * hin + iy0 + r) * hin + x;
        sIn[i] = in_u8 ? __fdiv_rn((float)((const uint8_t*)in)[g], 255.f) : ((const float*)in)[g];
    }
    for (int i = threadIdx.x; i < cout * cin * kk / 4; i += 256) ((float4*)sW)[i] = ((const float4*)w)[i];
    __syncthreads();
    const int ng = cout / 8, nxq = (hout + PX - 1) / PX, nitem = ny * nxq;
    for (int it = threadIdx.x; it < nitem * ng; it += 256) {
        const int g = it / nitem, p = it % nitem;        // consecutive threads: consecutive pixels, same group
        const int ty = p / nxq, ox0 = (p % nxq) * PX;
        float acc[PX][8];
#pragma unroll
        for (int q = 0; q < PX; ++q)
#pragma unroll
            for (int c = 0; c < 8; ++c) acc[q][c] = 0.f;
        for (int ci = 0; ci < cin; ++ci)
            for (int ky = 0; ky < ks; ++ky) {
                const float* ip = sIn + ((size_t)ci * rows + 2 * ty + ky) * hin + 2 * ox0;
                const float* wp = sW + ((size_t)(ci * ks + ky) * ks) * cout + 8 * g;
                for (int kx = 0; kx < ks; ++kx) {
                    const float4 w0 = *(const float4*)(wp + kx * cout), w1 = *(const float4*)(wp + kx * cout + 4);
#pragma unroll
                    for (int q = 0; q < PX; ++q) {
                        const float v = ip[2 * q + kx];
                        acc[q][0] += w0.x * v; acc[q][1] += w0.y * v; acc[q][2] += w0.z * v; acc[q][3] += w0.w * v;
                        acc[q][4] += w1.x * v; acc[q][5] += w1.y * v; acc[q][6] += w1.z * v; acc[q][7] += w1.w * v;
                    }
                }
            }
#pragma unroll
        for (int q = 0; q < PX; ++q) {
            if (ox0 + q >= hout) break;
            float* op = out + (size_t)e * out_bstride + (size_t)(8 * g) * hout * hout + (size_t)(oy0 + ty) * hout + ox0 + q;
#pragma unroll
            for (int c = 0; c < 8; ++c) op[(size_t)c * hout * hout] = fmaxf(acc[q][c] + b[8 * g + c], 0.f);
        }
    }
}

// candidate actions act [B][H][Ts][A] -> the action columns of rows e * Td + r0 + r of X_t (t < H)
__global__ void scatter_actions_kernel(const float* act, float* X, size_t x_stride, int H, int Ts, int A, int Ap,
                                       int Kx, int B, int Td, int r0) {
    const size_t total = (size_t)B * H * Ts * Ap;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const int c = i % Ap;
        const size_t r = (i / Ap) % Ts;
        const int t = (i / ((size_t)Ap * Ts)) % H;
        const size_t e = i / ((size_t)Ap * Ts * H);
        const float v = c < A ? act[((e * H + t) * Ts + r) * A + c] : 0.f;
        X[(size_t)t * x_stride + pidx(e * Td + r0 + r, c, Kx)] = v;
    }
}

// the inverse: action columns of rows e * Td + r0 + r of X_t -> out [B][H][Ts][A]
__global__ void gather_actions_kernel(const float* X, size_t x_stride, int H, int Ts, int A, int Kx, int B, int Td,
                                      int r0, float* out) {
    const size_t total = (size_t)B * H * Ts * A;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const int c = i % A;
        const size_t r = (i / A) % Ts;
        const int t = (i / ((size_t)A * Ts)) % H;
        const size_t e = i / ((size_t)A * Ts * H);
        out[i] = X[(size_t)t * x_stride + pidx(e * Td + r0 + r, c, Kx)];
    }
}

__global__ void gather_z_kernel(const float* X, int Kx, int Ap, int L, int rows, float* out) {
    const size_t total = (size_t)rows * L;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x)
        out[i] = X[pidx(i / L, Ap + i % L, Kx)];
}

// ------------------------------------------------------------------------------------------------ host side
#define HIPCHK(x)                                                                                 \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) {                                                                   \
            snprintf(g_err, sizeof g_err, "%s:%d %s", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return TDMPC_E_HIP;                                                                   \
        }                                                                                         \
    } while (0)

template <int TM, int TN, int WGM, int WGN, int PRO, int KCH, bool ROLL>
int set_lds_attr() {
    HIPCHK(hipFuncSetAttribute((const void*)linear_kernel<TM, TN, WGM, WGN, PRO, KCH, ROLL>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    return 0;
}

#include "plan1.inc"
#include "wide_step.inc"
#include "wide_heads.inc"

#define FOR_EACH_LINEAR(X)                                                                          \
    X(1, 1, 1, 1, 0, 32, false) X(1, 1, 1, 1, 0, 64, false) X(1, 1, 1, 1, 0, 128, false)              \
    X(1, 2, 1, 1, 0, 32, false) X(1, 2, 1, 1, 0, 64, false) X(1, 2, 1, 1, 0, 128, false)              \
    X(1, 1, 1, 1, 1, 32, false) X(1, 1, 1, 1, 1, 64, false) X(1, 1, 1, 1, 1, 128, false)              \
    X(1, 2, 1, 1, 1, 32, false) X(1, 2, 1, 1, 1, 64, false) X(1, 2, 1, 1, 1, 128, false)              \
    X(2, 2, 2, 2, 1, 1, true)

int init_attrs() {
    static int done = 0;
    if (done) return 0;
    int rc = 0;
#define SET_ATTR(TM, TN, WGM, WGN, PRO, KCH, ROLL) rc |= set_lds_attr<TM, TN, WGM, WGN, PRO, KCH, ROLL>();
    FOR_EACH_LINEAR(SET_ATTR)
#undef SET_ATTR
    HIPCHK(hipFuncSetAttribute((const void*)cem_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    HIPCHK(hipFuncSetAttribute((const void*)plan1_kernel<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    HIPCHK(hipFuncSetAttribute((const void*)plan1_kernel<6>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
#define WIDE_ATTR(G1, NB3, MODE) \
    HIPCHK(hipFuncSetAttribute((const void*)wide_step_kernel<G1, NB3, MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    WIDE_FOR_EACH(WIDE_ATTR)
#undef WIDE_ATTR
#define WIDE_HEADS_ATTR(G1P, NB3P, G1Q, NSTQ) \
    HIPCHK(hipFuncSetAttribute((const void*)wide_heads_kernel<G1P, NB3P, G1Q, NSTQ>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    WIDE_HEADS_FOR_EACH(WIDE_HEADS_ATTR)
#undef WIDE_HEADS_ATTR
    HIPCHK(hipFuncSetAttribute((const void*)qstat_chol_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    HIPCHK(hipFuncSetAttribute((const void*)conv_tile_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    HIPCHK(hipFuncSetAttribute((const void*)conv_tile_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    HIPCHK(hipFuncSetAttribute((const void*)conv_tile_kernel<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
#define LDS_ATTR1(...) \
    HIPCHK(hipFuncSetAttribute((const void*)linear_lds_kernel<__VA_ARGS__>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
#define LDS_ATTR(...) LDS_ATTR1(__VA_ARGS__, true) LDS_ATTR1(__VA_ARGS__, false)
    LDS_ATTR(2, 1, 2, 4, 32) LDS_ATTR(3, 1, 2, 4, 32) LDS_ATTR(1, 1, 2, 2, 32)
#undef LDS_ATTR
#undef LDS_ATTR1
#define CHAIN_ATTR(MODE, TN) \
    HIPCHK(hipFuncSetAttribute((const void*)chain_kernel<MODE, TN>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    CHAIN_ATTR(CH_STEP, 1) CHAIN_ATTR(CH_STEP, 2) CHAIN_ATTR(CH_STEP, 4)
    CHAIN_ATTR(CH_PI, 1) CHAIN_ATTR(CH_PI, 2) CHAIN_ATTR(CH_PI, 4)
    CHAIN_ATTR(CH_Q, 1) CHAIN_ATTR(CH_Q, 2) CHAIN_ATTR(CH_Q, 4)
#undef CHAIN_ATTR
    HIPCHK(hipFuncSetAttribute((const void*)chain_kernel<CH_STEP, 2, 8, 2, X6_D3, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    HIPCHK(hipFuncSetAttribute((const void*)chain_kernel<CH_STEP, 4, 4, 2, 2, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    HIPCHK(hipFuncSetAttribute((const void*)chain_kernel<CH_PI, 2, 8, 2, X6_D3, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    HIPCHK(hipFuncSetAttribute((const void*)chain_kernel<CH_PI, 4, 4, 2, 2, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    HIPCHK(hipFuncSetAttribute((const void*)chain_kernel<CH_Q, 2, 8, 2, X6_D3, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    HIPCHK(hipFuncSetAttribute((const void*)chain_kernel<CH_Q, 4, 4, 2, 2, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    HIPCHK(hipFuncSetAttribute((const void*)chain_kernel<CH_STEP, 1, 16>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    HIPCHK(hipFuncSetAttribute((const void*)chain_kernel<CH_PI, 1, 16>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    HIPCHK(hipFuncSetAttribute((const void*)chain_kernel<CH_Q, 1, 16>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
#define CHAIN16_ATTR(MODE, NT) \
    HIPCHK(hipFuncSetAttribute((const void*)chain16_kernel<MODE, NT>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    CHAIN16_ATTR(CH_STEP, 2) CHAIN16_ATTR(CH_STEP, 4) CHAIN16_ATTR(CH_PI, 2) CHAIN16_ATTR(CH_PI, 4)
    CHAIN16_ATTR(CH_Q, 2) CHAIN16_ATTR(CH_Q, 4)
    HIPCHK(hipFuncSetAttribute((const void*)chain16_kernel<CH_STEP, 4, 4, 4, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    HIPCHK(hipFuncSetAttribute((const void*)chain16_kernel<CH_PI, 4, 4, 4, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    HIPCHK(hipFuncSetAttribute((const void*)chain16_kernel<CH_Q, 4, 4, 4, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
#undef CHAIN16_ATTR
    if (rc) return TDMPC_E_HIP;
    done = 1;
    return 0;
}

// Diagnostic kernel timer (tdmpc_profile_*): when armed on this thread, every linear_kernel launch of the
// selected configuration (cfg id: 1 = latency 32x32 tile, 2 = latency 32x64 tile, 3 = throughput 128x128
// tile; 0 = any) with K == N == kdim (if kdim > 0) and M == rows (if rows > 0) is bracketed by HIP events on its stream, and its
// algorithmic FLOPs (2*M*N*K per problem) are recorded. bench.py uses it for the dominant kernel's roofline.
struct Profiler {
    int armed = 0, cfg = 0, pro = -1, n = 0, cap = 0, kdim = 0, rows = 0;
    hipEvent_t* ev = nullptr;
    double flops = 0.0;
    char kernel[128] = "";   // the last timed launch's kernel (tdmpc_profile_kernel)
};
thread_local Profiler g_prof;

// Launch geometry chosen for a linear layer.
struct LinCfg {
    int id;      // 1 = LAT1 (32x32, K split), 2 = LAT2 (32x64, K split), 3 = THR (128x128, full K)
    int C;       // workgroup tile columns
    int bw;      // row-reduction block width (64 or 32)
};

int thr_rows() { return 4096; }

// Tile choice by shape (tools/mb/mb_linear.hip "sweep" on MI355X): the LDS-staged throughput tiles from
// thr_rows() rows on; below that the K-split latency tiles, 32x64 where K and N are wide enough to feed
// its 8 waves (512x512 hidden layers from 512 rows, the 100-wide latent layer from 2048 rows) or where the
// epilogue needs 64-column row blocks (wide64: LayerNorm moments are kept per 64 columns).
LinCfg pick_cfg(int M, int nmax, int K, int wide64) {
    if (M >= thr_rows() && nmax >= 256 && K >= 64) return LinCfg{3, 128, 64};
    if (wide64 || (nmax >= 256 ? (K >= 256 && M >= 512) : M >= 2048)) return LinCfg{2, 64, 64};
    return LinCfg{1, 32, 32};
}

template <int TM, int TN, int WGM, int WGN, int PRO, int KCH, bool ROLL>
int launch_lin_t(const LinArgs& a, int nprob, int nmax, int cfg_id, hipStream_t s) {
    constexpr int R = 32 * TM * WGM, C = 32 * TN * WGN;
    // ROLL: KCH is the number of K splits (1 or 2), each wave group rolls over K/KCH
    const int KS = ROLL ? KCH : (a.K + KCH - 1) / KCH;
    LinArgs b = a;
    b.kch = ROLL ? (int)rup((a.K + KCH - 1) / KCH, 8) : KCH;
    dim3 grid((a.M + R - 1) / R, (nmax + C - 1) / C, nprob);
    dim3 block(64 * WGM * WGN * KS);
    const size_t lds = ((size_t)KS * R * (C + 4) + 2 * C + (size_t)R * std::max(a.rpart_nt, 1)) * 4;
    Profiler& pf = g_prof;
    const bool prof = pf.armed && (pf.cfg == 0 || pf.cfg == cfg_id) && (pf.pro < 0 || pf.pro == PRO) &&
                      pf.n + 2 <= pf.cap && (pf.kdim == 0 || (a.K == pf.kdim && nmax == pf.kdim)) &&
                      (pf.rows == 0 || a.M == pf.rows);
    if (prof) HIPCHK(hipEventRecord(pf.ev[pf.n], s));
    hipLaunchKernelGGL((linear_kernel<TM, TN, WGM, WGN, PRO, KCH, ROLL>), grid, block, lds, s, b);
    HIPCHK(hipGetLastError());
    if (prof) {
        HIPCHK(hipEventRecord(pf.ev[pf.n + 1], s));
        pf.n += 2;
        for (int q = 0; q < nprob; ++q) pf.flops += 2.0 * a.M * std::min(a.p[q].N, nmax) * a.K;
    }
    return 0;
}

template <int TM, int TN, int WGM, int WGN, int KT>
int launch_lds_t(const LinArgs& a, int nprob, int nmax, hipStream_t s) {
    constexpr int R = 32 * TM * WGM, C = 32 * TN * WGN;
    constexpr int BUF = (R / 32 + C / 32) * KT * 32;
    static_assert(C % 64 == 0, "row reductions work on 64-column blocks");
    dim3 grid((a.M + R - 1) / R, (nmax + C - 1) / C, nprob);
    for (int q = 0; q < nprob; ++q)
        if (a.p[q].epi != EPI_ELU && a.p[q].epi != EPI_ELU_DOT && a.p[q].epi != EPI_LNSTATS) {
            snprintf(g_err, sizeof g_err, "LDS tile: unsupported epilogue %d", a.p[q].epi);
            return TDMPC_E_DIMS;
        }
    const size_t lds = ((size_t)3 * BUF + 2 * C + (size_t)R * (C / 32) * 2) * 4;
    Profiler& pf = g_prof;
    const bool prof = pf.armed && (pf.cfg == 0 || pf.cfg == 3) && (pf.pro <= 0) && pf.n + 2 <= pf.cap &&
                      (pf.kdim == 0 || (a.K == pf.kdim && nmax == pf.kdim)) && (pf.rows == 0 || a.M == pf.rows);
    if (prof) HIPCHK(hipEventRecord(pf.ev[pf.n], s));
    const dim3 block(64 * WGM * WGN);
    if (a.K % KT == 0) hipLaunchKernelGGL((linear_lds_kernel<TM, TN, WGM, WGN, KT, true>), grid, block, lds, s, a);
    else hipLaunchKernelGGL((linear_lds_kernel<TM, TN, WGM, WGN, KT, false>), grid, block, lds, s, a);
    HIPCHK(hipGetLastError());
    if (prof) {
        HIPCHK(hipEventRecord(pf.ev[pf.n + 1], s));
        pf.n += 2;
        for (int q = 0; q < nprob; ++q) pf.flops += 2.0 * a.M * std::min(a.p[q].N, nmax) * a.K;
    }
    return 0;
}

int num_cus() {
    static int n = 0;
    if (!n) {
        int dev = 0, v = 0;
        if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
            n = v;
        else
            n = 256;
    }
    return n;
}

// LDS-staged throughput tiles: 128x128 with 8 waves (64x32 each, 2 waves per SIMD) by default, 192x128
// (8 waves of 96x32) or 64x64 (4 waves of 32x32) when the work per CU says so.
int launch_lds(const LinArgs& a, int nprob, int nmax, hipStream_t s) {
    const int ctiles128 = (nmax + 127) / 128, rtiles = (a.M + 127) / 128;
    {   // Tile by the work of the busiest CU: ceil(WGs / CUs) x tile area, over the tile's efficiency.
        // 192x128 when 128x128 would need a second, partly idle round (6144 rows x 2 problems: 256 WGs
        // instead of 384); 64x64 (4 waves, 4 resident per CU) when 128x128 leaves CUs idle.
        const int cus = num_cus();
        const long w128 = (long)rtiles * ctiles128 * nprob, w192 = (long)((a.M + 191) / 192) * ctiles128 * nprob;
        const long w64 = (long)((a.M + 63) / 64) * ((nmax + 63) / 64) * nprob;
        const double c128 = (double)((w128 + cus - 1) / cus) * 128 * 128;
        const double c192 = (double)((w192 + cus - 1) / cus) * 192 * 128 / 1.05;
        const long r64 = (w64 + cus - 1) / cus;
        const double c64 = (double)r64 * 64 * 64 / (r64 >= 2 ? 0.8 : 0.4);
        if (c192 < c128 && c192 <= c64) return launch_lds_t<3, 1, 2, 4, 32>(a, nprob, nmax, s);
        if (c64 < c128) return launch_lds_t<1, 1, 2, 2, 32>(a, nprob, nmax, s);
    }
    return launch_lds_t<2, 1, 2, 4, 32>(a, nprob, nmax, s);
}

// Launch one fused linear layer with the configuration pick_cfg selects.
int launch_lin(const LinArgs& a, int nprob, int nmax, int wide64, int pro, hipStream_t s) {
    if (a.M <= 0) return 0;
    if (a.K % 8) { snprintf(g_err, sizeof g_err, "bad K %d", a.K); return TDMPC_E_DIMS; }
    const LinCfg cfg = pick_cfg(a.M, nmax, a.K, wide64);
    if (cfg.id == 3) {   // (the register-direct 128-row variants of rounds 1-2 measured slower: git history)
        if (pro == PRO_PLAIN) return launch_lds(a, nprob, nmax, s);
        return launch_lin_t<2, 2, 2, 2, 1, 1, true>(a, nprob, nmax, 3, s);
    }
    int kch = 32;
    if ((a.K + 31) / 32 > 8) kch = 64;
    if ((a.K + 63) / 64 > 8) kch = 128;
    if ((a.K + kch - 1) / kch > 8) { snprintf(g_err, sizeof g_err, "bad K %d", a.K); return TDMPC_E_DIMS; }
    const int tn = cfg.id == 2 ? 2 : 1;
#define DISPATCH(TN_, PRO_, KCH_) \
    if (tn == TN_ && pro == PRO_ && kch == KCH_) return launch_lin_t<1, TN_, 1, 1, PRO_, KCH_, false>(a, nprob, nmax, cfg.id, s);
    DISPATCH(1, 0, 32) DISPATCH(1, 0, 64) DISPATCH(1, 0, 128)
    DISPATCH(2, 0, 32) DISPATCH(2, 0, 64) DISPATCH(2, 0, 128)
    DISPATCH(1, 1, 32) DISPATCH(1, 1, 64) DISPATCH(1, 1, 128)
    DISPATCH(2, 1, 32) DISPATCH(2, 1, 64) DISPATCH(2, 1, 128)
#undef DISPATCH
    return TDMPC_E_DIMS;
}

// ---- chain path (chain_kernel / chain16_kernel): on the auto path used for launches of at least chain_wgs()
// 32-row-block equivalents x problems (TDMPC_CHAIN_WGS, default 64, 0 disables). Narrow launches run on 16-row
// blocks (chain_rb), so from 64 32-row blocks on they still spread over 128+ CUs; below that the layered
// GEMMs, whose K-split tiles spread the same rows over more CUs, finish first. Measured on MI355X (humanoid
// plan, round-1 run): threshold 64 vs 128: B = 2 envs 1.65 vs 1.87 ms, B = 4 1.88 vs 1.98 ms; 32 loses
// at one env (1.56 vs 1.38 ms).
int chain_wgs() { return 64; }

// Shapes the chain kernel supports: M = 256 * TN (TN = 1, 2, 4); the last layer's (block, K-part) items
// (<= 16) fit the activation block as 32x32 partial tiles.
bool chain_shape_ok(const Layout& w) {
    const int M = w.M;
    if (M % 256 || M / 256 > 4 || M / 256 == 3) return false;
    const size_t hfl = (size_t)std::max(w.Kx, M) * 32;
    for (int n3 : {w.Lr, w.Ar}) {
        const int nb3 = n3 / 32, ks = nb3 >= 8 ? 1 : 8 / nb3, items = nb3 * ks;
        if (items > 16 || (size_t)items * 1024 > hfl || (M / 8) % ks) return false;
    }
    // the pi noise is prefetched one quad per thread: Ap/4 * 32 <= 512
    if (w.Ap / 4 * 32 > 512) return false;
    const int pmax = std::max(chain_param_floats(CH_Q, M, 0), chain_param_floats(CH_STEP, M, std::max(w.Lr, w.Ar)));
    return (hfl + 512 + pmax) * 4 <= 160 * 1024;
}

// Shapes chain16_kernel supports: M = 128 * NT (NT = 2, 4); last-layer items (16-column tile, K part) <= 32.
bool chain16_shape_ok(const Layout& w) {
    const int M = w.M;
    if (M != 256 && M != 512) return false;
    const size_t hfl = (size_t)std::max((int)rup(w.Kx, 32), M) * 16;
    for (int n3 : {w.Lr, w.Ar}) {
        const int nb3 = n3 / 16, ks = nb3 >= 8 ? 1 : 8 / nb3, items = nb3 * ks;
        if (items > 32 || (size_t)items * 256 > hfl || (M / 16) % ks) return false;
    }
    if (w.Ap / 4 * 16 > 512) return false;
    const int pmax = std::max(chain_param_floats(CH_Q, M, 0), chain_param_floats(CH_STEP, M, std::max(w.Lr, w.Ar)));
    return (hfl + 256 + pmax) * 4 <= 64 * 1024;
}

// Algorithmic MACs per row of a chain launch (with the real widths, not the padded ones):
// CH_STEP d + R = 2 (K1 M + M^2) + M L + M, CH_PI K1 M + M^2 + M A, CH_Q 2 (K1 M + M^2 + M).
double chain_macs_per_row(int mode, const ChainArgs& a, int nprob) {
    const double K1 = a.k1_alg > 0 ? a.k1_alg : a.K1, M = a.M;   // unpadded widths: algorithmic MACs
    if (mode == CH_STEP) return 2 * (K1 * M + M * M) + M * a.nvalid + M;
    if (mode == CH_PI) return K1 * M + M * M + M * a.nvalid;
    return nprob * (K1 * M + M * M + M);
}

int launch_chain(int mode, const ChainArgs& a0, int nprob, hipStream_t s) {
    if (a0.rows <= 0) return 0;
    ChainArgs a = a0;
    if (a.rb != 32) a.z0c = nullptr;   // (chain16 runs the full first layer)
    const int nw = a.rb == 16 ? 8 : a.nw;
    const size_t lds = ((size_t)a.hfl + (a.rb == 16 ? 256 : 64 * nw) + chain_param_floats(mode, a.M, a.n3)) * 4;
    const int nblk = (a.rows + a.rb - 1) / a.rb;
    // (the problems along blockIdx.y: co-resident same-head workgroups on a CU share the weight stream through its L1;
    // interleaving the heads along x, or grouping them by XCD, measured 3-6 % slower -- round 1, git history)
    a.il = 0;
    const dim3 grid(nblk, nprob), block(64 * nw);
    const int tn = a.M / (32 * nw);
    // diagnostic timer (tdmpc_profile_begin cfg 4 + mode): HIP events around matching chain launches
    Profiler& pf = g_prof;
    // (t = 0 steps with the z0c first layer do less than the algorithmic work: not timed, so the roofline's
    // achieved rate is not flattered by them)
    const bool prof = pf.armed && pf.cfg == 4 + mode && pf.n + 2 <= pf.cap && (pf.rows == 0 || a.rows == pf.rows) &&
                      a.z0c == nullptr;
    if (prof) {
        static const char* mname[3] = {"CH_STEP", "CH_PI", "CH_Q"};
        snprintf(pf.kernel, sizeof pf.kernel, "%s<%s%s>", a.rb == 16 ? "chain16_kernel" : "chain_kernel", mname[mode],
                 a.x6 ? ", x6" : ", f32");
        HIPCHK(hipEventRecord(pf.ev[pf.n], s));
    }
    if (a.rb == 16) {
        const int nt = a.M / 128;
#define CHAIN16_LAUNCH(MODE, NT) \
        if (mode == MODE && nt == NT) { \
            if (a.x6 && NT == 4) hipLaunchKernelGGL((chain16_kernel<MODE, 4, 4, 4, 1>), grid, block, lds, s, a); \
            else hipLaunchKernelGGL((chain16_kernel<MODE, NT>), grid, block, lds, s, a); \
            HIPCHK(hipGetLastError()); \
            if (prof) { \
                HIPCHK(hipEventRecord(pf.ev[pf.n + 1], s)); \
                pf.n += 2; \
                pf.flops += 2.0 * a.rows * chain_macs_per_row(mode, a, nprob); \
            } \
            return 0; \
        }
        CHAIN16_LAUNCH(CH_STEP, 2) CHAIN16_LAUNCH(CH_STEP, 4) CHAIN16_LAUNCH(CH_PI, 2) CHAIN16_LAUNCH(CH_PI, 4)
        CHAIN16_LAUNCH(CH_Q, 2) CHAIN16_LAUNCH(CH_Q, 4)
#undef CHAIN16_LAUNCH
        snprintf(g_err, sizeof g_err, "chain16: unsupported mode %d / M %d", mode, a.M);
        return TDMPC_E_DIMS;
    }
#define CHAIN_LAUNCH(MODE, TN) \
    if (mode == MODE && tn == TN) { \
        if (a.x6 == 3 && TN == 4 && nw == 4) hipLaunchKernelGGL((chain_kernel<MODE, 4, 4, 2, 2, 1>), grid, block, lds, s, a); \
        else if (a.x6 && TN == 2) hipLaunchKernelGGL((chain_kernel<MODE, 2, 8, 2, X6_D3, 1>), grid, block, lds, s, a); \
        else if (nw == 16 && TN == 1) hipLaunchKernelGGL((chain_kernel<MODE, 1, 16>), grid, block, lds, s, a); \
        else hipLaunchKernelGGL((chain_kernel<MODE, TN>), grid, block, lds, s, a); \
        HIPCHK(hipGetLastError()); \
        if (prof) { \
            HIPCHK(hipEventRecord(pf.ev[pf.n + 1], s)); \
            pf.n += 2; \
            pf.flops += 2.0 * a.rows * chain_macs_per_row(mode, a, nprob); \
        } \
        return 0; \
    }
    CHAIN_LAUNCH(CH_STEP, 1) CHAIN_LAUNCH(CH_STEP, 2) CHAIN_LAUNCH(CH_STEP, 4)
    CHAIN_LAUNCH(CH_PI, 1) CHAIN_LAUNCH(CH_PI, 2) CHAIN_LAUNCH(CH_PI, 4)
    CHAIN_LAUNCH(CH_Q, 1) CHAIN_LAUNCH(CH_Q, 2) CHAIN_LAUNCH(CH_Q, 4)
#undef CHAIN_LAUNCH
    snprintf(g_err, sizeof g_err, "chain: unsupported mode %d / M %d", mode, a.M);
    return TDMPC_E_DIMS;
}

LinArgs args0() {
    LinArgs a;
    memset(&a, 0, sizeof a);
    a.amap = {1 << 30, 0, 0};
    a.cmap = {1 << 30, 0, 0};
    return a;
}

// The planner's per-call context.
struct Ctx {
    const tdmpc_dims* d; Layout w; Work k; const float* pw; hipStream_t s;
    int B, N, P, T, H, A, M, Kx;
    int path;        // TDMPC_PATH_*
    long eps_env, eps_cem_off, eps_iter, eps_term_off, eps_act_off;
    // split-step finish deferred into the next step's launch (step_next(..., defer = 1))
    mutable int split_pend = 0, split_par = 0, split_first = 0;
    mutable float split_disc = 0.f;
    mutable RowMap split_map = {1 << 30, 0, 0};
    mutable int split_rows = 0, split_t = 0;
    int z0c_ready = 0;   // k.z0c holds this call's per-env first-layer z0 shares (tdmpc_plan)
    int fold_ok = 0;     // tdmpc_plan: the sampled rows' rollout runs wide at every t with the folded first layer
    int fold_heads = 0;  // ... and their terminal pi / Q read h2_{H-1} through folded first layers (no z_H formed)
    int fold_policy = 0; // ... and the policy rows' pre-rollout carries h2 too (chain kernels, folded first layers)
};

float* Xt(const Ctx& c, int t) { return c.k.X + (size_t)t * c.k.x_stride; }
const unsigned short* x6p(const Ctx& c, int i) { return (const unsigned short*)(c.pw + c.w.x6[i]); }
// Per-head thresholds (TDMPC_CHAIN_WGS_STEP / _PI / _Q override). The Q heads' layered form is four launches
// (two GEMMs with LayerNorm partial moments, the LN+tanh pass, the value kernel), so the chain form wins from half
// the step threshold: one env's 768 terminal rows 1.42 -> 1.32 ms per plan (round-1 run); the step and pi
// heads keep chain_wgs() (lower thresholds measured slower for them).
enum { CK_STEP = 0, CK_PI = 1, CK_Q = 2 };
int chain_wgs_kind(int kind) {
    static int v[3] = {-2, -2, -2};
    if (v[kind] == -2) {
        static const char* names[3] = {"TDMPC_CHAIN_WGS_STEP", "TDMPC_CHAIN_WGS_PI", "TDMPC_CHAIN_WGS_Q"};
        const char* e = getenv(names[kind]);
        v[kind] = e ? atoi(e) : -1;
    }
    if (v[kind] >= 0) return v[kind];
    return kind == CK_Q ? chain_wgs() / 2 : chain_wgs();
}

bool use_chain(const Ctx& c, int rows, int nprob, int kind) {
    if (c.path == TDMPC_PATH_LAYERED || c.path == TDMPC_PATH_SPLIT || c.path == TDMPC_PATH_SPLIT_X6 || !chain_shape_ok(c.w))
        return false;
    const int th = chain_wgs_kind(kind);
    return c.path != TDMPC_PATH_AUTO || (th > 0 && (rows + 31) / 32 * nprob >= th);
}

// 16-wave 32-row chain workgroups: M = 512 (TN = 1), last-layer items <= 32 within the activation block.
bool chain_nw16_ok(const Layout& w) {
    if (w.M != 512) return false;
    const size_t hfl = (size_t)std::max((int)rup(w.Kx, 16), w.M) * 32;
    for (int n3 : {w.Lr, w.Ar}) {
        const int nb3 = n3 / 32, ks = nb3 >= 16 ? 1 : 16 / nb3, items = nb3 * ks;
        if (items > 32 || (size_t)items * 1024 > hfl || (w.M / 8) % ks) return false;
    }
    const int pmax = std::max(chain_param_floats(CH_Q, w.M, 0), chain_param_floats(CH_STEP, w.M, std::max(w.Lr, w.Ar)));
    return (hfl + 1024 + pmax) * 4 <= 160 * 1024;
}

// Waves per 32-row chain workgroup (TDMPC_CHAIN_NW: 8 or 16; 16 needs M = 512).
int chain_nw() { return 8; }

// x6 chain kernels (fp32 products from a three-way bf16 split, chain_kernel<..., X6>) for 32-row chain launches:
// forced by TDMPC_PATH_CHAIN_X6, the default of the auto / chain paths (TDMPC_X6=0 turns it off there); the
// chain32 / chain16 paths keep the exact f32 MFMA. M = 512 only (the one instantiated width). Measured on MI355X
// (humanoid-run, round-1 run): 8.89 -> 6.52 ms per B = 32 plan, 3.03 -> 2.19 ms at B = 8.
// Returns the x6 mode of a chain launch (0 = f32 MFMA; 1 = 8-wave workgroups, activations split as read; 3 = mode 1
// on 4-wave workgroups of 128 columns per wave, the default: the per-wave split serves
// twice the MFMAs -- measured 6.37 vs 6.60 ms per B = 32 plan, 2.23 vs 2.28 at B = 8, round-1 run). TDMPC_X6
// picks the mode, 0 turns x6 off on the auto / chain paths.
int use_x6(const Ctx& c) {
    if (c.w.M != 512) return 0;
    static int en = -1;
    if (en < 0) {
        const char* e = getenv("TDMPC_X6");
        en = e ? atoi(e) : 3;
    }
    if (en == 2) en = 3;   // (mode 2, the split planes in LDS, retired)
    if (c.path == TDMPC_PATH_CHAIN_X6 || c.path == TDMPC_PATH_WIDE) return en == 1 || en == 3 ? en : 3;
    if (c.path == TDMPC_PATH_SPLIT_X6) return 1;
    return (c.path == TDMPC_PATH_AUTO || c.path == TDMPC_PATH_CHAIN) ? en : 0;
}

// Row block of a chain launch. Auto: 32-row blocks once they occupy more than half the CUs (their weight
// fragments serve twice the rows; measured on MI355X, humanoid: 57.5 vs 61 us for the 256-workgroup B = 8
// step, 99 vs 114 us at B = 16, and 16-row blocks lose on the 192-workgroup pi launch too), else 16-row
// blocks, which double the workgroups of a narrow launch (B = 4 step: 36.7 us vs 56 us on 128 32-row
// workgroups). TDMPC_CHAIN_RB forces 16 or 32 for experiments.
int chain_rb(const Ctx& c, int rows, int nprob) {
    if (!chain16_shape_ok(c.w) || c.path == TDMPC_PATH_CHAIN32 || c.path == TDMPC_PATH_CHAIN_X6 ||
        c.path == TDMPC_PATH_WIDE)
        return 32;
    if (c.path == TDMPC_PATH_CHAIN16) return 16;
    return (rows + 31) / 32 * nprob > num_cus() / 2 ? 32 : 16;
}

ChainArgs chain0(const Ctx& c, int rows, RowMap map, int t, int K1, int q1, int nprob) {
    ChainArgs a;
    memset(&a, 0, sizeof a);
    a.rows = rows; a.M = c.M; a.K1 = K1; a.q1 = q1; a.amap = map;
    a.k1_alg = K1 == c.Kx ? c.w.L + c.w.A : c.w.L;   // TOLD.next / Q take [z, a]; pi takes z
    a.rb = chain_rb(c, rows, nprob);
    a.x6 = a.rb == 32 ? use_x6(c) : (use_x6(c) ? 1 : 0);   // 16-row blocks: chain16_kernel<..., X6 = 1>
    // x6 mode 3: 4-wave workgroups, 128 columns per wave (the per-wave split amortised over twice the MFMAs); the pi
    // head's noise prefetch (two quads per thread) needs Ap / 4 * 32 <= 512, and the last layer's 32-column blocks
    // (at most four per wave) Lr, Ar <= 512; otherwise mode 1
    if (a.x6 == 3 && (c.w.Ap / 4 * 32 > 512 || std::max(c.w.Lr, c.w.Ar) > 4 * 4 * 32)) a.x6 = 1;
    a.nw = a.x6 == 3 ? 4 : a.rb == 32 && !a.x6 && chain_nw() == 16 && chain_nw16_ok(c.w) ? 16 : 8;
    // activation block: fp32 [K/4][rb][4]
    a.hfl = std::max((int)rup(c.Kx, 32), c.M) * a.rb;
    a.X = Xt(c, t); a.x_ts = (long)c.Kx * 32;
    return a;
}
Opnd xop(const Ctx& c, int t, int q0) { return Opnd{Xt(c, t), (long)c.Kx * 32, q0}; }
Outp xout(const Ctx& c, int t, int q0) { return Outp{Xt(c, t), (long)c.Kx * 32, q0}; }
Opnd hop(const float* H, const Ctx& c, int q0) { return Opnd{H, (long)2 * c.M * 32, q0}; }
Outp hout(float* H, const Ctx& c, int q0) { return Outp{H, (long)2 * c.M * 32, q0}; }
Opnd wop(const Ctx& c, size_t off, int K) { return Opnd{c.pw + off, (long)K * 32, 0}; }

// split_step_kernel for a step launch: auto where the chain kernels are not used (narrow launches, TDMPC_SPLIT=0
// disables), forced by TDMPC_PATH_SPLIT; M = 512 (NT = 4), the rows fit the partial buffers, LDS fits.
bool use_split(const Ctx& c, int rows) {
    const Layout& w = c.w;
    if (w.M != 512 || rows > c.k.split_rows || (size_t)split_lds_floats(w.Kx, w.M) * 4 > 64 * 1024) return false;
    if (c.path == TDMPC_PATH_SPLIT || c.path == TDMPC_PATH_SPLIT_X6) return true;
    // auto: only while the first layer, repeated per slice, stays cheap next to the slice of the M x M layer
    // (humanoid-run L512: K1 = 536 made the one-env plan 1.3x slower than the layered path)
    if (c.path != TDMPC_PATH_AUTO || (int)rup(w.Kx, 16) > w.M / 2) return false;
    return !use_chain(c, rows, 2, CK_STEP);
}

// split_step_kernel for the pi head (grid z = 1: no reward head; its finish is split_pi_finish_kernel).
bool use_split_pi(const Ctx& c, int rows) {
    const Layout& w = c.w;
    if (w.M != 512 || rows > c.k.split_rows || (size_t)split_lds_floats(w.Lp, w.M) * 4 > 64 * 1024) return false;
    if (c.path == TDMPC_PATH_SPLIT || c.path == TDMPC_PATH_SPLIT_X6) return true;
    if (c.path != TDMPC_PATH_AUTO || (int)rup(w.Lp, 16) > w.M / 2) return false;
    return !use_chain(c, rows, 1, CK_PI);
}

// One TOLD.next step (tdmpc.py:34-37) for `rows` logical rows mapped onto X rows, plus the return update
// of estimate_value (:88-90). X_t holds the rows' [a|z] (prep_kernel wrote the sampled actions and z0).
// The split step's separate finish launch: partial sums of step t into X_{t+1}'s latent columns and the return.
int split_finish(const Ctx& c, int t, int rows, RowMap map, const float* zp, const float* rp, float disc, int first,
                 int last) {
    const Layout& w = c.w;
    SplitFinishArgs f;
    memset(&f, 0, sizeof f);
    f.rows = rows; f.amap = map; f.zpart = zp; f.rpart = rp; f.prow = c.k.split_rows;
    f.n3 = w.Lr; f.L = w.L; f.Lp = w.Lp; f.b3d = c.pw + w.b3d; f.b3r = c.pw + w.b3r;
    f.Xo = Xt(c, t + 1); f.x_ts = (long)c.Kx * 32; f.out_q0 = w.Ap / 4;
    f.G = c.k.G; f.rlast = c.k.rlast; f.disc = disc; f.first = first; f.last = last;
    const long nth = (long)rows * (w.Lp / 4 + 1);
    hipLaunchKernelGGL(split_finish_kernel, dim3((unsigned)((nth + 255) / 256)), dim3(256), 0, c.s, f);
    HIPCHK(hipGetLastError());
    return 0;
}

// A deferred split finish that no later step launch picked up (a non-split launch comes next): run it now.
int flush_split(const Ctx& c) {
    if (!c.split_pend) return 0;
    c.split_pend = 0;
    const int par = 1 - c.split_par;
    const size_t zs = (size_t)SPLIT_S * c.k.split_rows * std::max(c.w.Lr, c.w.Ar), rs = (size_t)SPLIT_S * c.k.split_rows;
    return split_finish(c, c.split_t, c.split_rows, c.split_map, c.k.zpart + par * zs, c.k.rpart_s + par * rs,
                        c.split_disc, c.split_first, 0);
}

// z0c split point: the action columns rounded up to a 16-k group (TDMPC_Z0C=0 disables the split)
int z0c_k1c(const Ctx& c) { return (int)rup(c.w.Ap, 16); }
bool z0c_eligible(const Ctx& c) {
    static const int v = [] { const char* e = getenv("TDMPC_Z0C"); return e ? atoi(e) : 1; }();
    return v && z0c_k1c(c) < (int)rup(c.Kx, 16);
}
int z0c_launch(const Ctx& c) {
    hipLaunchKernelGGL(z0c_kernel, dim3(c.B, 2, (c.M + 255) / 256), dim3(256), 0, c.s, c.pw + c.w.w1x, c.pw + c.w.b1x,
                       c.k.z0, c.Kx, c.w.Ap, c.w.Lp, z0c_k1c(c), c.M, c.k.z0c);
    HIPCHK(hipGetLastError());
    return 0;
}

unsigned long long* g_p1_stamps = nullptr;   // tdmpc_debug_plan1_stamps (diagnostic; also the wide kernel's stamps)

// ---- the wide step kernel (wide_step.inc) for TOLD.next launches with >= one 128-row block per CU and head (B >= 32
// envs at N = 512; TDMPC_WIDE=0 turns it off, TDMPC_PATH_WIDE forces it at every width it supports)
int wide_g1(const Ctx& c, bool z0c) {   // first-layer 32-k groups the kernel runs
    return (int)rup(z0c ? z0c_k1c(c) : c.Kx, 32) / 32;
}
bool use_wide(const Ctx& c, int rows, const RowMap& map, bool z0c) {
    static const int en = [] { const char* e = getenv("TDMPC_WIDE"); return e ? atoi(e) : 1; }();
    if (c.w.M != 512 || !use_x6(c) || !num_cus()) return false;
    if (c.path != TDMPC_PATH_AUTO && c.path != TDMPC_PATH_CHAIN && c.path != TDMPC_PATH_WIDE) return false;
    if (c.path != TDMPC_PATH_WIDE && !en) return false;
    if (rows % 16 || map.G % 16 || map.S % 16 || map.O % 16) return false;   // a wave's 16 rows in one X panel block
    if (z0c && map.G % 128) return false;   // the per-env first-layer bias is per workgroup
    const int g1 = wide_g1(c, z0c), nb3 = (int)rup(c.w.L, 16) / 16;
    const bool inst = (g1 <= 5 && (nb3 == 4 || nb3 == 7)) || (nb3 == 32 && (g1 == 1 || g1 == 17));
    if (!inst) return false;
    return c.path == TDMPC_PATH_WIDE || (rows + 127) / 128 * 2 >= num_cus();
}
// the folded first layer for a plan's sampled-row rollout (latent_dim == mlp_dim; TDMPC_FOLD=0 turns it off)
bool fold_on() {
    static const int v = [] { const char* e = getenv("TDMPC_FOLD"); return e ? atoi(e) : 1; }();
    return v != 0;
}
// fold: this launch is a step of a rollout whose every step runs here with the folded layout (Ctx::fold_ok): steps
// t >= 1 read the previous step's h2 through the folded first layer, every step but the last stores h2 instead of z'
int launch_wide(const Ctx& c, int t, int rows, RowMap map, float disc, int first, int last, bool z0c, bool fold = false) {
    const Layout& w = c.w;
    const int M = c.M;
    WideArgs a;
    memset(&a, 0, sizeof a);
    auto q6 = [&](int i) { return (const unsigned short*)(c.pw + w.x6q[i]); };
    a.g1s = (int)(rup(c.Kx, 32) / 32);
    const size_t rb1 = (size_t)(M / 16) * a.g1s * 1536;   // bf16 per M rows of x6q W1
    const bool fold_in = fold && t >= 1 && !z0c, outh = fold && (!last || c.fold_heads);
    a.p[0].X1 = q6(X6_W1X); a.p[1].X1 = q6(X6_W1X) + rb1;
    a.p[0].X2 = q6(X6_W2D); a.p[1].X2 = q6(X6_W2R);
    a.p[0].b1 = c.pw + w.b1x; a.p[1].b1 = c.pw + w.b1x + M;
    if (fold_in) {
        const unsigned short* xf = (const unsigned short*)(c.pw + w.x6qw);
        a.p[0].X1 = xf; a.p[1].X1 = xf + rb1;
        a.p[0].b1 = c.pw + w.bfw; a.p[1].b1 = c.pw + w.bfw + M;
    }
    a.p[0].b2 = c.pw + w.b2d; a.p[1].b2 = c.pw + w.b2r;
    a.p[1].w3v = c.pw + w.w3r; a.p[1].b3v = c.pw + w.b3r;
    a.X3 = q6(X6_W3D); a.b3 = c.pw + w.b3d; a.nvalid = w.L; a.nstore = w.Lp;
    a.rows = rows; a.nrb = (rows + 127) / 128; a.amap = map;
    a.X = Xt(c, t); a.x_ts = (long)c.Kx * 32;
    a.kq = (z0c ? z0c_k1c(c) : c.Kx) / 4;
    a.Xo = Xt(c, t + 1); a.out_q0 = w.Ap / 4;
    a.G = c.k.G; a.rlast = c.k.rlast; a.disc = disc; a.first = first; a.last = last;
    if (z0c) { a.z0c = c.k.z0c; a.z0_G = map.G; }
    a.stamps = g_p1_stamps;   // (read only by a -DWS_STAMPS diagnostic build)
    const int g1 = wide_g1(c, z0c), nb3 = (int)rup(w.L, 16) / 16;
    const int mode = (g1 > 5 ? WS_XS : 0) | (outh ? WS_OUTH : 0);
    const dim3 grid((unsigned)rup(a.nrb, 4) * 2), block(64 * WS_NW);
    // diagnostic timer (tdmpc_profile_begin cfg 4: the step kernel); t = 0 launches with the z0c first layer are not
    // timed (less than the algorithmic work), as in launch_chain
    Profiler& pf = g_prof;
    const bool prof = pf.armed && pf.cfg == 4 + CH_STEP && pf.n + 2 <= pf.cap && (pf.rows == 0 || rows == pf.rows) && !z0c;
    if (prof) {
        if (mode) snprintf(pf.kernel, sizeof pf.kernel, "wide_step_kernel<%d, %d, %s%s%s>", g1, nb3,
                           mode & WS_XS ? "XS" : "", mode == (WS_XS | WS_OUTH) ? "|" : "", mode & WS_OUTH ? "OUTH" : "");
        else snprintf(pf.kernel, sizeof pf.kernel, "wide_step_kernel<%d, %d>", g1, nb3);
        HIPCHK(hipEventRecord(pf.ev[pf.n], c.s));
    }
    bool done = false;
#define WIDE_LAUNCH(G1, NB3, MODE) \
    if (!done && g1 == G1 && nb3 == NB3 && mode == (MODE)) { \
        hipLaunchKernelGGL((wide_step_kernel<G1, NB3, MODE>), grid, block, (wsm_lds<G1, MODE>()), c.s, a); \
        done = true; \
    }
    WIDE_FOR_EACH(WIDE_LAUNCH)
#undef WIDE_LAUNCH
    if (!done) { snprintf(g_err, sizeof g_err, "wide step: no instance for G1 %d NB3 %d mode %d", g1, nb3, mode); return TDMPC_E_DIMS; }
    HIPCHK(hipGetLastError());
    if (prof) {
        HIPCHK(hipEventRecord(pf.ev[pf.n + 1], c.s));
        pf.n += 2;
        const double K1 = w.L + w.A;   // (executed products: WS_OUTH launches skip layer 3)
        pf.flops += 2.0 * rows * (2 * (K1 * M + (double)M * M) + (outh ? 0.0 : (double)M * w.L) + M);
    }
    return 0;
}

// defer = 1 (a loop of consecutive steps over the same rows, nothing reading X_{t+1}'s latents in between): on the
// split path the finish of this step is folded into the next step's launch.

// fold (the policy rows of a plan with Ctx::fold_policy, on chain_kernel x6): t >= 1 reads h2 through the folded first
// layer, every step stores h2 (the terminal heads are folded too)
int step_next(const Ctx& c, int t, int rows, RowMap map, float disc, int first, int last, int defer = 0,
              bool nowide = false, bool fold = false) {
    const Layout& w = c.w;
    const int M = c.M;
    int rc;
    if (c.split_pend && (!use_split(c, rows) || rows != c.split_rows || t != c.split_t + 1 ||
                         memcmp(&map, &c.split_map, sizeof map)))
        if ((rc = flush_split(c))) return rc;
    {
        const bool z0c = t == 0 && c.z0c_ready && map.G % 32 == 0;
        if (!nowide && use_wide(c, rows, map, z0c)) {
            if ((rc = flush_split(c))) return rc;
            // Iteration 0's fused launch over all T = N + P rows of every env is 1.5 rounds of workgroups at B = 32
            // (384 blocks on 256 CUs): the sampled rows of every env run on the wide kernel (one whole round) and the
            // policy rows on the chain kernel's many small workgroups, instead of a half-empty second round. The
            // split is by a row's role, never by the launch's size or a row's position in it, so a row's kernel (and
            // its rounding) does not depend on the batch size (tests/test_gpu_sharded.py: two 32-env shards equal
            // the 64-env batch bitwise). At t = 0 both parts keep the z0c first layer (the per-env bias is indexed by
            // logical row / G, and G is the per-env row count of each part's map).
            const RowMap rm = {c.N, map.S, 0}, pm = {c.P, map.S, c.N};
            const int envs = rows / std::max(1, map.G);
            const bool z0c_rm = t == 0 && c.z0c_ready;   // (rm.G = N: use_wide checks N % 128 for the z0c bias)
            if (c.P > 0 && c.N + c.P == c.T && map.G == c.T && map.S == c.T && map.O == 0 && rows == envs * c.T &&
                use_wide(c, envs * c.N, rm, z0c_rm)) {
                if ((rc = launch_wide(c, t, envs * c.N, rm, disc, first, last, z0c_rm, c.fold_ok))) return rc;
                return step_next(c, t, envs * c.P, pm, disc, first, last, 0, true, c.fold_policy != 0);
            }
            const bool sampled = map.G == c.N && map.S == c.T && map.O == 0;   // (the folded rollout's rows only)
            return launch_wide(c, t, rows, map, disc, first, last, z0c, c.fold_ok && sampled);
        }
    }
    if (use_chain(c, rows, 2, CK_STEP)) {
        ChainArgs a = chain0(c, rows, map, t, c.Kx, 0, 2);
        ChainProb& d = a.p[0];
        d.W1 = c.pw + w.w1x; d.b1 = c.pw + w.b1x; d.W2 = c.pw + w.w2d; d.b2 = c.pw + w.b2d;
        ChainProb& r = a.p[1];
        r.W1 = c.pw + w.w1x + (size_t)M * c.Kx; r.b1 = c.pw + w.b1x + M; r.W2 = c.pw + w.w2r; r.b2 = c.pw + w.b2r;
        r.w3v = c.pw + w.w3r; r.b3v = c.pw + w.b3r;
        a.W3 = c.pw + w.w3d; a.b3 = c.pw + w.b3d; a.n3 = w.Lr; a.nvalid = w.L; a.nstore = w.Lp;
        if (a.x6) {
            const size_t rb1 = (size_t)(M / 32) * (rup(c.Kx, 16) / 16) * 1536;   // bf16 per M rows of x6 W1
            d.X1 = x6p(c, X6_W1X); r.X1 = x6p(c, X6_W1X) + rb1;
            d.X2 = x6p(c, X6_W2D); r.X2 = x6p(c, X6_W2R); a.X3 = x6p(c, X6_W3D);
        }
        a.Xo = Xt(c, t + 1); a.out_q0 = w.Ap / 4;
        a.G = c.k.G; a.rlast = c.k.rlast; a.disc = disc; a.first = first; a.last = last;
        if (t == 0 && c.z0c_ready && map.G % 32 == 0) { a.z0c = c.k.z0c; a.z0_G = map.G; a.k1c = z0c_k1c(c); }
        if (fold) {
            if (a.rb != 32 || !a.x6 || !c.w.fold) {
                snprintf(g_err, sizeof g_err, "folded step: chain_kernel x6 only");
                return TDMPC_E_DIMS;
            }
            if (t >= 1) {
                const size_t rb1 = (size_t)(M / 32) * (rup(c.Kx, 16) / 16) * 1536;
                d.X1 = (const unsigned short*)(c.pw + w.fw1_x6); r.X1 = d.X1 + rb1;
                d.b1 = c.pw + w.bfw; r.b1 = c.pw + w.bfw + M;
            }
            a.outh = 1;
        }
        return launch_chain(CH_STEP, a, 2, c.s);
    }
    if (use_split(c, rows)) {
        const int par = c.split_par;
        const size_t zs = (size_t)SPLIT_S * c.k.split_rows * std::max(w.Lr, w.Ar), rs = (size_t)SPLIT_S * c.k.split_rows;
        SplitArgs a;
        memset(&a, 0, sizeof a);
        a.rows = rows; a.M = M; a.K1 = c.Kx; a.q1 = 0; a.amap = map;
        a.X = Xt(c, t); a.x_ts = (long)c.Kx * 32;
        ChainProb& d = a.p[0];
        d.W1 = c.pw + w.w1x; d.b1 = c.pw + w.b1x; d.W2 = c.pw + w.w2d; d.b2 = c.pw + w.b2d;
        ChainProb& r = a.p[1];
        r.W1 = c.pw + w.w1x + (size_t)M * c.Kx; r.b1 = c.pw + w.b1x + M; r.W2 = c.pw + w.w2r; r.b2 = c.pw + w.b2r;
        r.w3v = c.pw + w.w3r;
        a.W3 = c.pw + w.w3d; a.n3 = w.Lr;
        a.zpart = c.k.zpart + par * zs; a.rpart = c.k.rpart_s + par * rs; a.prow = c.k.split_rows;
        a.b3d = c.pw + w.b3d; a.b3r = c.pw + w.b3r; a.L = w.L; a.Lp = w.Lp; a.zq0 = w.Ap / 4;
        const bool x6 = use_x6(c) != 0;
        if (x6) {
            d.X1 = x6p(c, X6_W1X); r.X1 = x6p(c, X6_W1X) + (size_t)(M / 32) * (rup(c.Kx, 16) / 16) * 1536;
            d.X2 = x6p(c, X6_W2D); r.X2 = x6p(c, X6_W2R); a.X3 = x6p(c, X6_W3D);
        }
        if (c.split_pend) {   // the previous step's finish, folded into this launch's staging
            a.zin = c.k.zpart + (1 - par) * zs; a.rin = c.k.rpart_s + (1 - par) * rs;
            a.Xw = Xt(c, t); a.G = c.k.G; a.disc_in = c.split_disc; a.first_in = c.split_first;
        }
        const size_t lds = (size_t)split_lds_floats(c.Kx, M) * 4;
        if (x6) hipLaunchKernelGGL((split_step_kernel<4, 4, 1>), dim3((rows + 15) / 16, SPLIT_S, 2), dim3(512), lds, c.s, a);
        else hipLaunchKernelGGL((split_step_kernel<4>), dim3((rows + 15) / 16, SPLIT_S, 2), dim3(512), lds, c.s, a);
        HIPCHK(hipGetLastError());
        c.split_pend = 0;
        c.split_par = 1 - par;
        if (defer && !last) {
            c.split_pend = 1; c.split_disc = disc; c.split_first = first;
            c.split_map = map; c.split_rows = rows; c.split_t = t;
            return 0;
        }
        return split_finish(c, t, rows, map, a.zpart, a.rpart, disc, first, last);
    }
    {   // h1 = ELU(W1[d;r] [a|z] + b)   (dynamics.0 and reward.0 fused: N = 2M)
        LinArgs a = args0();
        a.M = rows; a.K = c.Kx; a.a_mapped = 1; a.amap = map;
        LinProb& p = a.p[0];
        p.A = xop(c, t, 0); p.W = wop(c, w.w1x, c.Kx); p.bias = c.pw + w.b1x;
        p.C = hout(c.k.H1, c, 0); p.N = p.nvalid = p.nstore = 2 * M; p.epi = EPI_ELU;
        if ((rc = launch_lin(a, 1, 2 * M, 0, PRO_PLAIN, c.s))) return rc;
    }
    {   // h2_d = ELU(W2d h1_d + b); reward partial dots of ELU(W2r h1_r + b) with reward.4.weight
        LinArgs a = args0();
        a.M = rows; a.K = M;
        LinProb& p0 = a.p[0];
        p0.A = hop(c.k.H1, c, 0); p0.W = wop(c, w.w2d, M); p0.bias = c.pw + w.b2d;
        p0.C = hout(c.k.H2, c, 0); p0.N = p0.nvalid = p0.nstore = M; p0.epi = EPI_ELU;
        LinProb& p1 = a.p[1];
        p1.A = hop(c.k.H1, c, M / 4); p1.W = wop(c, w.w2r, M); p1.bias = c.pw + w.b2r;
        p1.N = p1.nvalid = M; p1.nstore = 0; p1.epi = EPI_ELU_DOT;
        p1.dotw = c.pw + w.w3r; p1.dot_out = c.k.rpart; p1.dot_ld = M / pick_cfg(rows, M, M, 0).bw;
        if ((rc = launch_lin(a, 2, M, 0, PRO_PLAIN, c.s))) return rc;
    }
    {   // z' = W3d h2_d + b -> X_{t+1} latent columns; reward = sum(partials) + b; G update
        LinArgs a = args0();
        a.M = rows; a.K = M; a.c_mapped = 1; a.cmap = map;
        LinProb& p = a.p[0];
        p.A = hop(c.k.H2, c, 0); p.W = wop(c, w.w3d, M); p.bias = c.pw + w.b3d;
        p.C = xout(c, t + 1, w.Ap / 4); p.N = w.L; p.nvalid = w.L; p.nstore = w.Lp; p.epi = EPI_LIN_Z;
        a.rpart = c.k.rpart; a.rpart_nt = M / pick_cfg(rows, M, M, 0).bw; a.b3r = c.pw + w.b3r;
        a.G = c.k.G; a.rlast = c.k.rlast; a.disc = disc; a.first = first; a.last = last;
        if ((rc = launch_lin(a, 1, w.L, 0, PRO_PLAIN, c.s))) return rc;
    }
    return 0;
}

// pi(z_t) with TruncatedNormal noise for `rows` rows of X_t -> X_t action columns (tdmpc.py:39-45).
// fold: the rows' latent columns hold h2_{t-1} (Ctx::fold_heads): the first layer is the folded [Wp1 W3], bp1 + Wp1 b3
// (chain x6 only)
int policy(const Ctx& c, int t, int rows, RowMap map, const float* eps, long eps_env, int eps_G, long eps_off,
           float min_std, float* mu_out = nullptr, bool fold = false) {
    const Layout& w = c.w;
    const int M = c.M;
    int rc;
    if (fold && !(use_chain(c, rows, 1, CK_PI) && use_x6(c))) {
        snprintf(g_err, sizeof g_err, "folded pi: chain x6 kernels only");
        return TDMPC_E_DIMS;
    }
    if (use_chain(c, rows, 1, CK_PI)) {
        ChainArgs a = chain0(c, rows, map, t, w.Lp, w.Ap / 4, 1);
        ChainProb& p = a.p[0];
        p.W1 = c.pw + w.wp1; p.b1 = c.pw + w.bp1; p.W2 = c.pw + w.wp2; p.b2 = c.pw + w.bp2;
        a.W3 = c.pw + w.wp3; a.b3 = c.pw + w.bp3; a.n3 = w.Ar; a.nvalid = w.A; a.nstore = w.Ap;
        if (a.x6) { p.X1 = x6p(c, X6_WP1); p.X2 = x6p(c, X6_WP2); a.X3 = x6p(c, X6_WP3); }
        if (fold) { p.X1 = (const unsigned short*)(c.pw + w.fpi_x6); p.b1 = c.pw + w.fpi_b; }
        a.Xo = Xt(c, t); a.out_q0 = 0;
        a.eps = eps; a.eps_G = eps_G; a.eps_env = eps_env; a.eps_off = eps_off; a.A = w.A;
        a.min_std = min_std; a.lo = (float)(-1.0 + 1e-6); a.hi = (float)(1.0 - 1e-6);
        a.mu_out = mu_out;
        return launch_chain(CH_PI, a, 1, c.s);
    }
    if (use_split_pi(c, rows)) {
        if ((rc = flush_split(c))) return rc;
        SplitArgs a;
        memset(&a, 0, sizeof a);
        a.rows = rows; a.M = M; a.K1 = w.Lp; a.q1 = w.Ap / 4; a.amap = map;
        a.X = Xt(c, t); a.x_ts = (long)c.Kx * 32;
        ChainProb& p = a.p[0];
        p.W1 = c.pw + w.wp1; p.b1 = c.pw + w.bp1; p.W2 = c.pw + w.wp2; p.b2 = c.pw + w.bp2;
        a.W3 = c.pw + w.wp3; a.n3 = w.Ar;
        a.zpart = c.k.zpart; a.rpart = c.k.rpart_s; a.prow = c.k.split_rows;
        const size_t lds = (size_t)split_lds_floats(w.Lp, M) * 4;
        if (use_x6(c)) {
            p.X1 = x6p(c, X6_WP1); p.X2 = x6p(c, X6_WP2); a.X3 = x6p(c, X6_WP3);
            hipLaunchKernelGGL((split_step_kernel<4, 4, 1>), dim3((rows + 15) / 16, SPLIT_S, 1), dim3(512), lds, c.s, a);
        } else {
            hipLaunchKernelGGL((split_step_kernel<4>), dim3((rows + 15) / 16, SPLIT_S, 1), dim3(512), lds, c.s, a);
        }
        HIPCHK(hipGetLastError());
        SplitPiArgs f;
        memset(&f, 0, sizeof f);
        f.rows = rows; f.amap = map; f.part = c.k.zpart; f.prow = c.k.split_rows; f.n3 = w.Ar; f.A = w.A;
        f.Ap = w.Ap; f.b3 = c.pw + w.bp3; f.Xo = Xt(c, t); f.x_ts = (long)c.Kx * 32;
        f.eps = eps; f.eps_G = eps_G; f.eps_env = eps_env; f.eps_off = eps_off; f.min_std = min_std;
        f.lo = (float)(-1.0 + 1e-6); f.hi = (float)(1.0 - 1e-6);
        const long nth = (long)rows * (w.Ap / 4);
        hipLaunchKernelGGL(split_pi_finish_kernel, dim3((unsigned)((nth + 255) / 256)), dim3(256), 0, c.s, f);
        HIPCHK(hipGetLastError());
        return 0;
    }
    {
        LinArgs a = args0();
        a.M = rows; a.K = w.Lp; a.a_mapped = 1; a.amap = map;
        LinProb& p = a.p[0];
        p.A = xop(c, t, w.Ap / 4); p.W = wop(c, w.wp1, w.Lp); p.bias = c.pw + w.bp1;
        p.C = hout(c.k.H1, c, 0); p.N = p.nvalid = p.nstore = M; p.epi = EPI_ELU;
        if ((rc = launch_lin(a, 1, M, 0, PRO_PLAIN, c.s))) return rc;
    }
    {
        LinArgs a = args0();
        a.M = rows; a.K = M;
        LinProb& p = a.p[0];
        p.A = hop(c.k.H1, c, 0); p.W = wop(c, w.wp2, M); p.bias = c.pw + w.bp2;
        p.C = hout(c.k.H2, c, 0); p.N = p.nvalid = p.nstore = M; p.epi = EPI_ELU;
        if ((rc = launch_lin(a, 1, M, 0, PRO_PLAIN, c.s))) return rc;
    }
    {
        LinArgs a = args0();
        a.M = rows; a.K = M; a.c_mapped = 1; a.cmap = map;
        LinProb& p = a.p[0];
        p.A = hop(c.k.H2, c, 0); p.W = wop(c, w.wp3, M); p.bias = c.pw + w.bp3;
        p.C = xout(c, t, 0); p.N = w.A; p.nvalid = w.A; p.nstore = w.Ap; p.epi = EPI_PI;
        a.eps = eps; a.eps_G = eps_G; a.eps_env = eps_env; a.eps_off = eps_off; a.A = w.A;
        a.min_std = min_std;
        a.lo = (float)(-1.0 + 1e-6); a.hi = (float)(1.0 - 1e-6);
        return launch_lin(a, 1, w.A, 0, PRO_PLAIN, c.s);
    }
}

// TDMPC_PI_CACHE=0: the pi rows' terminal mean is recomputed in every CEM iteration (A/B switch; default on)
int pi_cache_on() {
    static const int v = [] { const char* e = getenv("TDMPC_PI_CACHE"); return e ? atoi(e) : 1; }();
    return v;
}

// pi(z_H) of `rows` rows from the cached means k.pimu (pi_from_mu_kernel) -> X_H action columns.
PiMuArgs pimu_args(const Ctx& c, int rows, RowMap map, const float* eps, long eps_env, int eps_G, long eps_off,
                   float min_std, float* Xo = nullptr, const RowMap* mmap = nullptr) {
    PiMuArgs f;
    memset(&f, 0, sizeof f);
    f.rows = rows; f.amap = map; f.mmap = mmap ? *mmap : map; f.mu = c.k.pimu; f.Ap = c.w.Ap; f.A = c.w.A;
    f.Xo = Xo ? Xo : Xt(c, c.H); f.x_ts = (long)c.Kx * 32;
    f.eps = eps; f.eps_G = eps_G; f.eps_env = eps_env; f.eps_off = eps_off; f.min_std = min_std;
    f.lo = (float)(-1.0 + 1e-6); f.hi = (float)(1.0 - 1e-6);
    return f;
}

int policy_from_mu(const Ctx& c, int rows, RowMap map, const float* eps, long eps_env, int eps_G, long eps_off,
                   float min_std, float* Xo = nullptr, const RowMap* mmap = nullptr) {
    const PiMuArgs f = pimu_args(c, rows, map, eps, eps_env, eps_G, eps_off, min_std, Xo, mmap);
    const long nth = (long)rows * (c.w.Ap / 4);
    if (!nth) return 0;
    hipLaunchKernelGGL(pi_from_mu_kernel, dim3((unsigned)((nth + 255) / 256)), dim3(256), 0, c.s, f);
    HIPCHK(hipGetLastError());
    return 0;
}

// Terminal value: Q(z_H, pi(z_H)) for all T rows of every env (tdmpc.py:91-92).
// prep_kernel launch: candidates of CEM iteration `iter` for all H steps (if noise) and, with z0, the
// latent columns of X_0 for every row; with pm, the policy rows' terminal redraw of that iteration in the same launch
// (it reads only the cached pi mean and the noise, so it need not wait for the rollout).
int prep(const Ctx& c, const float* noise, int iter, const float* z0, const PiMuArgs* pm = nullptr) {
    PrepArgs a;
    memset(&a, 0, sizeof a);
    a.X = c.k.X; a.x_stride = c.k.x_stride; a.Kx = c.Kx; a.apq = c.w.Ap / 4; a.lpq = c.w.Lp / 4;
    a.B = c.B; a.N = c.N; a.T = c.T; a.H = c.H; a.A = c.A;
    a.mean = c.k.mean; a.stdv = c.k.stdv; a.mstride = c.d->max_horizon * c.A;
    a.eps = noise; a.eps_env = c.eps_env; a.eps_off = c.eps_cem_off + (long)iter * c.eps_iter;
    a.z0 = z0;
    a.n_zq = z0 ? (long)c.B * a.lpq * c.T : 0;
    a.n_sq = noise ? (long)c.B * c.H * a.apq * c.N : 0;
    if (pm) {
        a.pm = *pm;
        a.n_pm = (long)pm->rows * (pm->Ap / 4);
    }
    const long total = a.n_zq + a.n_sq + a.n_pm;
    if (!total) return 0;
    const int blocks = (int)std::min<long>((total + 255) / 256, 2048);
    hipLaunchKernelGGL(prep_kernel, dim3(blocks), dim3(256), 0, c.s, a);
    HIPCHK(hipGetLastError());
    return 0;
}

// helper.q for both heads over `rows` rows of X_H mapped by `map`, on the chain kernel: q_p per row into k.qv
// (the value combination happens where it is consumed: cem_kernel / qvalue_kernel).
int q_chain(const Ctx& c, int rows, RowMap map, const float* X = nullptr, float* qo = nullptr, int q_ld = 0,
            bool fold = false) {
    const Layout& w = c.w;
    const int M = c.M;
    ChainArgs a = chain0(c, rows, map, c.H, c.Kx, 0, 2);
    if (X) a.X = X;
    if (fold && !a.x6) {
        snprintf(g_err, sizeof g_err, "folded Q: chain x6 kernels only");
        return TDMPC_E_DIMS;
    }
    for (int q = 0; q < 2; ++q) {
        ChainProb& p = a.p[q];
        p.W1 = c.pw + w.wq1x + (size_t)q * M * c.Kx; p.b1 = c.pw + w.bq1x + q * M;
        p.g1 = c.pw + w.g1 + q * M; p.be1 = c.pw + w.be1 + q * M;
        p.W2 = c.pw + w.wq2 + (size_t)q * M * M; p.b2 = c.pw + w.bq2 + q * M;
        p.g2 = c.pw + w.g2 + q * M; p.be2 = c.pw + w.be2 + q * M;
        p.w3v = c.pw + w.wq3 + q * M; p.b3v = c.pw + w.bq3 + q;
        if (a.x6) {
            p.X1 = x6p(c, X6_WQ1X) + (size_t)q * (M / 32) * (rup(c.Kx, 16) / 16) * 1536;
            p.X2 = x6p(c, X6_WQ2) + (size_t)q * (M / 32) * (M / 16) * 1536;
        }
        if (fold) {   // the rows' latent columns hold h2_{H-1}: [Wq1a | Wq1z W3], bq1 + Wq1z b3
            p.X1 = (const unsigned short*)(c.pw + w.fq_x6) + (size_t)q * (M / 32) * (rup(c.Kx, 16) / 16) * 1536;
            p.b1 = c.pw + w.fq_b + q * M;
        }
    }
    a.q = qo ? qo : c.k.qv; a.q_ld = qo ? q_ld : c.k.xrows;
    return launch_chain(CH_Q, a, 2, c.s);
}

// ---- the wide heads (wide_heads.inc): terminal pi and helper.q on the wide step kernel's design, for plans whose
// sampled rows' steps run on the wide step kernel (B N rows fill 128-row blocks on every CU). TDMPC_WIDE_HEADS=0
// keeps the chain kernels. A row's kernel follows its role, never the launch size (as in step_next): the sampled rows'
// terminal pi and both Q heads and the policy rows' Q heads run here, the policy rows' cached pi mean on the chain
// kernel (iteration 0) and pi_from_mu_kernel.
int wh_g1p(const Ctx& c) { return (int)rup(c.w.Lp, 32) / 32; }
int wh_nb3p(const Ctx& c) { return (int)rup(c.w.A, 16) / 16; }
int wh_g1q(const Ctx& c) { return (int)rup(c.Kx, 32) / 32; }
bool wh_instance(const Ctx& c) {
    const int g1p = wh_g1p(c), nb3 = wh_nb3p(c), g1q = wh_g1q(c), nst = c.w.nsr / 16;
#define WH_HAS(G1P, NB3P, G1Q, NSTQ) if (g1p == G1P && nb3 == NB3P && g1q == G1Q && nst == NSTQ) return true;
    WIDE_HEADS_FOR_EACH(WH_HAS)
#undef WH_HAS
    return false;
}
bool use_wide_heads(const Ctx& c) {
    static const int en = [] { const char* e = getenv("TDMPC_WIDE_HEADS"); return e ? atoi(e) : 1; }();
    if (!en || !c.w.nqs || c.w.M != 512 || !use_x6(c) || !num_cus()) return false;
    if (c.path != TDMPC_PATH_AUTO && c.path != TDMPC_PATH_CHAIN && c.path != TDMPC_PATH_WIDE) return false;
    if (c.N + c.P != c.T || c.N % 16 || c.P % 16) return false;
    if (!use_wide(c, c.B * c.N, RowMap{c.N, c.T, 0}, false) || !wh_instance(c)) return false;
    // the policy rows' pi mean comes from the chain kernel (mu_out)
    return c.P == 0 || use_chain(c, c.B * c.P, 1, CK_PI);
}
WHJob wh_job(int role, int head, int x0, int nx, int rows, RowMap map) {
    WHJob j;
    memset(&j, 0, sizeof j);
    j.role = role; j.head = head; j.x0 = x0; j.nx = nx; j.rows = rows; j.nrb = (rows + 127) / 128; j.map = map;
    j.eps_G = 1;
    return j;
}
int launch_wide_heads(const Ctx& c, const WHJob* jobs, int nj, const float* eps, float min_std) {
    const Layout& w = c.w;
    const int M = c.M;
    WHArgs a;
    memset(&a, 0, sizeof a);
    for (int i = 0; i < nj; ++i) a.job[i] = jobs[i];
    a.njob = nj;
    a.X = Xt(c, c.H); a.x_ts = (long)c.Kx * 32;
    auto q6 = [&](int i) { return (const unsigned short*)(c.pw + w.x6q[i]); };
    a.P1 = q6(X6_WP1); a.P2 = q6(X6_WP2); a.P3 = q6(X6_WP3);
    a.pb1 = c.pw + w.bp1; a.pb2 = c.pw + w.bp2; a.pb3 = c.pw + w.bp3;
    a.A = w.A; a.Ap = w.Ap; a.pq1 = w.Ap / 4; a.pkq = w.Lp / 4; a.pg1s = wh_g1p(c);
    a.eps = eps; a.min_std = min_std; a.lo = (float)(-1.0 + 1e-6); a.hi = (float)(1.0 - 1e-6);
    const int g1q = wh_g1q(c);
    for (int h = 0; h < 2; ++h) {
        WHQHead& q = a.q[h];
        q.S = (const unsigned short*)(c.pw + w.x6qs) + (size_t)h * (w.nsr / 16) * g1q * 1536;
        q.X1 = (const unsigned short*)(c.pw + w.x6qf) + (size_t)h * (M / 16) * g1q * 1536;   // (folded, see wide_heads.inc)
        q.X2 = q6(X6_WQ2) + (size_t)h * (M / 16) * (M / 32) * 1536;
        q.bs = c.pw + w.bqs + (size_t)h * w.nsr;
        q.b1 = c.pw + w.bqf + h * M; q.g1 = c.pw + w.g1 + h * M; q.be1 = c.pw + w.be1 + h * M;
        q.b2 = c.pw + w.bq2 + h * M; q.g2 = c.pw + w.g2 + h * M; q.be2 = c.pw + w.be2 + h * M;
        q.w3 = c.pw + w.wq3 + h * M; q.b3 = c.pw + w.bq3 + h;
    }
    a.qkq = c.Kx / 4; a.qg1s = g1q;
    a.qv = c.k.qv; a.q_ld = c.k.xrows;
    int slots = 0;
    bool allq = true;
    double flops = 0.0;
    for (int i = 0; i < nj; ++i) {
        const WHJob& J = jobs[i];
        if (J.rows % 16 || J.x0 < 0 || J.nx <= 0 || J.x0 + J.nx > 8) {
            snprintf(g_err, sizeof g_err, "wide heads: bad job %d", i);
            return TDMPC_E_DIMS;
        }
        slots = std::max(slots, (J.nrb + J.nx - 1) / J.nx);
        allq = allq && J.role == WH_Q;
        flops += 2.0 * J.rows * (J.role == WH_PI ? (double)w.L * M + (double)M * M + (double)M * w.A
                                                 : (double)(w.L + w.A) * M + (double)M * M + M);
    }
    if (!slots) return 0;
    const dim3 grid((unsigned)slots * 8), block(64 * WS_NW);
    const int g1p = wh_g1p(c), nb3 = wh_nb3p(c), nst = w.nsr / 16;
    // diagnostic timer (tdmpc_profile_begin cfg 4 + CH_Q: the all-Q launch, cfg 4 + CH_PI: the mixed one)
    Profiler& pf = g_prof;
    const bool prof = pf.armed && pf.cfg == 4 + (allq ? CH_Q : CH_PI) && pf.n + 2 <= pf.cap &&
                      (pf.rows == 0 || jobs[0].rows == pf.rows);
    if (prof) {
        snprintf(pf.kernel, sizeof pf.kernel, "wide_heads_kernel<%d, %d, %d, %d> (%s)", g1p, nb3, g1q, nst,
                 allq ? "Q1 + Q2" : "pi + Q1 + Q2 of the policy rows");
        HIPCHK(hipEventRecord(pf.ev[pf.n], c.s));
    }
    bool done = false;
#define WH_LAUNCH(G1P, NB3P, G1Q, NSTQ) \
    if (!done && g1p == G1P && nb3 == NB3P && g1q == G1Q && nst == NSTQ) { \
        hipLaunchKernelGGL((wide_heads_kernel<G1P, NB3P, G1Q, NSTQ>), grid, block, \
                           ws_lds<(G1P > G1Q ? G1P : G1Q)>(), c.s, a); \
        done = true; \
    }
    WIDE_HEADS_FOR_EACH(WH_LAUNCH)
#undef WH_LAUNCH
    if (!done) { snprintf(g_err, sizeof g_err, "wide heads: no instance"); return TDMPC_E_DIMS; }
    HIPCHK(hipGetLastError());
    if (prof) {
        HIPCHK(hipEventRecord(pf.ev[pf.n + 1], c.s));
        pf.n += 2;
        pf.flops += flops;
    }
    return 0;
}

// The terminal heads of one CEM iteration on the wide heads: launch A = the sampled rows' pi (XCD groups 0-3) beside the
// policy rows' Q1 (4-5) and Q2 (6-7), launch B = the sampled rows' Q1 (0-3) and Q2 (4-7). The policy rows' actions at
// X_H are in place (chain pi with the mean cache at iteration 0, pi_from_mu after).
int terminal_wide(const Ctx& c, const float* noise, long toff, float min_std) {
    const RowMap rm = {c.N, c.T, 0}, pm = {c.P, c.T, c.N};
    WHJob ja[3];
    int na = 0;
    ja[na] = wh_job(WH_PI, 0, 0, c.P > 0 ? 4 : 8, c.B * c.N, rm);
    ja[na].eps_env = c.eps_env; ja[na].eps_off = toff; ja[na].eps_G = c.N;
    ++na;
    if (c.P > 0) {
        ja[na++] = wh_job(WH_Q, 0, 4, 2, c.B * c.P, pm);
        ja[na++] = wh_job(WH_Q, 1, 6, 2, c.B * c.P, pm);
    }
    int rc;
    if ((rc = launch_wide_heads(c, ja, na, noise, min_std))) return rc;
    const WHJob jb[2] = {wh_job(WH_Q, 0, 0, 4, c.B * c.N, rm), wh_job(WH_Q, 1, 4, 4, c.B * c.N, rm)};
    return launch_wide_heads(c, jb, 2, noise, min_std);
}

// Terminal value of `rows` rows of X_H mapped by `map`: the chain path leaves q1, q2 per row in k.qv (consumed
// by cem_kernel / qvalue_kernel); the layered path gathers the rows into H1, runs the Q heads and writes
// value = nan_to_num(G + gamma^H min(Q1, Q2)) back to the mapped rows (value_kernel).
int terminal_q_rows(const Ctx& c, int rows, RowMap map, float discH, bool chain) {
    const Layout& w = c.w;
    const int M = c.M;
    int rc;
    if (chain) return q_chain(c, rows, map);
    {   // y1 = Wq1[Q1;Q2] [a|z] + b -> H1, with LayerNorm partial moments per 64 columns
        LinArgs a = args0();
        a.M = rows; a.K = c.Kx; a.a_mapped = 1; a.amap = map;
        LinProb& p = a.p[0];
        p.A = xop(c, c.H, 0); p.W = wop(c, w.wq1x, c.Kx); p.bias = c.pw + w.bq1x;
        p.C = hout(c.k.H1, c, 0); p.N = p.nvalid = p.nstore = 2 * M; p.epi = EPI_LNSTATS;
        p.st_out = c.k.st1; p.st_ld = 2 * M / 64;
        if ((rc = launch_lin(a, 1, 2 * M, 1, PRO_PLAIN, c.s))) return rc;
    }
    {   // a1 = tanh(LN(y1)) -> H2
        LnArgs l;
        l.Y = c.k.H1; l.O = c.k.H2; l.ts = (long)2 * M * 32; l.st = c.k.st1; l.st_ld = 2 * M / 64; l.M_ = M;
        l.rows = rows; l.g = c.pw + w.g1; l.b = c.pw + w.be1;
        hipLaunchKernelGGL(ln_tanh_kernel, dim3((rows + 31) / 32, 2), dim3(512), 0, c.s, l);
        HIPCHK(hipGetLastError());
    }
    {   // y2_p = Wq2_p a1_p + b -> H1, moments again
        LinArgs a = args0();
        a.M = rows; a.K = M;
        for (int q = 0; q < 2; ++q) {
            LinProb& p = a.p[q];
            p.A = hop(c.k.H2, c, q * M / 4); p.W = wop(c, w.wq2 + (size_t)q * M * M, M);
            p.bias = c.pw + w.bq2 + q * M; p.C = hout(c.k.H1, c, q * M / 4); p.N = p.nvalid = p.nstore = M;
            p.epi = EPI_LNSTATS; p.st_out = c.k.st2 + q * (M / 64); p.st_ld = 2 * M / 64;
        }
        if ((rc = launch_lin(a, 2, M, 1, PRO_PLAIN, c.s))) return rc;
    }
    {
        ValueArgs v;
        v.Y = c.k.H1; v.yts = (long)2 * M * 32; v.st = c.k.st2; v.st_ld = 2 * M / 64; v.M_ = M;
        v.g2 = c.pw + w.g2; v.be2 = c.pw + w.be2; v.w3 = c.pw + w.wq3; v.b3 = c.pw + w.bq3;
        v.G = c.k.G; v.disc = discH; v.value = c.k.value; v.rows = rows; v.map = map;
        hipLaunchKernelGGL(value_kernel, dim3((rows + 31) / 32), dim3(512), 0, c.s, v);
        HIPCHK(hipGetLastError());
    }
    return 0;
}

int terminal_q(const Ctx& c, float discH) {
    const int rows = c.B * c.T;
    return terminal_q_rows(c, rows, RowMap{1 << 30, 0, 0}, discH, use_chain(c, rows, 2, CK_Q));
}

// TOLD.h for `batch` observations -> z0 [B][Lp]; optionally initialises the CEM mean/std.
int encode(const Ctx& c, const void* obs, int obs_is_u8, int batch, const float* prev_mean, int warm,
           int warm_keep_last = 0, float init_std = 2.f, const int* warm_flags = nullptr) {
    const Layout& w = c.w;
    const float* pw = c.pw;
    EncArgs a;
    memset(&a, 0, sizeof a);
    a.L = w.L; a.Lp = w.Lp; a.z0 = c.k.z0;
    if (w.modality == 0) {
        a.x = (const float*)obs; a.x_stride = w.obs_dim; a.xdim = w.obs_dim; a.E = w.E;
        a.w1t = pw + w.enc_w1t; a.b1 = pw + w.enc_b1; a.w2t = pw + w.enc_w2t; a.b2 = pw + w.enc_b2;
        if (w.enc_norm) { a.ln_g = pw + w.enc_lng; a.ln_b = pw + w.enc_lnb; }
    } else {
        static const int ks[4] = {7, 5, 3, 3};
        const size_t act = pixel_act_floats(w);
        float* bufs[2] = {c.k.enc_tmp, c.k.enc_tmp + (size_t)batch * act};
        const void* in = obs;
        int in_u8 = obs_is_u8;
        long in_bs = (long)w.img_c * w.img_hw * w.img_hw;
        int cin = w.img_c;
        for (int i = 0; i < 4; ++i) {
            const int ho = w.conv_hw[i + 1], hi = w.conv_hw[i];
            const int total = w.nch * ho * ho;
            float* out = bufs[i & 1];
            // tiled form when the channels split into groups of 8: (pixels per item, output rows per tile) by a
            // cost model -- rounds of workgroups over the CUs x rounds of items over 256 threads x an item's
            // instructions, plus the staging -- among the shapes whose tile fits LDS
            int toy = 0, px = 1;
            if (w.nch % 8 == 0) {
                double best = 1e300;
                const int kk = ks[i] * ks[i];
                for (int pxc : {1, 2, 4})
                    for (int t = 1; t <= ho; ++t) {
                        const size_t fl = rup((size_t)cin * (2 * (t - 1) + ks[i]) * hi, 4) + (size_t)w.nch * cin * kk;
                        if (fl * 4 > 160 * 1024) break;
                        const long tiles = (long)((ho + t - 1) / t) * batch;
                        const long items = (long)t * ((ho + pxc - 1) / pxc) * (w.nch / 8);
                        const double cost = (double)((tiles + num_cus() - 1) / num_cus()) *
                                            ((double)((items + 255) / 256) * cin * kk * (8.0 * pxc + pxc + 2) +
                                             (double)fl / 256 * 4);
                        if (cost < best) { best = cost; toy = t; px = pxc; }
                    }
            }
            if (toy > 0) {
                const size_t lds = (rup((size_t)cin * (2 * (toy - 1) + ks[i]) * hi, 4) + (size_t)w.nch * cin * ks[i] * ks[i]) * 4;
                const dim3 grid((ho + toy - 1) / toy, batch);
                if (px == 4)
                    hipLaunchKernelGGL(conv_tile_kernel<4>, grid, dim3(256), lds, c.s, in, in_u8, in_bs, cin, hi, out,
                                       (long)act, w.nch, ho, ks[i], toy, pw + w.cwt[i], pw + w.cb[i]);
                else if (px == 2)
                    hipLaunchKernelGGL(conv_tile_kernel<2>, grid, dim3(256), lds, c.s, in, in_u8, in_bs, cin, hi, out,
                                       (long)act, w.nch, ho, ks[i], toy, pw + w.cwt[i], pw + w.cb[i]);
                else
                    hipLaunchKernelGGL(conv_tile_kernel<1>, grid, dim3(256), lds, c.s, in, in_u8, in_bs, cin, hi, out,
                                       (long)act, w.nch, ho, ks[i], toy, pw + w.cwt[i], pw + w.cb[i]);
            } else {
                hipLaunchKernelGGL(conv_relu_kernel, dim3((total + 255) / 256, batch), dim3(256), 0, c.s, in, in_u8,
                                   in_bs, cin, hi, out, (long)act, w.nch, ho, ks[i], pw + w.cw[i], pw + w.cb[i]);
            }
            HIPCHK(hipGetLastError());
            in = out; in_u8 = 0; in_bs = (long)act; cin = w.nch;
        }
        a.x = (const float*)in; a.x_stride = (long)act; a.xdim = w.flat;
        a.E = w.flat; a.w1t = nullptr; a.w2t = pw + w.pl_wt; a.b2 = pw + w.pl_b;
    }
    if (prev_mean) {
        a.mean = c.k.mean; a.stdv = c.k.stdv; a.prev_mean = prev_mean; a.warm = warm; a.warm_flags = warm_flags;
        a.warm_keep_last = warm_keep_last; a.init_std = init_std;
        a.H = c.H; a.A = c.A; a.Hmax = c.d->max_horizon;
    }
    const size_t lds = (rup(a.xdim, 4) + rup(std::max(a.E, 1), 4) + 1024) * 4;
    hipLaunchKernelGGL(encode_kernel, dim3(batch), dim3(1024), lds, c.s, a);
    HIPCHK(hipGetLastError());
    return 0;
}


// The persistent one-env plan (plan1.inc) for this call? The auto path's choice (TDMPC_PERSIST=0 turns it off) and
// TDMPC_PATH_PERSIST, when the shape fits, batch 1, >= 256 CUs (every workgroup of its 256-block grid must be
// resident). Measured on MI355X (humanoid-run, one env, same box, alternating): 1.083-1.087 vs 1.142-1.144 ms per
// plan_batch call, 1.185-1.198 vs 1.237-1.251 ms per literal plan() -- see DESIGN.md §4 for its per-phase timeline.
// Can every workgroup of plan1's 256-block grid be resident at once (one per CU: its LDS and registers)? Its hand-offs
// assume so; the occupancy query is checked once per LDS size, and a grid that does not fit takes the launch chain.
bool plan1_resident(const Ctx& c) {
    static size_t ok_lds[2] = {0, 0}, bad_lds[2] = {0, 0};
    const int ks = p1_ks(c.w) == 4 ? 0 : 1;
    const size_t lds = p1_lds_bytes(c.H, c.d->num_elites, c.w.A, c.T);
    if (ok_lds[ks] == lds) return true;
    if (bad_lds[ks] == lds) return false;
    int per_cu = 0;
    const hipError_t e = ks == 0
        ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, plan1_kernel<4>, P1_NT, lds)
        : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, plan1_kernel<6>, P1_NT, lds);
    const bool ok = e == hipSuccess && (long)per_cu * num_cus() >= P1_NG * P1_WPG;
    (ok ? ok_lds : bad_lds)[ks] = lds;
    return ok;
}

bool use_plan1(const Ctx& c) {
    static int en = -1;
    if (en < 0) {
        const char* e = getenv("TDMPC_PERSIST");
        en = e ? atoi(e) : 1;
    }
    if (c.path != TDMPC_PATH_PERSIST && (c.path != TDMPC_PATH_AUTO || !en)) return false;
    return c.B == 1 && c.k.p1 && num_cus() >= P1_NG * P1_WPG && c.H <= 16 && plan1_resident(c);
}

// encode_kernel has written z0 and the initial mean / std; one memset node (the hand-off counters) + one launch.
// zero fill as a kernel of our own (the graph-captured paths avoid hipMemsetAsync nodes: see plan1_launch)
__global__ void zero_words_kernel(unsigned* p, int n) {
    for (int i = threadIdx.x; i < n; i += blockDim.x) p[i] = 0u;
}

// the packed buffer's sticky pack status (PackHdr::status, TDMPC_STATUS_PACK_STALE)
inline const int* pack_status(const Ctx& c) {
    return (const int*)((const char*)(c.pw + c.w.jobtab) + offsetof(PackHdr, status));
}

int plan1_launch(const Ctx& c, const tdmpc_plan_params* prm, const float* noise, const double* u, float* prev_mean,
                 float* action, float* metrics, float* elite_out, float* score_out, float* value_out, float* mean_out,
                 float* std_out) {
    const Layout& w = c.w;
    const float* pw = c.pw;
    const P1Region rg = p1_region(c.d, w);
    P1Args a;
    memset(&a, 0, sizeof a);
    a.A = w.A; a.L = w.L; a.Ap = w.Ap; a.Lp = w.Lp; a.KG1 = (w.Kx + 15) / 16; a.KGP = (w.Lp + 15) / 16;
    a.KXS = p1_kxs(w); a.Lr = w.Lr; a.Ar = w.Ar; a.H = c.H; a.I = prm->iterations; a.N = c.N; a.P = c.P; a.T = c.T;
    a.K = c.d->num_elites; a.sr = (c.N + P1_NG - 1) / P1_NG; a.pr = (c.P + P1_NG - 1) / P1_NG;
    a.x1x = x6p(c, X6_W1X); a.x2d = x6p(c, X6_W2D); a.x2r = x6p(c, X6_W2R); a.x3d = x6p(c, X6_W3D);
    a.xp1 = x6p(c, X6_WP1); a.xp2 = x6p(c, X6_WP2); a.xp3 = x6p(c, X6_WP3); a.xq1 = x6p(c, X6_WQ1X); a.xq2 = x6p(c, X6_WQ2);
    a.b1x = pw + w.b1x; a.b2d = pw + w.b2d; a.b2r = pw + w.b2r; a.b3d = pw + w.b3d; a.w3r = pw + w.w3r; a.b3r = pw + w.b3r;
    a.bp1 = pw + w.bp1; a.bp2 = pw + w.bp2; a.bp3 = pw + w.bp3; a.bq1 = pw + w.bq1x; a.g1 = pw + w.g1; a.be1 = pw + w.be1;
    a.bq2 = pw + w.bq2; a.g2 = pw + w.g2; a.be2 = pw + w.be2; a.wq3 = pw + w.wq3; a.bq3 = pw + w.bq3;
    a.z0 = c.k.z0; a.mean0 = c.k.mean; a.std0 = c.k.stdv;
    a.noise = noise; a.cem_off = c.eps_cem_off; a.iter_len = c.eps_iter; a.term_off = c.eps_term_off; a.act_off = c.eps_act_off;
    a.u = u; a.prev_mean = prev_mean; a.action = action; a.metrics = metrics;
    a.elite_out = elite_out; a.score_out = score_out; a.value_out = value_out; a.mean_out = mean_out; a.std_out = std_out;
    a.eval_mode = prm->eval_mode; a.min_std = prm->min_std; a.temperature = prm->temperature; a.momentum = prm->momentum;
    a.omm = prm->one_minus_momentum; a.std_floor = prm->std_floor; a.std_floor_p = prm->std_floor_dev;
    for (int t = 0; t <= c.H && t < 17; ++t) a.disc[t] = prm->discount_pow[t];
    a.base = c.k.p1; a.bytes = (unsigned)c.k.p1_bytes;
    a.o_sync = rg.o_sync; a.o_xb = rg.o_xb; a.o_h1 = rg.o_h1; a.o_zp = rg.o_zp; a.o_rp = rg.o_rp; a.o_pp = rg.o_pp;
    a.o_qm = rg.o_qm; a.o_qp = rg.o_qp; a.o_val = rg.o_val; a.o_rl = rg.o_rl; a.o_mu = rg.o_mu; a.o_y2 = rg.o_y2; a.pi_cache = pi_cache_on(); a.xb_t = rg.xb_t; a.xb_g = rg.xb_g;
    a.stamps = g_p1_stamps;
    a.status = prm->status;
    a.pstatus = pack_status(c);
    {
        const char* e = getenv("TDMPC_P1_DEBUG_SKIP");   // test knob, read per launch (captured with the graph)
        a.debug_skip = e && atoi(e) ? 1 : 0;
    }
    // counters + error word zeroed by a kernel of our own, not hipMemsetAsync: in a replayed HIP graph the memset
    // node was seen writing a stale 16-byte pattern instead of zeros (the kernel then exits on a garbage error word
    // with the NaN-poisoned outputs; tests/test_gpu_plan.py::test_plan_reference_draws_device_equals_torch)
    hipLaunchKernelGGL(zero_words_kernel, dim3(1), dim3(P1_NG * 64 + 64), 0, c.s, (unsigned*)(c.k.p1 + rg.o_sync),
                       P1_NG * 64 + 64);
    HIPCHK(hipGetLastError());
    const size_t lds = p1_lds_bytes(c.H, a.K, w.A, c.T);
    if (p1_ks(w) == 4) hipLaunchKernelGGL(plan1_kernel<4>, dim3(P1_NG * P1_WPG), dim3(P1_NT), lds, c.s, a);
    else hipLaunchKernelGGL(plan1_kernel<6>, dim3(P1_NG * P1_WPG), dim3(P1_NT), lds, c.s, a);
    HIPCHK(hipGetLastError());
    return 0;
}

int setup_ctx(Ctx& c, const tdmpc_dims* d, const void* packed, void* ws, size_t ws_bytes, int batch, int H,
              int I, hipStream_t s, int extra_rows = 0) {
    if (!check_dims(d)) { snprintf(g_err, sizeof g_err, "bad dims"); return TDMPC_E_DIMS; }
    c.d = d;
    make_layout(d, &c.w);
    Work probe;
    make_work(d, c.w, nullptr, &probe, extra_rows);
    if (ws_bytes < probe.total) { snprintf(g_err, sizeof g_err, "workspace too small"); return TDMPC_E_SIZE; }
    make_work(d, c.w, (char*)ws, &c.k, extra_rows);
    c.pw = (const float*)packed; c.s = s;
    c.B = batch; c.N = d->num_samples; c.P = d->num_pi; c.T = c.N + c.P; c.H = H; c.path = TDMPC_PATH_AUTO;
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

// ---- the fused weight pack (tdmpc_pack_weights): ONE launch writes every region of the packed buffer -- fp32
// copies, transposes, weight panels, their x6 and x6q bf16 planes -- straight from the reference's tensors (the
// learner passes views of its flat parameter buffer, so a post-update repack is one kernel, capturable into the
// update's HIP graph). Each job's padded region is written whole (zeros where the layout pads), so no memset.
// The x6 / x6q planes are split from the source tensors directly (the same values as from the fp32 panel).
struct PackSrc {                 // a weight panel's source: rows [0, r0) of p0, then [r0, r0 + r1) of p1
    const float* p0; const float* p1;
    int r0, r1, sld, ncols;      // source row length; plain map: panel column k < ncols <- source column k
    int first;                   // first-layer map: panel [a | 0 | z | 0] <- source [z | a] (L = ncols, A below)
    int L, A, Ap;
};
__host__ __device__ inline float pack_val(const PackSrc& m, int r, int k) {
    const float* row;
    if (r < m.r0) row = m.p0 + (size_t)r * m.sld;
    else if (r < m.r0 + m.r1) row = m.p1 + (size_t)(r - m.r0) * m.sld;
    else return 0.f;
    int col;
    if (m.first) col = k < m.A ? m.L + k : (k >= m.Ap && k < m.Ap + m.L ? k - m.Ap : -1);
    else col = k < m.ncols ? k : -1;
    return col < 0 ? 0.f : row[col];
}
enum { PJ_COPY, PJ_TRANS, PJ_PANEL, PJ_X6, PJ_X6Q };
struct PackJob {
    int kind;
    int blk0;                    // first workgroup of this job in the launch
    size_t dst;                  // float offset into the packed buffer
    long work;                   // work items
    const float* src; int n, rows, cols;   // COPY: n values then zeros to `work`; TRANS: [rows][cols] -> [cols][rows]
    PackSrc m; int prow, pk;     // PANEL: [prow][pk] panel; X6 / X6Q: prow rows x pk k of the source map
};
static_assert(sizeof(PackJob) <= PACK_JOB_BYTES, "job-table slot");
constexpr int PACK_WG = 256, PACK_PER = 8;   // threads per workgroup, items per thread
// elements per item: an x6 / x6q lane's 8 values (16-B stores per plane), a panel's k quad, else one; items per
// thread: one for those (the split and the gathered reads of 4 - 8 values already give each thread its work), else
// PACK_PER
__host__ __device__ constexpr int pack_per_item(int kind) { return kind == PJ_X6 || kind == PJ_X6Q ? 8 : kind == PJ_PANEL ? 4 : 1; }
__host__ __device__ constexpr int pack_items(int kind) { return pack_per_item(kind) > 1 ? 1 : PACK_PER; }

__global__ void __launch_bounds__(PACK_WG) pack_fused_kernel(PackHdr* hdr, const PackJob* jobs, int nj, float* pw,
                                                              unsigned long long nonce, long nweights) {
    if (hdr->nonce != nonce) {
        // not the table this launch was issued for (the buffer was re-allocated, re-zeroed or re-keyed since): pack
        // nothing from it, poison every weight region and raise the buffer's sticky status (plans pass it on)
        for (long i = (long)blockIdx.x * PACK_WG + threadIdx.x; i < nweights; i += (long)gridDim.x * PACK_WG)
            pw[i] = __builtin_nanf("");
        if (blockIdx.x == 0 && threadIdx.x == 0)
            __hip_atomic_fetch_or(&hdr->status, TDMPC_STATUS_PACK_STALE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    // the workgroup's job: last job whose blk0 <= blockIdx.x (binary search over the job table)
    int lo = 0, hi = nj - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (jobs[mid].blk0 <= (int)blockIdx.x) lo = mid;
        else hi = mid - 1;
    }
    const PackJob& J = jobs[lo];
    const int epi = pack_per_item(J.kind), ipt = pack_items(J.kind);
    const long base = (long)(blockIdx.x - J.blk0) * PACK_WG * ipt;
    for (int u = 0; u < ipt; ++u) {
        const long i = (base + (long)u * PACK_WG + threadIdx.x) * epi;   // first element of the thread's item
        if (i >= J.work) break;
        switch (J.kind) {
            case PJ_COPY: pw[J.dst + i] = i < J.n ? J.src[i] : 0.f; break;
            case PJ_TRANS: {
                const long r = i % J.rows, c = i / J.rows;   // dst[c * rows + r] = src[r * cols + c]
                pw[J.dst + i] = J.src[r * J.cols + c];
                break;
            }
            case PJ_PANEL: {   // dst index i = pidx(r, k, pk): [r / 32][k / 4][r % 32][k % 4]; the item: one k quad
                const int rr = (i >> 2) & 31;
                const long q = i >> 7;
                const int kq = (int)(q % (J.pk / 4));
                const int r = (int)(q / (J.pk / 4)) * 32 + rr, k = kq * 4;
                *(float4*)(pw + J.dst + i) = make_float4(pack_val(J.m, r, k), pack_val(J.m, r, k + 1),
                                                         pack_val(J.m, r, k + 2), pack_val(J.m, r, k + 3));
                break;
            }
            case PJ_X6: case PJ_X6Q: {   // the item: one lane's 8 values of a block, 16 B per plane
                const int lane = (i >> 3) & 63;
                const long blk = i >> 9;
                int r, k0, k1;   // values j = 0..3 at k0 + j, j = 4..7 at k1 + j - 4
                if (J.kind == PJ_X6) {   // the x6 layout (Layout::x6): 32-row x 16-k blocks
                    const int G = (J.pk + 15) / 16;
                    const int g = (int)(blk % G), nb = (int)(blk / G);
                    r = 32 * nb + (lane & 31);
                    k0 = 16 * g + 4 * (lane >> 5);
                    k1 = k0 + 8;
                } else {                 // the x6q layout (Layout::x6q): 16-row x 32-k blocks
                    const int G = (J.pk + 31) / 32;
                    const int g = (int)(blk % G), nb = (int)(blk / G);
                    r = 16 * nb + (lane & 15);
                    k0 = 32 * g + 4 * (lane >> 4);
                    k1 = k0 + 16;
                }
                unsigned short hv[8], mv[8], lv[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int k = (j < 4 ? k0 : k1) + (j & 3);
                    const float x = k < J.pk && r < J.prow ? pack_val(J.m, r, k) : 0.f;
                    __bf16 h, m, l;
                    split3(x, h, m, l);
                    hv[j] = __builtin_bit_cast(unsigned short, h);
                    mv[j] = __builtin_bit_cast(unsigned short, m);
                    lv[j] = __builtin_bit_cast(unsigned short, l);
                }
                auto pk8 = [](const unsigned short (&v)[8]) {
                    return make_uint4(v[0] | (unsigned)v[1] << 16, v[2] | (unsigned)v[3] << 16, v[4] | (unsigned)v[5] << 16,
                                      v[6] | (unsigned)v[7] << 16);
                };
                uint4* d = (uint4*)(pw + J.dst);   // 1 KiB per plane and block, 16 B per lane
                d[(blk * 3 + 0) * 64 + lane] = pk8(hv);
                d[(blk * 3 + 1) * 64 + lane] = pk8(mv);
                d[(blk * 3 + 2) * 64 + lane] = pk8(lv);
                break;
            }
        }
    }
}

// ---- the folded first layer (latent_dim == mlp_dim; Layout::fold): W1z W3 and b1 + W1z b3 for both TOLD.next heads,
// from the packed fp32 panels (w1x's z columns [2M][Ap .. Ap + L), w3d [Lr][M], b3d, b1x), fp64 sums rounded once to
// fp32, then split into the x6q planes with the a columns of w1x in front. A step whose input latent columns hold the
// previous step's h2 = ELU(W2 h1 + b2) computes W1 [a; W3 h2 + b3] + b1 as [W1a | W1z W3] [a; h2] + (b1 + W1z b3).
struct FoldArgs {
    const float* W; int Kp, zoff;          // source first layer: fp32 panel [R][Kp], z in columns [zoff, zoff + L)
    const float* w3d; const float* b3; const float* b;   // W3 panel [Lr][M], b3 [L], the source bias [R]
    float* fw; float* bf;                  // W_z W3 [R][M] fp32 and b + W_z b3 [R]
    unsigned short* x6; int kind, pk;      // planes of [W_a | W_z W3] (k < zoff from W, then fw): kind 0 x6q, 1 x6
    int M, L;
};
__global__ void __launch_bounds__(256) fold_gemm_kernel(const FoldArgs a) {
    // 16 x 16 output tile per workgroup: rows i [0, R), columns j of W3 [0, M) -- tile column M / 16 is the bias
    // column (j = M: b3)
    __shared__ double sA[16][17], sB[16][17];
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    const int i0 = blockIdx.y * 16, j0 = blockIdx.x * 16;
    const int i = i0 + ty, j = j0 + tx;
    double acc = 0.0;
    for (int l0 = 0; l0 < a.L; l0 += 16) {
        const int la = l0 + tx, lb = l0 + ty;
        sA[ty][tx] = la < a.L ? (double)a.W[pidx(i0 + ty, a.zoff + la, a.Kp)] : 0.0;
        double b = 0.0;
        if (lb < a.L) b = j < a.M ? (double)a.w3d[pidx(lb, j, a.M)] : (j == a.M ? (double)a.b3[lb] : 0.0);
        sB[ty][tx] = b;
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 16; ++k) acc = fma(sA[ty][k], sB[k][tx], acc);
        __syncthreads();
    }
    if (j < a.M) a.fw[(size_t)i * a.M + j] = (float)acc;
    else if (j == a.M) a.bf[i] = (float)((double)a.b[i] + acc);
}
__global__ void __launch_bounds__(256) fold_split_kernel(const FoldArgs a, long work) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= work) return;
    const int j = (int)(i & 7), lane = (int)((i >> 3) & 63);
    const long blk = i >> 9;
    int r, k;
    if (a.kind == 0) {   // x6q: 16-row x 32-k blocks (the wide kernels)
        const int G = (a.pk + 31) / 32;
        const int g = (int)(blk % G), nb = (int)(blk / G);
        r = 16 * nb + (lane & 15);
        k = 32 * g + 16 * (j >> 2) + 4 * (lane >> 4) + (j & 3);
    } else {             // x6: 32-row x 16-k blocks (the chain kernels)
        const int G = (a.pk + 15) / 16;
        const int g = (int)(blk % G), nb = (int)(blk / G);
        r = 32 * nb + (lane & 31);
        k = 16 * g + 8 * (j >> 2) + 4 * (lane >> 5) + (j & 3);
    }
    float x = 0.f;
    if (k < a.zoff) x = a.W[pidx(r, k, a.Kp)];
    else if (k < a.zoff + a.M && k < a.pk) x = a.fw[(size_t)r * a.M + (k - a.zoff)];
    __bf16 h, m, l;
    split3(x, h, m, l);
    a.x6[(blk * 3 + 0) * 512 + lane * 8 + j] = __builtin_bit_cast(unsigned short, h);
    a.x6[(blk * 3 + 1) * 512 + lane * 8 + j] = __builtin_bit_cast(unsigned short, m);
    a.x6[(blk * 3 + 2) * 512 + lane * 8 + j] = __builtin_bit_cast(unsigned short, l);
}
int fold_one(const Layout& w, float* pw, hipStream_t s, size_t W, int R, int Kp, int zoff, size_t b, size_t fw,
             size_t bf, size_t x6, int kind, int pk, bool gemm = true) {
    FoldArgs f;
    memset(&f, 0, sizeof f);
    f.W = pw + W; f.Kp = Kp; f.zoff = zoff; f.w3d = pw + w.w3d; f.b3 = pw + w.b3d; f.b = pw + b;
    f.fw = pw + fw; f.bf = pw + bf; f.x6 = (unsigned short*)(pw + x6); f.kind = kind; f.pk = pk;
    f.M = w.M; f.L = w.L;
    if (gemm) {
        hipLaunchKernelGGL(fold_gemm_kernel, dim3(w.M / 16 + 1, R / 16), dim3(256), 0, s, f);
        HIPCHK(hipGetLastError());
    }
    const long work = kind == 0 ? (long)(R / 16) * ((pk + 31) / 32) * 512 : (long)((R + 31) / 32) * ((pk + 15) / 16) * 512;
    hipLaunchKernelGGL(fold_split_kernel, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, s, f, work);
    HIPCHK(hipGetLastError());
    return 0;
}
int pack_fold(const Layout& w, float* pw, hipStream_t s) {
    int rc, r, k;
    // TOLD.next (both heads, the wide kernel's x6q): [W1a | W1z W3], b1 + W1z b3
    if ((rc = fold_one(w, pw, s, w.w1x, 2 * w.M, w.Kx, w.Ap, w.b1x, w.fold_w, w.bfw, w.x6qw, 0, w.Kx))) return rc;
    // (the same product split again into the chain kernels' x6 layout)
    x6_shape(w, X6_W1X, &r, &k);
    if ((rc = fold_one(w, pw, s, w.w1x, 2 * w.M, w.Kx, w.Ap, w.b1x, w.fold_w, w.bfw, w.fw1_x6, 1, k, false))) return rc;
    // pi (chain x6): [Wp1 W3], bp1 + Wp1 b3
    x6_shape(w, X6_WP1, &r, &k);
    if ((rc = fold_one(w, pw, s, w.wp1, w.M, w.Lp, 0, w.bp1, w.fold_p, w.fpi_b, w.fpi_x6, 1, k))) return rc;
    // Q1 | Q2 (chain x6): [Wq1a | Wq1z W3], bq1 + Wq1z b3
    x6_shape(w, X6_WQ1X, &r, &k);
    return fold_one(w, pw, s, w.wq1x, 2 * w.M, w.Kx, w.Ap, w.bq1x, w.fold_q, w.fq_b, w.fq_x6, 1, k);
}

// The job list of a layout and the reference tensors t (state_dict order, tdmpc_num_param_tensors of them)
void pack_jobs(const Layout& w, const float* const* t, std::vector<PackJob>& jobs) {
    const int M = w.M, L = w.L, A = w.A;
    auto job = [&](int kind, size_t dst, long work) -> PackJob& {
        PackJob j;
        memset(&j, 0, sizeof j);
        j.kind = kind; j.dst = dst; j.work = work;
        jobs.push_back(j);
        return jobs.back();
    };
    auto cp = [&](size_t dst, const float* src, int n) {   // zero tail to the 64-float slot take() reserved
        PackJob& j = job(PJ_COPY, dst, (long)rup(n, 64));
        j.src = src; j.n = n;
    };
    auto tr = [&](size_t dst, const float* src, int rows, int cols) {
        PackJob& j = job(PJ_TRANS, dst, (long)rows * cols);
        j.src = src; j.rows = rows; j.cols = cols;
    };
    auto msrc = [&](const float* p0, const float* p1, int r0, int r1, int sld, int ncols, int first) {
        PackSrc m;
        memset(&m, 0, sizeof m);
        m.p0 = p0; m.p1 = p1 ? p1 : p0; m.r0 = r0; m.r1 = r1; m.sld = sld; m.ncols = ncols; m.first = first;
        m.L = L; m.A = A; m.Ap = w.Ap;
        return m;
    };
    auto panel = [&](size_t dst, const PackSrc& m, int prow, int pk) {
        PackJob& j = job(PJ_PANEL, dst, (long)rup(prow, 32) * pk);
        j.m = m; j.prow = prow; j.pk = pk;
    };
    int i = 0;
    if (w.modality == 0) {
        tr(w.enc_w1t, t[i++], w.E, w.obs_dim);
        cp(w.enc_b1, t[i++], w.E);
        if (w.enc_norm) { cp(w.enc_lng, t[i++], w.E); cp(w.enc_lnb, t[i++], w.E); }
        tr(w.enc_w2t, t[i++], L, w.E);
        cp(w.enc_b2, t[i++], L);
    } else {
        static const int ks[4] = {7, 5, 3, 3};
        int cin = w.img_c;
        for (int c = 0; c < 4; ++c) {
            const float* cw = t[i++];
            cp(w.cw[c], cw, w.nch * cin * ks[c] * ks[c]);
            tr(w.cwt[c], cw, w.nch, cin * ks[c] * ks[c]);
            cp(w.cb[c], t[i++], w.nch);
            cin = w.nch;
        }
        tr(w.pl_wt, t[i++], L, w.flat);
        cp(w.pl_b, t[i++], L);
    }
    const int KI = L + A;
    const float* const* dyn = t + i;        // 0.w 0.b 2.w 2.b 4.w 4.b
    const float* const* rew = dyn + 6;
    const float* const* pi = rew + 6;
    const float* const* q1 = pi + 6;        // 0.w 0.b 1.w 1.b 3.w 3.b 4.w 4.b 6.w 6.b
    const float* const* q2 = q1 + 10;
    const PackSrc sW1X = msrc(dyn[0], rew[0], M, M, KI, L, 1), sW2D = msrc(dyn[2], nullptr, M, 0, M, M, 0),
                  sW2R = msrc(rew[2], nullptr, M, 0, M, M, 0), sW3D = msrc(dyn[4], nullptr, L, 0, M, M, 0),
                  sWP1 = msrc(pi[0], nullptr, M, 0, L, L, 0), sWP2 = msrc(pi[2], nullptr, M, 0, M, M, 0),
                  sWP3 = msrc(pi[4], nullptr, A, 0, M, M, 0), sWQ1X = msrc(q1[0], q2[0], M, M, KI, L, 1),
                  sWQ2 = msrc(q1[4], q2[4], M, M, M, M, 0);
    panel(w.w1x, sW1X, 2 * M, w.Kx);
    cp(w.b1x, dyn[1], M); cp(w.b1x + M, rew[1], M);
    panel(w.w2d, sW2D, M, M); cp(w.b2d, dyn[3], M);
    panel(w.w3d, sW3D, w.Lr, M); cp(w.b3d, dyn[5], L);
    panel(w.w2r, sW2R, M, M); cp(w.b2r, rew[3], M);
    cp(w.w3r, rew[4], M); cp(w.b3r, rew[5], 1);
    panel(w.wp1, sWP1, M, w.Lp); cp(w.bp1, pi[1], M);
    panel(w.wp2, sWP2, M, M); cp(w.bp2, pi[3], M);
    panel(w.wp3, sWP3, w.Ar, M); cp(w.bp3, pi[5], A);
    panel(w.wq1x, sWQ1X, 2 * M, w.Kx);
    panel(w.wq2, sWQ2, 2 * M, M);
    const float* const* qs[2] = {q1, q2};
    for (int q = 0; q < 2; ++q) {
        const float* const* Q = qs[q];
        // (the 2M-float LN / bias slots hold both heads: each copy's zero tail stops at the next head's start)
        PackJob* jb;
        cp(w.bq1x + q * M, Q[1], M); cp(w.g1 + q * M, Q[2], M); cp(w.be1 + q * M, Q[3], M);
        cp(w.bq2 + q * M, Q[5], M); cp(w.g2 + q * M, Q[6], M); cp(w.be2 + q * M, Q[7], M);
        cp(w.wq3 + q * M, Q[8], M);
        jb = &job(PJ_COPY, w.bq3 + q, 1);
        jb->src = Q[9]; jb->n = 1;
    }
    const PackSrc* xs[X6_N] = {&sW1X, &sW2D, &sW2R, &sW3D, &sWP1, &sWP2, &sWP3, &sWQ1X, &sWQ2};
    for (int x = 0; x < X6_N; ++x) {
        int rows, k;
        x6_shape(w, x, &rows, &k);
        PackJob& j = job(PJ_X6, w.x6[x], (long)((rows + 31) / 32) * ((k + 15) / 16) * 512);
        j.m = *xs[x]; j.prow = rows; j.pk = k;
    }
    for (int x = 0; x < X6_N; ++x) {
        int rows, k;
        x6_shape(w, x, &rows, &k);
        PackJob& j = job(PJ_X6Q, w.x6q[x], (long)((rows + 15) / 16) * ((k + 31) / 32) * 512);
        j.m = *xs[x]; j.prow = rows; j.pk = k;
    }
}

// The job table lives in the caller's packed buffer (Layout::jobtab), so it lives and dies with that buffer and the
// HIP graphs the caller captured over it -- nothing device-side is global or leaks. Every pack outside a stream
// capture uploads header + table (an async copy from a pinned staging buffer kept per packed buffer, whose previous
// copy's event is waited for before it is rewritten -- long done by then); a pack inside a capture uploads nothing and
// requires the table last uploaded into that buffer to be this one (pack once before capturing, as the learner does).
// Staleness is checked on the device, not trusted from the host record: every launch carries the nonce of the table
// the record says is in the buffer and pack_fused_kernel compares it with the header's (a buffer re-allocated at a
// recorded address or zeroed again fails loudly: NaN weights + TDMPC_STATUS_PACK_STALE). An uncaptured pack keeps the
// record's nonce when its table is unchanged (graphs captured over the buffer stay valid) and draws a new one
// otherwise; once a capture has packed from a buffer, an uncaptured pack with OTHER tensors is refused (it would
// silently re-point the captured graph) until tdmpc_pack_forget drops the record -- after which such a graph's pack
// sees a nonce mismatch and fails loudly. Records live until tdmpc_pack_forget; only their pinned staging buffers are
// recycled (PACK_PINNED of them, least recently used first). One mutex guards it.
struct PackTable {
    std::vector<PackJob> host; const float* pw; int device;
    unsigned long long nonce; bool captured;
    char* pinned; hipEvent_t done; bool recorded;
};
std::vector<PackTable> g_pack_tables;   // most recently used last
std::mutex g_pack_mu;
constexpr size_t PACK_PINNED = 64;
constexpr size_t PACK_UPLOAD_BYTES = (size_t)PACK_HDR_BYTES + (size_t)PACK_MAX_JOBS * sizeof(PackJob);

void pack_table_unpin(PackTable& t) {
    if (t.recorded) (void)hipEventSynchronize(t.done);
    if (t.done) (void)hipEventDestroy(t.done);
    if (t.pinned) (void)hipHostFree(t.pinned);
    t.pinned = nullptr;
    t.done = nullptr;
    t.recorded = false;
}

// table nonces: never 0 (a zeroed buffer's header) and distinct across processes and buffers with high probability
unsigned long long pack_next_nonce() {
    static std::atomic<unsigned long long> ctr{0};
    static const unsigned long long base =
        ((unsigned long long)std::chrono::high_resolution_clock::now().time_since_epoch().count() * 0x9E3779B97F4A7C15ull) ^
        ((unsigned long long)getpid() << 32);
    for (;;) {
        unsigned long long z = base + 0x9E3779B97F4A7C15ull * (ctr.fetch_add(1) + 1);   // splitmix64 finaliser
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        if (z) return z;
    }
}

int launch_pack(std::vector<PackJob>& jobs, const Layout& w, float* pw, hipStream_t s) {
    if (jobs.size() > (size_t)PACK_MAX_JOBS) {
        snprintf(g_err, sizeof g_err, "tdmpc_pack_weights: %zu jobs > %d", jobs.size(), PACK_MAX_JOBS);
        return TDMPC_E_SIZE;
    }
    int blk = 0;
    for (PackJob& j : jobs) {
        j.blk0 = blk;
        const long per_blk = (long)PACK_WG * pack_items(j.kind) * pack_per_item(j.kind);
        blk += (int)((j.work + per_blk - 1) / per_blk);
    }
    const size_t nb = jobs.size() * sizeof(PackJob);
    int device = 0;
    HIPCHK(hipGetDevice(&device));
    PackHdr* hdr = (PackHdr*)(pw + w.jobtab);
    PackJob* dev = (PackJob*)((char*)hdr + PACK_HDR_BYTES);
    unsigned long long nonce = 0;
    {
        std::lock_guard<std::mutex> lock(g_pack_mu);
        size_t hit = g_pack_tables.size();
        for (size_t i = 0; i < g_pack_tables.size(); ++i)
            if (g_pack_tables[i].pw == pw && g_pack_tables[i].device == device) { hit = i; break; }
        const bool same = hit < g_pack_tables.size() && g_pack_tables[hit].host.size() == jobs.size() &&
                          !memcmp(g_pack_tables[hit].host.data(), jobs.data(), nb);
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        HIPCHK(hipStreamIsCapturing(s, &cs));
        if (cs != hipStreamCaptureStatusNone) {
            if (!same) {
                snprintf(g_err, sizeof g_err, hit == g_pack_tables.size()
                         ? "tdmpc_pack_weights: no table uploaded into this buffer while capturing (pack once before capture)"
                         : "tdmpc_pack_weights: new tensors while capturing (pack once before capture)");
                return TDMPC_E_DIMS;
            }
            g_pack_tables[hit].captured = true;
        } else {
            if (hit < g_pack_tables.size() && g_pack_tables[hit].captured && !same) {
                snprintf(g_err, sizeof g_err, "tdmpc_pack_weights: a captured graph packs into this buffer from other "
                         "tensors; call tdmpc_pack_forget(packed) first (that graph's pack then fails loudly)");
                return TDMPC_E_DIMS;
            }
            if (hit == g_pack_tables.size()) {
                g_pack_tables.push_back(PackTable{{}, pw, device, 0, false, nullptr, nullptr, false});
                hit = g_pack_tables.size() - 1;
            }
            PackTable& t = g_pack_tables[hit];
            if (!same || !t.nonce) t.nonce = pack_next_nonce();
            if (!t.pinned) {
                size_t npin = 0;
                for (const PackTable& o : g_pack_tables) npin += o.pinned != nullptr;
                for (size_t i = 0; npin >= PACK_PINNED && i < g_pack_tables.size(); ++i)
                    if (g_pack_tables[i].pinned) { pack_table_unpin(g_pack_tables[i]); --npin; }
                HIPCHK(hipHostMalloc((void**)&t.pinned, PACK_UPLOAD_BYTES, hipHostMallocDefault));
                HIPCHK(hipEventCreateWithFlags(&t.done, hipEventDisableTiming));
            }
            if (t.recorded) HIPCHK(hipEventSynchronize(t.done));
            PackHdr h;
            memset(&h, 0, sizeof h);
            h.nonce = t.nonce; h.status = 0; h.njobs = (int)jobs.size();
            memset(t.pinned, 0, PACK_HDR_BYTES);
            memcpy(t.pinned, &h, sizeof h);
            memcpy(t.pinned + PACK_HDR_BYTES, jobs.data(), nb);
            HIPCHK(hipMemcpyAsync(hdr, t.pinned, PACK_HDR_BYTES + nb, hipMemcpyHostToDevice, s));
            HIPCHK(hipEventRecord(t.done, s));
            t.recorded = true;
            t.host = jobs;
        }
        nonce = g_pack_tables[hit].nonce;
        PackTable t = std::move(g_pack_tables[hit]);   // most recently used last
        g_pack_tables.erase(g_pack_tables.begin() + hit);
        g_pack_tables.push_back(std::move(t));
    }
    hipLaunchKernelGGL(pack_fused_kernel, dim3((unsigned)blk), dim3(PACK_WG), 0, s, hdr, (const PackJob*)dev,
                       (int)jobs.size(), pw, nonce, (long)w.jobtab);
    HIPCHK(hipGetLastError());
    return 0;
}

}  // namespace

namespace tdmpc_internal {
// error text for tdmpc_last_error() from the other translation units of the library (replay_kernels.hip)
void set_error(const char* msg) { snprintf(g_err, sizeof g_err, "%s", msg); }
}  // namespace tdmpc_internal

// ================================================================================================ C ABI
extern "C" {

int tdmpc_abi_version(void) { return TDMPC_ABI_VERSION; }

// Diagnostic: later persistent plans record per-hand-off realtime stamps into `dev` (device, 2048 uint64; NULL off).
int tdmpc_debug_plan1_stamps(void* dev) {
    g_p1_stamps = (unsigned long long*)dev;
    return 0;
}

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

// ---------------------------------------------------------------- reference-order draws in one launch
// The reference takes its planning noise from torch's global device generator, one normal_/randn launch per
// draw (tdmpc.py:117 per horizon step, 131 and 91 per iteration, 158): at humanoid sizes 18 launches per env.
// Each of those is ATen's grid-stride Philox kernel, so the value of element li of a draw is a pure function of
// (seed, draw's counter offset, li, the draw's grid): this kernel recomputes every element of every draw of
// every env in one pass, one thread per stream float.
// Per call a table of the env's draws (the same for every env): draw k covers blocks [blk[k], blk[k+1]) of the
// env's grid row, so a block belongs to one draw and finds it with a scalar search.
constexpr int REF_MAX_DRAWS = 96;
struct RefNormalsArgs {
    float* noise;
    int64_t env_stride;
    uint64_t seed, offset, env_adv;   // generator state at the call; counter advance per env
    const uint64_t* gen_state;        // non-null: {seed, offset} read from device memory when the kernel runs
    int32_t ndraw;
    int32_t blk[REF_MAX_DRAWS + 1];   // first block of each draw
    int32_t n[REF_MAX_DRAWS];         // elements
    int32_t out[REF_MAX_DRAWS];       // float offset in the env stream
    int32_t S[REF_MAX_DRAWS];         // ATen grid stride (threads)
    uint32_t coff[REF_MAX_DRAWS];     // counter offset from the env's first draw
};

// rocrand's Box-Muller (normal_distribution4 on one Philox output) with the instruction sequence of the
// normal_ kernel in the installed torch build (its code object, disassembled): logf as v_log_f32 plus the
// two-product ln2 scaling finished by a separate ADD, which a newer compiler fuses into one FMA (a 1-2 ulp
// difference in ~15% of values); sqrtf correctly rounded; sin/cos native on v / 2pi. Fused multiply-adds are
// written out, everything else is kept unfused.
DEVI float torch_bm_log(float u) {
#pragma clang fp contract(off)
    const bool tiny = u < 0x1p-126f;
    const float L = __builtin_amdgcn_logf(tiny ? ldexpf(u, 32) : u);   // log2
    const float hi = L * 0x1.62e42ep-1f;                                  // ln2 (hi)
    float e = fmaf(L, 0x1.62e42ep-1f, -hi);
    e = fmaf(0x1.efa39ep-25f, L, e);                                      // ln2 (lo)
    const float r = fabsf(L) < INFINITY ? hi + e : L;
    return r - (tiny ? 0x1.62e430p+4f : 0.f);                             // 32 ln2
}

DEVI float torch_normal_component(uint4 r, int c) {
#pragma clang fp contract(off)
    const unsigned x = c < 2 ? r.x : r.z, y = c < 2 ? r.y : r.w;
    const float u = fmaf((float)x, 0x1p-32f, 0x1p-32f);                   // ROCRAND_2POW32_INV
    const float v = fmaf((float)y, 0x1.921fb6p-30f, 0x1.921fb6p-30f);     // ROCRAND_2POW32_INV_2PI
    const float s = sqrtf(-2.0f * torch_bm_log(u));
    const float t = v * 0x1.45f306p-3f;
    return ((c & 1) ? __builtin_amdgcn_cosf(t) : __builtin_amdgcn_sinf(t)) * s;
}

__global__ void __launch_bounds__(256) ref_normals_kernel(RefNormalsArgs a) {
    const int e = blockIdx.y, bx = blockIdx.x;
    int k = 0;
    while (k + 1 < a.ndraw && a.blk[k + 1] <= bx) ++k;
    const int li = (bx - a.blk[k]) * 256 + (int)threadIdx.x;
    if (li >= a.n[k]) return;
    const int S = a.S[k];
    const int j = li < S ? 0 : li / S;   // ATen grid-stride pass (0 unless the draw exceeds the grid cap)
    uint64_t seed = a.seed, off = a.offset;
    if (a.gen_state) seed = a.gen_state[0], off = a.gen_state[1];
    hiprandStatePhilox4_32_10_t st;
    hiprand_init(seed, (unsigned long long)(li - j * S), off + (uint64_t)e * a.env_adv + a.coff[k], &st);
    uint4 r = hiprand4(&st);
    for (int p = 0; p < j / 4; ++p) r = hiprand4(&st);
    const float x = torch_normal_component(r, j & 3);
    a.noise[e * a.env_stride + a.out[k] + li] = x * 1.0f + 0.0f;   // transformation::normal(x, 0, 1)
}

int tdmpc_reference_normals(const tdmpc_dims* d, float* noise, int32_t B, int64_t env_stride, int32_t H,
                            int32_t I, int32_t eval_mode, uint64_t seed, uint64_t offset, const uint64_t* gen_state,
                            int32_t grid_cap, uint64_t* offset_advance, void* stream) {
    if (!d || !noise || !offset_advance) return TDMPC_E_NULL;
    if (!check_dims(d)) return TDMPC_E_DIMS;
    const int64_t A = d->action_dim, N = d->num_samples, P = d->num_pi, T = N + P;
    const int64_t per_env = (int64_t)tdmpc_noise_floats(d, H, I) - (eval_mode ? A : 0);
    if (B < 1 || H < 1 || I < 1 || grid_cap < 1 || env_stride < (int64_t)tdmpc_noise_floats(d, H, I)) {
        snprintf(g_err, sizeof g_err, "reference_normals: batch %d horizon %d iterations %d grid_cap %d stride %lld",
                 B, H, I, grid_cap, (long long)env_stride);
        return TDMPC_E_DIMS;
    }
    RefNormalsArgs a{};
    // ATen calc_execution_policy: block 256, grid min(cap, ceil(n/256)), advance 4 per unrolled pass
    auto stride = [&](int64_t n) { return 256 * std::min<int64_t>(grid_cap, (n + 255) / 256); };
    auto adv = [&](int64_t n) { return (uint64_t)(((n - 1) / (stride(n) * 4) + 1) * 4); };
    int64_t out = 0, blk = 0;
    uint64_t coff = 0;
    auto draw = [&](int64_t n) {
        const int k = a.ndraw++;
        a.blk[k] = (int32_t)blk, a.n[k] = (int32_t)n, a.out[k] = (int32_t)out, a.S[k] = (int32_t)stride(n);
        a.coff[k] = (uint32_t)coff;
        blk += (n + 255) / 256, out += n, coff += adv(n);
    };
    const int64_t D = (P > 0 ? H : 0) + 2 * I + (eval_mode ? 0 : 1);
    if (D > REF_MAX_DRAWS || per_env >= (1ll << 31)) {
        snprintf(g_err, sizeof g_err, "reference_normals: %lld draws (max %d), %lld floats per env", (long long)D,
                 REF_MAX_DRAWS, (long long)per_env);
        return TDMPC_E_DIMS;
    }
    if (P > 0)
        for (int t = 0; t < H; ++t) draw(P * A);   // tdmpc.py:117 (helper.py:88), one per horizon step
    for (int i = 0; i < I; ++i) {
        draw((int64_t)H * N * A);                   // tdmpc.py:131
        draw(T * A);                                // tdmpc.py:91 (pi at the horizon)
    }
    if (!eval_mode) draw(A);                        // tdmpc.py:158
    a.blk[a.ndraw] = (int32_t)blk;
    a.noise = noise;
    a.env_stride = env_stride;
    a.seed = seed, a.offset = offset, a.env_adv = coff, a.gen_state = gen_state;
    *offset_advance = (uint64_t)B * coff;
    hipLaunchKernelGGL(ref_normals_kernel, dim3((unsigned)blk, (unsigned)B), dim3(256), 0, (hipStream_t)stream, a);
    HIPCHK(hipGetLastError());
    return 0;
}

int tdmpc_num_param_tensors(const tdmpc_dims* d) {
    if (!d) return TDMPC_E_NULL;
    return (d->modality ? 10 : (d->enc_norm ? 6 : 4)) + 6 + 6 + 6 + 10 + 10;
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
    for (int i = 0; i < n; ++i)
        if (!t[i]) return TDMPC_E_NULL;
    std::vector<PackJob> jobs;
    pack_jobs(w, t, jobs);
    int rc = launch_pack(jobs, w, (float*)packed, (hipStream_t)stream);
    if (rc) return rc;
    if (w.fold && (rc = pack_fold(w, (float*)packed, (hipStream_t)stream))) return rc;
    if (!w.nqs) return 0;
    // helper.q's LayerNorm-1 statistics block from the packed first layer (wide_heads.inc): Gram, Cholesky, x6q
    float* pw = (float*)packed;
    QStatArgs q;
    memset(&q, 0, sizeof q);
    q.W1 = pw + w.wq1x; q.b1 = pw + w.bq1x; q.gram = (double*)(pw + w.qs_gram);
    q.M = w.M; q.Kx = w.Kx; q.A = w.A; q.L = w.L; q.Ap = w.Ap; q.n = w.nqs;
    q.S = (unsigned short*)(pw + w.x6qs); q.bs = pw + w.bqs; q.nsr = w.nsr; q.g1s = (int)(rup(w.Kx, 32) / 32);
    q.F = (unsigned short*)(pw + w.x6qf); q.bf = pw + w.bqf; q.g1 = pw + w.g1;
    const hipStream_t s = (hipStream_t)stream;
    const int nt = (w.nqs + 15) / 16;
    hipLaunchKernelGGL(qstat_gram_kernel, dim3(nt, nt, 2), dim3(256), 0, s, q);
    HIPCHK(hipGetLastError());
    const size_t lds = ((size_t)w.nqs * (w.nqs + 1) / 2 + w.nqs) * 8;
    hipLaunchKernelGGL(qstat_chol_kernel, dim3(2), dim3(1024), lds, s, q);
    HIPCHK(hipGetLastError());
    return 0;
}

int tdmpc_pack_forget(const void* packed) {
    std::lock_guard<std::mutex> lock(g_pack_mu);
    for (size_t i = 0; i < g_pack_tables.size(); ++i)
        if (g_pack_tables[i].pw == (const float*)packed) {
            pack_table_unpin(g_pack_tables[i]);
            g_pack_tables.erase(g_pack_tables.begin() + i);
            break;
        }
    return 0;
}

int tdmpc_debug_pack_check(const tdmpc_dims* d, const int64_t* numel, int32_t n) {
    // Host-only bounds check of the fused pack's job table (no HIP call): every write inside the layout, every
    // read inside its source tensor. Tensor i is given the fake base address (i + 1) << 40.
    if (!d || !numel) return TDMPC_E_NULL;
    if (!check_dims(d)) return TDMPC_E_DIMS;
    Layout w;
    make_layout(d, &w);
    if (n != tdmpc_num_param_tensors(d)) return TDMPC_E_DIMS;
    std::vector<const float*> t(n);
    for (int i = 0; i < n; ++i) t[i] = (const float*)((uintptr_t)(i + 1) << 40);
    std::vector<PackJob> jobs;
    pack_jobs(w, t.data(), jobs);
    auto in_tensor = [&](const float* p, long last) -> bool {   // reads p[0 .. last]
        const uintptr_t u = (uintptr_t)p;
        const long i = (long)(u >> 40) - 1;
        if (i < 0 || i >= n) return false;
        const long off = (long)((u & (((uintptr_t)1 << 40) - 1)) / 4);
        return off + last < numel[i];
    };
    auto src_ok = [&](const PackSrc& m, int maxk) -> bool {
        const int maxcol = m.first ? m.L + m.A - 1 : std::min(maxk, m.ncols - 1);
        if (m.r0 > 0 && !in_tensor(m.p0, (long)(m.r0 - 1) * m.sld + maxcol)) return false;
        if (m.r1 > 0 && !in_tensor(m.p1, (long)(m.r1 - 1) * m.sld + maxcol)) return false;
        return true;
    };
    for (size_t j = 0; j < jobs.size(); ++j) {
        const PackJob& J = jobs[j];
        const double end = J.kind == PJ_X6 || J.kind == PJ_X6Q ? (double)J.dst + 1.5 * J.work : (double)(J.dst + J.work);
        bool ok = end <= (double)w.total;
        if (J.kind == PJ_COPY) ok = ok && J.n <= J.work && in_tensor(J.src, J.n - 1);
        else if (J.kind == PJ_TRANS) ok = ok && in_tensor(J.src, (long)J.rows * J.cols - 1);
        else ok = ok && src_ok(J.m, J.pk - 1);
        if (!ok) {
            snprintf(g_err, sizeof g_err, "pack job %d (kind %d, dst %zu) out of bounds", (int)j, J.kind, J.dst);
            return TDMPC_E_SIZE;
        }
    }
    return (int)jobs.size();
}

int tdmpc_encode(const tdmpc_dims* d, const void* packed, const void* obs, int32_t obs_is_u8, int32_t batch,
                 void* workspace, float* z0, void* stream) {
    if (!d || !packed || !obs || !z0 || !workspace) return TDMPC_E_NULL;
    Ctx c;
    tdmpc_sizes sz;
    int rc = tdmpc_sizes_for(d, &sz);
    if (rc) return rc;
    if ((rc = setup_ctx(c, d, packed, workspace, sz.workspace_bytes, batch, 1, 1, (hipStream_t)stream))) return rc;
    if ((rc = encode(c, obs, obs_is_u8, batch, nullptr, 0))) return rc;
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
    if (prm->path < 0 || prm->path > TDMPC_PATH_WIDE) { snprintf(g_err, sizeof g_err, "bad path"); return TDMPC_E_DIMS; }
    c.path = prm->path == TDMPC_PATH_CHAIN64 ? TDMPC_PATH_CHAIN_X6 : prm->path;   // (64-row blocks retired: path 6)
    const int N = c.N, P = c.P, T = c.T;
    // TDMPC_PATH_PERSIST: the persistent plan where it applies (one env, supported shape), the auto path elsewhere
    if (c.path == TDMPC_PATH_PERSIST && !use_plan1(c)) c.path = TDMPC_PATH_AUTO;
    // z0 = h(obs) and mean = 0 (warm: prev_mean shifted), std = 2
    if ((rc = encode(c, obs, obs_is_u8, B, prev_mean, prm->warm_start, 0, 2.f, prm->warm_flags))) return rc;
    if (use_plan1(c))
        return plan1_launch(c, prm, noise, u, prev_mean, action, metrics, elite_out, score_out, value_out, mean_out, std_out);
    if ((rc = prep(c, noise, 0, c.k.z0))) return rc;
    if (z0c_eligible(c)) {
        if ((rc = z0c_launch(c))) return rc;
        c.z0c_ready = 1;
    }
    {   // latent 512: the sampled rows' rollout on the wide kernel at every t, through the folded first layer
        const RowMap rm0 = {N, T, 0};
        c.fold_ok = fold_on() && c.w.fold && H > 1 && use_wide(c, B * N, rm0, c.z0c_ready != 0) &&
                    use_wide(c, B * N, rm0, false);
        // the terminal pi / Q of the sampled rows on the chain x6 kernels with folded first layers (the wide heads
        // carry no folded form): then the last step stores h2 too and z_H is never formed
        c.fold_heads = c.fold_ok && !use_wide_heads(c) && use_x6(c) && use_chain(c, B * N, 1, CK_PI) &&
                       use_chain(c, B * N, 2, CK_Q) && (P == 0 || use_chain(c, B * P, 2, CK_Q));
        // the policy rows' pre-rollout (iteration 0's pi + TOLD.next on the chain kernels) through the folded layers
        // too: needs the 32-row x6 chain kernel for their steps (its h2 epilogue)
        if (c.fold_heads && P > 0 && use_chain(c, B * P, 2, CK_STEP) && use_chain(c, B * P, 1, CK_PI)) {
            const ChainArgs probe = chain0(c, B * P, RowMap{P, T, N}, 0, c.Kx, 0, 2);
            c.fold_policy = probe.rb == 32 && probe.x6;
        }
    }

    // pi pre-rollout (tdmpc.py:113-118) fused with CEM iteration 0: at each step t the policy rows get
    // pi(z_t) first, then ONE TOLD.next launch advances all T rows of every env (rollout rows with the
    // sampled candidates, pi rows with their pi actions). The pi rows' rollout, reward prefix and z_H are
    // identical in every CEM iteration (same z0, same pi actions), so later iterations only roll out the N
    // sampled rows and reuse rows N..T-1 of X_t, G and rlast.
    const RowMap all = {T, T, 0};
    const RowMap pm = {P, T, N};
    const RowMap rm = {N, T, 0};
    if (P > 0) {
        for (int t = 0; t < H; ++t) {
            if ((rc = policy(c, t, B * P, pm, noise, c.eps_env, P, (long)t * P * c.A, prm->min_std, nullptr,
                             c.fold_policy && t >= 1)))
                return rc;
            if ((rc = step_next(c, t, B * T, all, prm->discount_pow[t], t == 0, t == H - 1)))
                return rc;
        }
    }
    CemArgs ca;
    memset(&ca, 0, sizeof ca);
    ca.H = H; ca.N = N; ca.P = P; ca.T = T; ca.A = c.A; ca.K = d->num_elites; ca.Kx = c.Kx;
    ca.Hmax = d->max_horizon; ca.I = I;
    ca.Tw = T; ca.NE = T; ca.pi_base = 0;
    ca.X = c.k.X; ca.x_stride = c.k.x_stride; ca.value = c.k.value; ca.rlast = c.k.rlast;
    ca.mean = c.k.mean; ca.stdv = c.k.stdv;
    ca.eps = noise; ca.eps_env = c.eps_env; ca.eps_cem_off = c.eps_cem_off; ca.eps_iter = c.eps_iter;
    ca.eps_act_off = c.eps_act_off; ca.u = u; ca.prev_mean = prev_mean;
    ca.eval_mode = prm->eval_mode; ca.temperature = prm->temperature; ca.momentum = prm->momentum;
    ca.omm = prm->one_minus_momentum; ca.std_floor = prm->std_floor; ca.action = action; ca.metrics = metrics;
    ca.std_floor_p = prm->std_floor_dev;
    ca.elite_out = elite_out; ca.score_out = score_out; ca.mean_out = mean_out; ca.std_out = std_out;
    ca.value_out = value_out;
    ca.pstatus = pack_status(c); ca.status = prm->status;
    const bool wide_heads = use_wide_heads(c);
    if (wide_heads || c.fold_heads || use_chain(c, B * T, 2, CK_Q)) {   // q1, q2 per row in k.qv; cem_kernel forms the values
        ca.G = c.k.G; ca.qv = c.k.qv; ca.q_ld = c.k.xrows; ca.discH = prm->discount_pow[H];
    }
    const size_t cem_lds = cem_lds_bytes(T, H, ca.K, c.A);

    // The pi rows' terminal mean tanh(pi(z_H)) is the same in every iteration: the first iteration's pi launch over
    // all T rows caches it (chain path), later ones run pi over the N sampled rows only and redraw the pi rows'
    // TruncatedNormal sample from the cache (TDMPC_PI_CACHE=0: pi over all T rows every iteration).
    const bool pi_cache = pi_cache_on() && P > 0 && use_chain(c, B * T, 1, CK_PI);
    const RowMap pmH = {P, T, N};
    for (int i = 0; i < I; ++i) {
        const long toff = c.eps_cem_off + (long)i * c.eps_iter + c.eps_term_off;
        // wide heads: the policy rows' terminal redraw (pi_from_mu) rides in this iteration's prep launch
        const bool pm_in_prep = wide_heads && P > 0 && i > 0;
        if (i > 0) {
            const PiMuArgs pm = pimu_args(c, B * P, pmH, noise, c.eps_env, P, toff + (long)N * c.A, prm->min_std);
            if ((rc = prep(c, noise, i, nullptr, pm_in_prep ? &pm : nullptr))) return rc;
        }
        if (i > 0 || P == 0)
            for (int t = 0; t < H; ++t)
                if ((rc = step_next(c, t, B * N, rm, prm->discount_pow[t], t == 0, t == H - 1, 1)))
                    return rc;
        if (wide_heads) {
            if (P > 0) {
                if (i == 0) rc = policy(c, H, B * P, pmH, noise, c.eps_env, P, toff + (long)N * c.A, prm->min_std, c.k.pimu);
                if (rc || (rc = flush_split(c))) return rc;
            }
            if ((rc = terminal_wide(c, noise, toff, prm->min_std))) return rc;
        } else if (c.fold_heads) {
            // the sampled rows' X_H holds h2_{H-1} (folded first layers), the policy rows' holds z_H: one launch each
            if ((rc = policy(c, H, B * N, rm, noise, c.eps_env, N, toff, prm->min_std, nullptr, true))) return rc;
            if (P > 0) {
                if (i == 0 || !pi_cache)
                    rc = policy(c, H, B * P, pmH, noise, c.eps_env, P, toff + (long)N * c.A, prm->min_std,
                                pi_cache ? c.k.pimu : nullptr, c.fold_policy != 0);
                else
                    rc = policy_from_mu(c, B * P, pmH, noise, c.eps_env, P, toff + (long)N * c.A, prm->min_std);
                if (rc) return rc;
            }
            if ((rc = q_chain(c, B * N, rm, nullptr, nullptr, 0, true))) return rc;
            if (P > 0 && (rc = q_chain(c, B * P, pmH, nullptr, nullptr, 0, c.fold_policy != 0))) return rc;
        } else if (pi_cache && i > 0) {
            if ((rc = policy(c, H, B * N, rm, noise, c.eps_env, N, toff, prm->min_std))) return rc;
            if ((rc = flush_split(c))) return rc;
            if ((rc = policy_from_mu(c, B * P, pmH, noise, c.eps_env, P, toff + (long)N * c.A, prm->min_std)))
                return rc;
        } else if ((rc = policy(c, H, B * T, all, noise, c.eps_env, T, toff, prm->min_std,
                                pi_cache ? c.k.pimu : nullptr))) {
            return rc;
        }
        if (!wide_heads && !c.fold_heads && (rc = terminal_q(c, prm->discount_pow[H]))) return rc;
        ca.final_iter = i == I - 1;
        ca.iter = i;
        hipLaunchKernelGGL(cem_kernel, dim3(B), dim3(1024), cem_lds, c.s, ca);
        HIPCHK(hipGetLastError());
    }
    return 0;
}

int tdmpc_icem_sizes_for(const tdmpc_dims* d, tdmpc_sizes* out) {
    if (!d || !out) return TDMPC_E_NULL;
    if (!check_dims(d)) return TDMPC_E_DIMS;
    Layout w;
    make_layout(d, &w);
    Work k;
    make_work(d, w, nullptr, &k, d->num_elites);
    out->packed_weight_bytes = rup(w.total * 4, 256);
    out->workspace_bytes = k.total;
    out->noise_floats_per_env = 0;   // the iCEM noise layout is the caller's (tdmpc_icem_params offsets)
    return 0;
}

int tdmpc_plan_icem(const tdmpc_dims* d, const tdmpc_icem_params* prm, const void* packed, const void* obs,
                    int32_t obs_is_u8, const float* noise, const double* u, float* prev_mean, float* elites,
                    float* action, float* metrics, float* value_out, float* mean_out, float* std_out,
                    void* workspace, size_t ws_bytes, void* stream) {
    if (!d || !prm || !packed || !obs || !noise || !u || !prev_mean || !elites || !action || !metrics || !workspace)
        return TDMPC_E_NULL;
    Ctx c;
    int rc;
    const int H = prm->horizon, I = prm->iterations, B = prm->batch, K = d->num_elites;
    if (I <= 0 || I > 16) { snprintf(g_err, sizeof g_err, "iCEM: 1..16 iterations"); return TDMPC_E_DIMS; }
    if ((rc = setup_ctx(c, d, packed, workspace, ws_bytes, B, H, I, (hipStream_t)stream, K))) return rc;
    if (prm->path < 0 || prm->path > TDMPC_PATH_WIDE) { snprintf(g_err, sizeof g_err, "bad path"); return TDMPC_E_DIMS; }
    c.path = prm->path == TDMPC_PATH_PERSIST ? TDMPC_PATH_AUTO : prm->path == TDMPC_PATH_CHAIN64 ? TDMPC_PATH_CHAIN_X6
           : prm->path;   // (persist: whole plans only; the retired 64-row path is path 6)
    const int N = d->num_samples, Pmax = d->num_pi, Tw = N + K + Pmax, pi_base = N + K, P0 = prm->n_pi0;
    c.T = Tw;
    if (P0 <= 0 || P0 > Pmax || prm->n_samples[0] != N) { snprintf(g_err, sizeof g_err, "iCEM: bad counts"); return TDMPC_E_DIMS; }
    for (int i = 0; i < I; ++i) {
        const int Ni = prm->n_samples[i], Pi = prm->n_pi[i], Ei = prm->n_elite[i];
        if (Ni <= 0 || Ni > N || Pi <= 0 || Pi > P0 || Ei < 0 || Ei > K || Ni + Ei + Pi < K ||
            (Ei > 0 && i == 0 && !prm->has_elites) || (i == 0 && Ei > 0 && prm->elite_horizon != H && prm->elite_horizon != H - 1)) {
            snprintf(g_err, sizeof g_err, "iCEM: bad counts at iteration %d", i);
            return TDMPC_E_DIMS;
        }
    }
    const long A = c.A, env = prm->env_stride;
    // z0 = h(obs); mean = 0 (warm: mean[:-1] = prev[1:], mean[-1] = prev[-1]), std = init_std (0.5)
    if ((rc = encode(c, obs, obs_is_u8, B, prev_mean, prm->warm_start, 1, prm->init_std))) return rc;
    // pi pre-rollout of the P0 policy rows (tdmpc_icem_similarity_mlp.py:193-199); their rollout, reward
    // prefix and z_H are the same in every iteration (same z, same pi actions), so they are computed once
    const RowMap pm0 = {P0, Tw, pi_base};
    {
        PrepArgs pa;
        memset(&pa, 0, sizeof pa);
        pa.X = c.k.X; pa.x_stride = c.k.x_stride; pa.Kx = c.Kx; pa.apq = c.w.Ap / 4; pa.lpq = c.w.Lp / 4;
        pa.B = B; pa.N = N; pa.T = Tw; pa.H = H; pa.A = c.A; pa.z0 = c.k.z0; pa.n_zq = (long)B * pa.lpq * Tw;
        hipLaunchKernelGGL(prep_kernel, dim3((int)std::min<long>((pa.n_zq + 255) / 256, 2048)), dim3(256), 0, c.s, pa);
        HIPCHK(hipGetLastError());
    }
    for (int t = 0; t < H; ++t) {
        if ((rc = policy(c, t, B * P0, pm0, noise, env, P0, prm->pi_off + (long)t * P0 * A, prm->min_std))) return rc;
        if ((rc = step_next(c, t, B * P0, pm0, prm->discount_pow[t], t == 0, t == H - 1))) return rc;
    }
    CemArgs ca;
    memset(&ca, 0, sizeof ca);
    ca.H = H; ca.A = c.A; ca.K = K; ca.Kx = c.Kx; ca.Hmax = d->max_horizon; ca.I = I;
    ca.X = c.k.X; ca.x_stride = c.k.x_stride; ca.value = c.k.value; ca.rlast = c.k.rlast;
    ca.mean = c.k.mean; ca.stdv = c.k.stdv; ca.Tw = Tw; ca.pi_base = pi_base;
    ca.eps = noise; ca.eps_env = env; ca.eps_act_off = prm->act_off; ca.u = u; ca.prev_mean = prev_mean;
    ca.eval_mode = prm->eval_mode; ca.temperature = prm->temperature; ca.momentum = prm->momentum;
    ca.omm = prm->one_minus_momentum; ca.std_floor = prm->std_floor; ca.action = action; ca.metrics = metrics;
    ca.mean_out = mean_out; ca.std_out = std_out; ca.elite_store = elites;
    ca.G = c.k.G; ca.q_ld = c.k.xrows; ca.discH = prm->discount_pow[H]; ca.value_out = value_out;
    ca.pstatus = pack_status(c); ca.status = prm->status;
    const size_t cem_lds = cem_lds_bytes(Tw, H, K, c.A);
    for (int i = 0; i < I; ++i) {
        const int Ni = prm->n_samples[i], Pi = prm->n_pi[i], Ei = prm->n_elite[i], NE = Ni + Ei;
        {   // sampled candidates clamp(mean + std * noise) for rows [0, Ni) (sample_mix_action_sequence)
            PrepArgs pa;
            memset(&pa, 0, sizeof pa);
            pa.X = c.k.X; pa.x_stride = c.k.x_stride; pa.Kx = c.Kx; pa.apq = c.w.Ap / 4; pa.lpq = c.w.Lp / 4;
            pa.B = B; pa.N = Ni; pa.T = Tw; pa.H = H; pa.A = c.A;
            pa.mean = c.k.mean; pa.stdv = c.k.stdv; pa.mstride = d->max_horizon * c.A;
            pa.eps = noise; pa.eps_env = env; pa.eps_off = prm->samp_off[i];
            pa.n_sq = (long)B * H * pa.apq * Ni;
            hipLaunchKernelGGL(prep_kernel, dim3((int)std::min<long>((pa.n_sq + 255) / 256, 2048)), dim3(256), 0, c.s, pa);
            HIPCHK(hipGetLastError());
        }
        if (Ei > 0 || i == I - 1) {
            FillArgs fa;
            memset(&fa, 0, sizeof fa);
            fa.X = c.k.X; fa.x_stride = c.k.x_stride; fa.Kx = c.Kx; fa.apq = c.w.Ap / 4; fa.Tw = Tw;
            fa.B = B; fa.H = H; fa.A = c.A; fa.Hmax = d->max_horizon; fa.K = K;
            fa.n0 = Ni; fa.E = Ei; fa.mode = i == 0 ? 1 : 2; fa.eH = prm->elite_horizon; fa.mean_row = i == I - 1;
            fa.mean = c.k.mean; fa.stdv = c.k.stdv; fa.elites = elites;
            fa.eps = noise; fa.eps_env = env; fa.reuse_off = prm->reuse_off;
            const long tot = (long)B * H * fa.apq * (Ei + fa.mean_row);
            hipLaunchKernelGGL(icem_fill_kernel, dim3((int)std::min<long>((tot + 255) / 256, 2048)), dim3(256), 0, c.s, fa);
            HIPCHK(hipGetLastError());
        }
        // rollout of the sampled + reused rows (the pi rows' is cached from the pre-rollout)
        const RowMap blk = {NE, Tw, 0};
        for (int t = 0; t < H; ++t)
            if ((rc = step_next(c, t, B * NE, blk, prm->discount_pow[t], t == 0, t == H - 1, 1))) return rc;
        // terminal value of all T_i = NE + Pi candidates: pi(z_H) with this iteration's noise, Q
        const RowMap pmi = {Pi, Tw, pi_base};
        if ((rc = policy(c, H, B * NE, blk, noise, env, NE, prm->term_off[i], prm->min_std))) return rc;
        if ((rc = policy(c, H, B * Pi, pmi, noise, env, Pi, prm->term_off[i] + (long)NE * A, prm->min_std))) return rc;
        // both row groups on the same Q path, so cem_kernel reads one kind of value (qv or value)
        const bool qchain = use_chain(c, B * NE, 2, CK_Q) && use_chain(c, B * Pi, 2, CK_Q);
        if ((rc = terminal_q_rows(c, B * NE, blk, prm->discount_pow[H], qchain))) return rc;
        if ((rc = terminal_q_rows(c, B * Pi, pmi, prm->discount_pow[H], qchain))) return rc;
        ca.qv = qchain ? c.k.qv : nullptr;
        ca.N = Ni; ca.P = Pi; ca.T = NE + Pi; ca.NE = NE;
        ca.final_iter = i == I - 1;
        ca.iter = i;
        hipLaunchKernelGGL(cem_kernel, dim3(B), dim3(1024), cem_lds, c.s, ca);
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
    if (prm->path < 0 || prm->path > TDMPC_PATH_WIDE) { snprintf(g_err, sizeof g_err, "bad path"); return TDMPC_E_DIMS; }
    c.path = prm->path == TDMPC_PATH_PERSIST ? TDMPC_PATH_AUTO : prm->path == TDMPC_PATH_CHAIN64 ? TDMPC_PATH_CHAIN_X6
           : prm->path;   // (persist: whole plans only; the retired 64-row path is path 6)
    if (rows != c.T) { snprintf(g_err, sizeof g_err, "rows must equal N+P"); return TDMPC_E_DIMS; }
    const int T = c.T, L = c.w.L;
    hipLaunchKernelGGL(zero_words_kernel, dim3(1), dim3(256), 0, c.s, (unsigned*)c.k.z0, (int)((size_t)B * c.w.Lp));
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpy2DAsync(c.k.z0, c.w.Lp * 4, z0, L * 4, L * 4, B, hipMemcpyDeviceToDevice, c.s));
    hipLaunchKernelGGL(scatter_actions_kernel, dim3(512), dim3(256), 0, c.s, actions, c.k.X, c.k.x_stride, H, T, c.A,
                       c.w.Ap, c.Kx, B, T, 0);
    HIPCHK(hipGetLastError());
    if ((rc = prep(c, nullptr, 0, c.k.z0))) return rc;
    const RowMap all = {T, T, 0};
    for (int t = 0; t < H; ++t)
        if ((rc = step_next(c, t, B * T, all, prm->discount_pow[t], t == 0, t == H - 1)))
            return rc;
    if (z_last) {
        hipLaunchKernelGGL(gather_z_kernel, dim3(256), dim3(256), 0, c.s, Xt(c, H), c.Kx, c.w.Ap, L, B * T, z_last);
        HIPCHK(hipGetLastError());
    }
    if ((rc = policy(c, H, B * T, all, eps_term, (long)T * c.A, T, 0, prm->min_std))) return rc;
    if ((rc = terminal_q(c, prm->discount_pow[H]))) return rc;
    if (use_chain(c, B * T, 2, CK_Q)) {
        hipLaunchKernelGGL(qvalue_kernel, dim3((B * T + 255) / 256), dim3(256), 0, c.s, c.k.G, c.k.qv, c.k.xrows,
                           prm->discount_pow[H], c.k.value, B * T);
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipMemcpyAsync(value, c.k.value, (size_t)B * T * 4, hipMemcpyDeviceToDevice, c.s));
    HIPCHK(hipMemcpyAsync(reward_last, c.k.rlast, (size_t)B * T * 4, hipMemcpyDeviceToDevice, c.s));
    return 0;
}

// z0 [B][L] -> the workspace's padded z0 [B][Lp] and the latent columns of X_0 for all T rows of every env
static int load_z0(const Ctx& c, const float* z0) {
    const int L = c.w.L;
    hipLaunchKernelGGL(zero_words_kernel, dim3(1), dim3(256), 0, c.s, (unsigned*)c.k.z0, (int)((size_t)c.B * c.w.Lp));
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpy2DAsync(c.k.z0, c.w.Lp * 4, z0, L * 4, L * 4, c.B, hipMemcpyDeviceToDevice, c.s));
    return prep(c, nullptr, 0, c.k.z0);
}

int tdmpc_pi_rollout(const tdmpc_dims* d, const tdmpc_plan_params* prm, const void* packed, const float* z0,
                     const float* eps_pi, float* pi_actions, void* workspace, size_t ws_bytes, void* stream) {
    if (!d || !prm || !packed || !z0 || !eps_pi || !pi_actions || !workspace) return TDMPC_E_NULL;
    Ctx c;
    int rc;
    const int H = prm->horizon, B = prm->batch;
    if ((rc = setup_ctx(c, d, packed, workspace, ws_bytes, B, H, 1, (hipStream_t)stream))) return rc;
    if (prm->path < 0 || prm->path > TDMPC_PATH_WIDE) { snprintf(g_err, sizeof g_err, "bad path"); return TDMPC_E_DIMS; }
    c.path = prm->path == TDMPC_PATH_PERSIST ? TDMPC_PATH_AUTO : prm->path == TDMPC_PATH_CHAIN64 ? TDMPC_PATH_CHAIN_X6
           : prm->path;   // (persist: whole plans only; the retired 64-row path is path 6)
    const int N = c.N, P = c.P, T = c.T;
    const long A = c.A;
    if (P <= 0) { snprintf(g_err, sizeof g_err, "num_pi is 0"); return TDMPC_E_DIMS; }
    if ((rc = load_z0(c, z0))) return rc;
    // the policy rows sit where tdmpc_plan keeps them: rows N..T-1 of each env's block of T
    const RowMap pm = {P, T, N};
    for (int t = 0; t < H; ++t) {
        if ((rc = policy(c, t, B * P, pm, eps_pi, (long)H * P * A, P, (long)t * P * A, prm->min_std))) return rc;
        if (t < H - 1 && (rc = step_next(c, t, B * P, pm, prm->discount_pow[t], t == 0, 0))) return rc;
    }
    hipLaunchKernelGGL(gather_actions_kernel, dim3(512), dim3(256), 0, c.s, c.k.X, c.k.x_stride, H, P, c.A, c.Kx, B,
                       T, N, pi_actions);
    HIPCHK(hipGetLastError());
    return 0;
}

int tdmpc_cem_iter(const tdmpc_dims* d, const tdmpc_plan_params* prm, const void* packed, const float* z0,
                   const float* pi_actions, const float* eps_cem, const float* eps_term, float* mean, float* stdv,
                   float* elite_actions, float* score, float* value, float* reward_mean, void* workspace,
                   size_t ws_bytes, void* stream) {
    if (!d || !prm || !packed || !z0 || !eps_cem || !eps_term || !mean || !stdv || !elite_actions || !score ||
        !reward_mean || !workspace)
        return TDMPC_E_NULL;
    Ctx c;
    int rc;
    const int H = prm->horizon, B = prm->batch;
    if ((rc = setup_ctx(c, d, packed, workspace, ws_bytes, B, H, 1, (hipStream_t)stream))) return rc;
    if (prm->path < 0 || prm->path > TDMPC_PATH_WIDE) { snprintf(g_err, sizeof g_err, "bad path"); return TDMPC_E_DIMS; }
    c.path = prm->path == TDMPC_PATH_PERSIST ? TDMPC_PATH_AUTO : prm->path == TDMPC_PATH_CHAIN64 ? TDMPC_PATH_CHAIN_X6
           : prm->path;   // (persist: whole plans only; the retired 64-row path is path 6)
    const int N = c.N, P = c.P, T = c.T, A = c.A, HA = H * A;
    if (P > 0 && !pi_actions) return TDMPC_E_NULL;
    // the caller's mean/std [B][H][A] -> the workspace's [B][Hmax][A]
    const size_t mp = (size_t)d->max_horizon * A * 4;
    HIPCHK(hipMemcpy2DAsync(c.k.mean, mp, mean, HA * 4, HA * 4, B, hipMemcpyDeviceToDevice, c.s));
    HIPCHK(hipMemcpy2DAsync(c.k.stdv, mp, stdv, HA * 4, HA * 4, B, hipMemcpyDeviceToDevice, c.s));
    if ((rc = load_z0(c, z0))) return rc;
    // candidates clamp(mean + std * eps_cem) in rows 0..N-1 (the eps stream of one env is [H][N][A])
    c.eps_env = (long)H * N * A; c.eps_cem_off = 0; c.eps_iter = 0;
    if ((rc = prep(c, eps_cem, 0, nullptr))) return rc;
    if (P > 0) {
        hipLaunchKernelGGL(scatter_actions_kernel, dim3(512), dim3(256), 0, c.s, pi_actions, c.k.X, c.k.x_stride, H, P,
                           A, c.w.Ap, c.Kx, B, T, N);
        HIPCHK(hipGetLastError());
    }
    const RowMap all = {T, T, 0};
    for (int t = 0; t < H; ++t)
        if ((rc = step_next(c, t, B * T, all, prm->discount_pow[t], t == 0, t == H - 1, 1))) return rc;
    if ((rc = policy(c, H, B * T, all, eps_term, (long)T * A, T, 0, prm->min_std))) return rc;
    if ((rc = terminal_q(c, prm->discount_pow[H]))) return rc;
    CemArgs ca;
    memset(&ca, 0, sizeof ca);
    ca.H = H; ca.N = N; ca.P = P; ca.T = T; ca.A = A; ca.K = d->num_elites; ca.Kx = c.Kx;
    ca.Hmax = d->max_horizon; ca.I = 1; ca.iter = 0; ca.final_iter = 1; ca.no_pick = 1;
    ca.Tw = T; ca.NE = T; ca.pi_base = 0;
    ca.X = c.k.X; ca.x_stride = c.k.x_stride; ca.value = c.k.value; ca.rlast = c.k.rlast;
    ca.mean = c.k.mean; ca.stdv = c.k.stdv;
    ca.temperature = prm->temperature; ca.momentum = prm->momentum; ca.omm = prm->one_minus_momentum;
    ca.std_floor = prm->std_floor; ca.std_floor_p = prm->std_floor_dev;
    ca.elite_out = elite_actions; ca.score_out = score; ca.value_out = value; ca.reward_out = reward_mean;
    ca.pstatus = pack_status(c); ca.status = prm->status;
    if (use_chain(c, B * T, 2, CK_Q)) { ca.G = c.k.G; ca.qv = c.k.qv; ca.q_ld = c.k.xrows; ca.discH = prm->discount_pow[H]; }
    hipLaunchKernelGGL(cem_kernel, dim3(B), dim3(1024), cem_lds_bytes(T, H, ca.K, A), c.s, ca);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpy2DAsync(mean, HA * 4, c.k.mean, mp, HA * 4, B, hipMemcpyDeviceToDevice, c.s));
    HIPCHK(hipMemcpy2DAsync(stdv, HA * 4, c.k.stdv, mp, HA * 4, B, hipMemcpyDeviceToDevice, c.s));
    return 0;
}

int tdmpc_profile_begin(int32_t cfg, int32_t pro, int32_t kdim, int32_t rows, int32_t max_launches) {
    Profiler& pf = g_prof;
    if (pf.ev) {
        for (int i = 0; i < pf.cap; ++i) (void)hipEventDestroy(pf.ev[i]);
        free(pf.ev);
    }
    pf = Profiler();
    pf.cap = 2 * std::max(1, (int)max_launches);
    pf.ev = (hipEvent_t*)calloc(pf.cap, sizeof(hipEvent_t));
    for (int i = 0; i < pf.cap; ++i) HIPCHK(hipEventCreate(&pf.ev[i]));
    pf.cfg = cfg; pf.pro = pro; pf.kdim = kdim; pf.rows = rows; pf.armed = 1;
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

const char* tdmpc_profile_kernel(void) { return g_prof.kernel; }

}  // extern "C"
