/*
 * tdmpc_learner.h -- C ABI of the learner's fused loss in libtdmpc_hip.so.
 *
 * Replaces the loss composition of TDMPC.update (/root/reference/src/algorithm/tdmpc.py:209-224: the rho-weighted
 * consistency / reward / value / priority losses over the horizon, the 1e4 clamps, the coefficient sum, the
 * IS-weighted mean) and its backward: ~60 one-op ATen launches per update become three HIP launches. Inputs are
 * the horizon-batched tensors of tdmpc_amd.learner (row-major, contiguous, float32, device pointers):
 *   zp [H][B][L] predicted latents z_{t+1}, nz [H][B][L] target-encoder latents, q1 q2 rp [H][B] Q heads and
 *   reward head, rw [H][B] rewards, td [H][B] TD targets, w [B] importance weights, rho [H] = float32(rho**t).
 * Stream-ordered, no allocation, graph-capturable; 0 or a negative TDMPC_E* code.
 */
#ifndef TDMPC_LEARNER_H
#define TDMPC_LEARNER_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct tdmpc_loss_args {
    const float* zp; const float* nz; const float* q1; const float* q2; const float* rp; const float* rw;
    const float* td; const float* w; const float* rho;
    int32_t H, B, L;
    float consistency_coef, reward_coef, value_coef;
} tdmpc_loss_args;

/* Forward. rows [5][B]: consistency, reward, value losses, priority loss clamped at 1e4, total loss per row;
 * scal [6]: mean consistency, mean reward, mean value, mean total, weighted = mean(total) * mean(w) (the
 * reference's mean over its [B, B] broadcast of total [B, 1] * w [B]), mean(w). */
int tdmpc_loss_forward(const tdmpc_loss_args* a, float* rows, float* scal, void* stream);

/* Backward of `weighted`: gw (device scalar) = dL/dweighted (the 1/H hook already applied). Writes dzp [H][B][L],
 * dq1, dq2, drp [H][B] (any may be null: not computed). rows / scal: the forward's outputs. */
int tdmpc_loss_backward(const tdmpc_loss_args* a, const float* rows, const float* scal, const float* gw,
                        float* dzp, float* dq1, float* dq2, float* drp, void* stream);

/* RandomShiftsAug (helper.py:250-283, the pixel learner's augmentation): out[k] = x[k] shifted by (shift[k][0],
 * shift[k][1]) - pad pixels with replicate padding, i.e. the reference's pad + grid_sample at its (integer) sample
 * points. x, out: float [n][c][h][w] (a 5-D [t][b] batch flattened to n = t * b, as the reference reshapes it);
 * shift: float [n][2] integers in [0, 2 pad] (the reference's torch.randint draw, x then y). */
int tdmpc_random_shift(const float* x, const float* shift, int32_t n, int32_t c, int32_t h, int32_t w, int32_t pad,
                       float* out, void* stream);
/* The same with the output divided by div (> 0; 0 = no division), rounded as helper.enc's NormalizeImg x / 255: the
 * learner engine augments straight into normalised frames for its conv stack (tdmpc_lg_conv_* with in_div = 0). */
int tdmpc_random_shift_scaled(const float* x, const float* shift, int32_t n, int32_t c, int32_t h, int32_t w,
                              int32_t pad, float div, float* out, void* stream);

/* ---------------------------------------------------------------------------------------------------------------
 * The learner engine: TDMPC.update / update_pi / _td_target (tdmpc.py:165-245) as explicit forward and backward
 * passes over the TOLD heads (tdmpc_amd/learner_engine.py drives them). Every pointer is a device
 * pointer to float32; strides in elements. Stream-ordered, no allocation, graph-capturable; 0 or TDMPC_E*.
 * ------------------------------------------------------------------------------------------------------------- */

/* One K segment of a GEMM: C[m][n] (+)= sum_k A(m, k) B(k, n), k < k_len.
 *   amode 0: A(m, k) = a[m * lda + k]   (activations, row-major)   amode 1: A(m, k) = a[k * lda + m]  (dY^T)
 *   bmode 0: B(k, n) = b[n * ldb + k]   (Linear weight [N][K])     bmode 1: B(k, n) = b[k * ldb + n]
 *   ones_col >= 0: B(k, ones_col) = 1 (the bias column of a weight gradient: db = colsum(dY)). */
typedef struct tdmpc_lg_seg {
    const float* a; const float* b;
    int32_t lda, ldb, k, amode, bmode, ones_col;
} tdmpc_lg_seg;

enum { TDMPC_LG_EPI_NONE = 0, TDMPC_LG_EPI_ELU = 1, TDMPC_LG_EPI_PI = 2, TDMPC_LG_EPI_ELU_BWD = 3,
       TDMPC_LG_EPI_PI_BWD = 4, TDMPC_LG_EPI_RELU_BWD = 5 };

/* One GEMM of a grouped launch: C = epi(sum over segments + bias[n] + res[m][n]).
 *   EPI_ELU:     elu(x)                                   (nn.ELU)
 *   EPI_PI:      mu = tanh(x); c = clamp(mu + clamp(std * aux, -0.3, 0.3), -1 + 1e-6, 1 - 1e-6); c2 = mu
 *                (TOLD.pi + TruncatedNormal.sample, helper.py:71-96; aux = the standard normal draws)
 *   EPI_ELU_BWD: x * (aux > 0 ? 1 : aux + 1)              (aux = the ELU's output)
 *   EPI_PI_BWD:  x * (1 - aux^2)                          (aux = mu: tanh' with the straight-through clamp)
 *   EPI_RELU_BWD: aux > 0 ? x : 0                         (aux = the ReLU's output)
 *   c2 (EPI_NONE): a second copy of C (ldc2).
 * splits > 1: split-K over workgroups; slice s of the raw sum goes to c + s * slice (no bias / res / epi). */
typedef struct tdmpc_lg_job {
    tdmpc_lg_seg seg[3];
    int32_t nseg, m, n, epi;
    float* c; float* c2; const float* bias; const float* aux; const float* res;
    int32_t ldc, ldc2, ldaux, ldres;
    float std_; int32_t splits; int64_t slice;
} tdmpc_lg_job;

/* Up to 12 GEMMs in one launch; tile 1: 32x32 output tiles, 2: 64x64 (4 waves split K inside a workgroup).
 * Products are fp32-accurate x6 (three bf16 parts per operand, six bf16 MFMAs per pair, fp32 accumulation);
 * tile | TDMPC_LG_TILE_EXACT runs the exact v_mfma_f32_32x32x2_f32 products instead.
 * tile 3 / 4: LDS-staged macro tiles of 64x64 / 64x128 outputs (m x n) per workgroup on the exact f32 MFMA (the
 * EXACT bit is implied), for the large products: every segment amode 0 without a ones column, splits 1, one bmode
 * per launch. */
#define TDMPC_LG_TILE_EXACT 0x100
int tdmpc_lg_gemm(const tdmpc_lg_job* jobs, int32_t njobs, int32_t tile, void* stream);

/* Row kernels over [rows][m] activations (one wave per row; m in {256, 512, 1024}), up to 3 heads. Every row operand
 * (x, y, xhat, yact, g, beta, w3) 16-B aligned and ldx / ldy multiples of 4 (16-B row accesses), else TDMPC_E_DIMS.
 * Forward, per head: v = x (ln: v = layer_norm(x) * g + beta, saving xhat [rows][m] and rstd [rows]); y = act(v)
 * (act 1 tanh, 2 elu) -> y (ldy); tail: out[r] = y . w3 + b3[0]. td != null: td[r] = reward[r] + gamma *
 * min(out_0[r], out_1[r]) (TDMPC._td_target, tdmpc.py:184-190).
 * Backward, per head: d = tail ? dq[r] * w3 : x (dA, ldx); d *= act'(yact); ln: d = layer_norm backward (xhat, rstd,
 * g) -> y (dP, ldy). part != null: per-workgroup column sums [nwg][..] of (ln: d*xhat, d) then (tail: dq*yact, dq),
 * i.e. the partial gradients of the LayerNorm affine and of the scalar output layer. pi mode (q1 != null): dq of
 * head h is d(-sum_t rho^t mean_b min(q1, q2)) / dq_h (ties split in half, as torch.min's backward). */
typedef struct tdmpc_lg_rowhead {
    const float* x; float* y; float* xhat; float* rstd; const float* yact;
    const float* g; const float* beta; const float* w3; const float* b3; float* out; const float* dq; float* part;
    int32_t ldx, ldy, ln, act, tail;
} tdmpc_lg_rowhead;

typedef struct tdmpc_lg_rows {
    tdmpc_lg_rowhead hd[3];
    int32_t nh, rows, m, bsz;
    const float* reward; float* td; float gamma;
    const float* q1; const float* q2; const float* rho;
} tdmpc_lg_rows;

int tdmpc_lg_rows_fwd(const tdmpc_lg_rows* a, void* stream);
int tdmpc_lg_rows_bwd(const tdmpc_lg_rows* a, int32_t nwg, void* stream);

/* pi_loss = sum_t rho^t * -(mean_b min(q1, q2)) over rows t * bsz + b, t < nt (TDMPC.update_pi) -> out[0]. */
int tdmpc_lg_pi_loss(const float* q1, const float* q2, const float* rho, int32_t nt, int32_t bsz, float* out,
                     void* stream);

/* Gradient finalisation: parameter tensor i occupies g[dst, dst + rows * cols) (in increasing dst order, no
 * overlap; gaps between tensors are left alone); its gradient is the sum of
 * nslices slices src + s * sstride, element (r, c) at src[r * ld + c]. Writes g, per-workgroup sums of squares to
 * normp (one workgroup per 2048 elements of a tensor; nblk = the capacity of normp, whose unused tail must hold
 * zeros) and step[0] += 1 (the optimiser's step count). */
typedef struct tdmpc_lg_gsrc {
    const float* src; int64_t dst; int64_t sstride;
    int32_t rows, cols, ld, nslices;
} tdmpc_lg_gsrc;

int tdmpc_lg_finalize(const tdmpc_lg_gsrc* t, int32_t nt, float* g, float* normp, int32_t nblk, int32_t* step,
                      void* stream);

/* clip_grad_norm_ (total norm = sqrt of the sum of normp [nblk]) + Adam (torch.optim.Adam, no weight decay) over n contiguous parameters;
 * norm_out[0] = the total norm (clip_grad_norm_'s return value). g is left clipped, as clip_grad_norm_ leaves .grad. */
int tdmpc_lg_adam(float* p, float* g, float* m, float* v, int64_t n, const float* normp, int32_t nblk,
                  const int32_t* step, float lr, float beta1, float beta2, float eps, float max_norm,
                  float* norm_out, void* stream);

/* t <- lerp(t, p, w) elementwise (helper.ema, helper.py:48-52). */
int tdmpc_lg_lerp(float* t, const float* p, int64_t n, float w, void* stream);

/* The pixel encoder's convolutions (helper.enc, helper.py:119-133: Conv2d(cin -> 32, k, stride 2, no padding) + ReLU,
 * NCHW fp32) for the learner, on the exact f32 MFMA (v_mfma_f32_32x32x2_f32), every sum in a fixed order.
 * Forward: y_p = relu(conv(x / in_div (in_div > 0; NormalizeImg's x / 255), w_p) + b_p) for nprob <= 2 weight sets
 * sharing the input (the online and target encoders on the same augmented frames). */
typedef struct tdmpc_lg_conv {
    const float* x;                  /* [n][cin][hin][hin] */
    const float* w[2];               /* [32][cin][k][k] */
    const float* b[2];               /* [32] */
    float* y[2];                     /* [n][32][ho][ho], ho = (hin - k) / 2 + 1 */
    int32_t nprob, n, cin, hin, k;
    float in_div;
} tdmpc_lg_conv;
int tdmpc_lg_conv_fwd(const tdmpc_lg_conv* a, void* stream);

/* Data gradient of a stride-2 conv masked by the ReLU that produced its input:
 * dx[n][ci][y][x] = (sum_{co,ky,kx: y = 2oy + ky, x = 2ox + kx} w[co][ci][ky][kx] dy[n][co][oy][ox]) * (xact > 0). */
int tdmpc_lg_conv_bwd_data(const float* dy, const float* w, const float* xact, float* dx, int32_t n, int32_t cin,
                           int32_t hin, int32_t k, void* stream);

/* Weight-gradient slices: part[s][co][c] = sum over the images of slice s (img_per_slice each, the last one short)
 * and their output pixels p of dy[n][co][p] * patch(x / in_div, p)[c], c < cin k k (c = ci k k + ky k + kx); column
 * c = cin k k is the bias gradient (sum of dy). part: [ceil(n / img_per_slice)][32][cin k k + 1], summed by
 * tdmpc_lg_finalize. */
int tdmpc_lg_conv_bwd_weight(const float* dy, const float* x, float in_div, float* part, int32_t n, int32_t cin,
                             int32_t hin, int32_t k, int32_t img_per_slice, void* stream);

/* In place over n elements: mode 0 x <- ELU(x) (nn.ELU, helper.py:172); mode 1 x <- x * ELU'(y) with y the saved
 * ELU output (y > 0 ? 1 : y + 1) -- the activation epilogues of a library GEMM's output. */
int tdmpc_lg_act(float* x, const float* y, int64_t n, int32_t mode, void* stream);

#ifdef __cplusplus
}
#endif
#endif
