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

#ifdef __cplusplus
}
#endif
#endif
