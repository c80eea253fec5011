// learner_kernels.hip -- the learner's fused loss (include/tdmpc_learner.h) for MI355X (gfx950).
//
// Reference: TDMPC.update's loss composition, /root/reference/src/algorithm/tdmpc.py:209-224 (helper.py:19-26
// mse / l1). One wave per batch row sums its H x L consistency terms and H reward / value / priority terms
// (fp32, lane-strided then a wave tree); one workgroup forms the batch means and the IS-weighted mean; the
// backward writes every input gradient in one elementwise pass. Against the reference's op-by-op ATen chain the
// sums run in another order (rounding only; tests/test_learner.py holds the whole update to the oracle).
#include <hip/hip_runtime.h>

#include <stdio.h>

#include <algorithm>

#include "../../include/tdmpc_hip.h"
#include "../../include/tdmpc_learner.h"

namespace tdmpc_internal {
void set_error(const char* msg);
}

namespace {

constexpr float CLAMP = 1e4f;

__device__ __forceinline__ float wsum(float v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// rows: [5][B] consistency, reward, value, priority (clamped), total
__global__ void __launch_bounds__(256) loss_rows_kernel(const tdmpc_loss_args a, float* rows) {
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= a.B) return;
    const int H = a.H, B = a.B, L = a.L;
    float cons = 0.f, rew = 0.f, val = 0.f, pri = 0.f;
    for (int t = 0; t < H; ++t) {
        const float rho = a.rho[t];
        const float* zp = a.zp + ((size_t)t * B + b) * L;
        const float* nz = a.nz + ((size_t)t * B + b) * L;
        float s = 0.f;
        for (int l = lane; l < L; l += 64) {
            const float d = zp[l] - nz[l];
            s += d * d;
        }
        s = wsum(s);
        cons += rho * (s / (float)L);
        const size_t i = (size_t)t * B + b;
        const float dr = a.rp[i] - a.rw[i], d1 = a.q1[i] - a.td[i], d2 = a.q2[i] - a.td[i];
        rew += rho * (dr * dr);
        val += rho * (d1 * d1 + d2 * d2);
        pri += rho * (fabsf(d1) + fabsf(d2));
    }
    if (lane == 0) {
        rows[b] = cons;
        rows[B + b] = rew;
        rows[2 * B + b] = val;
        rows[3 * B + b] = fminf(pri, CLAMP);
        rows[4 * B + b] = a.consistency_coef * fminf(cons, CLAMP) + a.reward_coef * fminf(rew, CLAMP) +
                          a.value_coef * fminf(val, CLAMP);
    }
}

// scal: mean consistency, reward, value, total; weighted; mean(w)
__global__ void __launch_bounds__(512) loss_means_kernel(const tdmpc_loss_args a, const float* rows, float* scal) {
    __shared__ float red[5][8];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int B = a.B;
    float s[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
    for (int b = tid; b < B; b += 512) {
        s[0] += rows[b];
        s[1] += rows[B + b];
        s[2] += rows[2 * B + b];
        s[3] += rows[4 * B + b];
        s[4] += a.w[b];
    }
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        const float v = wsum(s[k]);
        if (lane == 0) red[k][wave] = v;
    }
    __syncthreads();
    if (tid == 0) {
        float m[5];
        for (int k = 0; k < 5; ++k) {
            float v = 0.f;
            for (int w = 0; w < 8; ++w) v += red[k][w];
            m[k] = v / (float)B;
        }
        scal[0] = m[0]; scal[1] = m[1]; scal[2] = m[2]; scal[3] = m[3];
        scal[4] = m[3] * m[4];
        scal[5] = m[4];
    }
}

// d weighted / d total_b = mean(w) / B; the clamps pass gradient where the loss is <= 1e4 (torch.clamp)
__global__ void __launch_bounds__(256) loss_backward_kernel(const tdmpc_loss_args a, const float* rows,
                                                            const float* scal, const float* gw, float* dzp,
                                                            float* dq1, float* dq2, float* drp) {
    const int H = a.H, B = a.B, L = a.L;
    const long nz_el = (long)H * B * L;
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const float dtot = gw[0] * scal[5] / (float)B;
    if (i < nz_el) {
        const int b = (int)((i / L) % B), t = (int)(i / ((long)L * B));
        if (dzp) {
            const float dc = rows[b] <= CLAMP ? a.consistency_coef * dtot : 0.f;
            dzp[i] = a.rho[t] * (2.f * (a.zp[i] - a.nz[i]) / (float)L) * dc;
        }
    }
    if (i < (long)H * B) {
        const int b = (int)(i % B), t = (int)(i / B);
        const float rho = a.rho[t];
        const float dr = rows[B + b] <= CLAMP ? a.reward_coef * dtot : 0.f;
        const float dv = rows[2 * B + b] <= CLAMP ? a.value_coef * dtot : 0.f;
        if (drp) drp[i] = rho * (2.f * (a.rp[i] - a.rw[i])) * dr;
        if (dq1) dq1[i] = rho * (2.f * (a.q1[i] - a.td[i])) * dv;
        if (dq2) dq2[i] = rho * (2.f * (a.q2[i] - a.td[i])) * dv;
    }
}

int hip_fail(hipError_t e) {
    char m[256];
    snprintf(m, sizeof m, "learner_kernels: %s", hipGetErrorString(e));
    tdmpc_internal::set_error(m);
    return TDMPC_E_HIP;
}

bool args_ok(const tdmpc_loss_args* a) {
    return a && a->zp && a->nz && a->q1 && a->q2 && a->rp && a->rw && a->td && a->w && a->rho && a->H > 0 &&
           a->B > 0 && a->L > 0;
}

// RandomShiftsAug (helper.py:250-283) as the gather it is: the reference pads by `pad` with replicate padding and
// grid-samples (bilinear, zeros, align_corners=False) at base_grid + shift, whose points are exactly the integer
// pixel centres (linspace(-1 + 1/n, 1 - 1/n, n)[:h] unnormalises to 0..h-1, shift s * 2/n to s pixels). So output
// (i, j) of stacked image k is the padded image at (i + sy_k, j + sx_k) = the input at
// (clamp(i + sy_k - pad), clamp(j + sx_k - pad)). One thread per output pixel, a row per 64 consecutive lanes
// (coalesced, HBM-bound: 4 B read + 4 B written per pixel). shift: the reference's own draw, float [n][2] (x, y).
// div > 0: the output is x / div, rounded as helper.enc's NormalizeImg rounds it (the learner engine's conv stack
// then reads normalised frames: the division leaves its inner loops).
__global__ void __launch_bounds__(256) random_shift_kernel(const float* x, const float* shift, int C, int h, int w,
                                                           int pad, float div, float* out) {
    const int k = blockIdx.y;                        // stacked image
    const int sx = (int)shift[2 * k], sy = (int)shift[2 * k + 1];
    const size_t plane = (size_t)h * w;
    const int total = C * h * w;
    for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
        const int c = e / (h * w), r = e % (h * w), i = r / w, j = r % w;
        const int si = min(max(i + sy - pad, 0), h - 1), sj = min(max(j + sx - pad, 0), w - 1);
        const float v = x[(size_t)k * C * plane + c * plane + (size_t)si * w + sj];
        out[(size_t)k * C * plane + e] = div > 0.f ? __fdiv_rn(v, div) : v;
    }
}

}  // namespace

extern "C" {

int tdmpc_random_shift(const float* x, const float* shift, int32_t n, int32_t c, int32_t h, int32_t w, int32_t pad,
                       float* out, void* stream) {
    return tdmpc_random_shift_scaled(x, shift, n, c, h, w, pad, 0.f, out, stream);
}

int tdmpc_random_shift_scaled(const float* x, const float* shift, int32_t n, int32_t c, int32_t h, int32_t w,
                              int32_t pad, float div, float* out, void* stream) {
    if (!x || !shift || !out) return TDMPC_E_NULL;
    if (n <= 0 || c <= 0 || h <= 0 || w <= 0 || pad < 0 || (long)c * h * w >= (1L << 31)) return TDMPC_E_DIMS;
    const int per = c * h * w;
    hipLaunchKernelGGL(random_shift_kernel, dim3(std::min((per + 255) / 256, 64), n), dim3(256), 0,
                       (hipStream_t)stream, x, shift, c, h, w, pad, div, out);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        tdmpc_internal::set_error(hipGetErrorString(e));
        return TDMPC_E_HIP;
    }
    return 0;
}


int tdmpc_loss_forward(const tdmpc_loss_args* a, float* rows, float* scal, void* stream) {
    if (!args_ok(a) || !rows || !scal) return TDMPC_E_NULL;
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(loss_rows_kernel, dim3((a->B + 3) / 4), dim3(256), 0, s, *a, rows);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e);
    hipLaunchKernelGGL(loss_means_kernel, dim3(1), dim3(512), 0, s, *a, rows, scal);
    e = hipGetLastError();
    return e == hipSuccess ? 0 : hip_fail(e);
}

int tdmpc_loss_backward(const tdmpc_loss_args* a, const float* rows, const float* scal, const float* gw, float* dzp,
                        float* dq1, float* dq2, float* drp, void* stream) {
    if (!args_ok(a) || !rows || !scal || !gw) return TDMPC_E_NULL;
    const long n = (long)a->H * a->B * a->L;
    hipLaunchKernelGGL(loss_backward_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       *a, rows, scal, gw, dzp, dq1, dq2, drp);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : hip_fail(e);
}

}  // extern "C"
