// replay_kernels.hip -- MI355X (gfx950) prioritized replay sampling, C ABI in
// include/tdmpc_replay.h, built into libtdmpc_hip.so next to the planner.
//
// Reference: ReplayBuffer in /root/reference/src/algorithm/helper.py:434-534. Its sample() computes
// probs = p**alpha / sum(p**alpha) on the device, copies them to the host and runs
// np.random.choice(total, B, p=probs, replace=not full): numpy converts p to float64, cdf = cumsum(p),
// cdf /= cdf[-1], and takes searchsorted(cdf, uniform, side='right') -- once for B uniforms with
// replacement, in rounds (found entries' p zeroed, cdf recomputed, duplicates of a round dropped keeping
// first occurrences) without. This file does all of it on the device:
//   rp_pow_kernel     p = powf(prio, alpha) and per-2048-block fp32 sums           (HBM: 4 B read + 4 B write)
//   rp_scan_kernel    S = sum of the block sums (fixed tree order, recomputed per block), probs = p / S (fp32),
//                     float64 inclusive cdf per block                               (4 B read, 4 + 8 B write)
//   rp_offsets_kernel float64 block offsets, last = cdf[-1]
//   rp_choice_kernel  with replacement (and round 1 without): one wave per draw, 64-ary search on cdf/last
//   rp_norepl_kernel  without replacement: numpy's later rounds in one workgroup; the zeroed masses of the found
//                     entries are subtracted from the cdf instead of recomputing it
//   rp_gather_kernel  the H+1-step windows (state rows or pixel frame stacks), episode-end last_obs, and the
//                     importance weights (total * probs[idx])**-beta / max
// Exactness: the float64 cdf is a sum of float32 values; when every partial sum is exact in float64 (true
// unless the probabilities span more than ~2^29 in ratio) any summation order -- numpy's sequential one,
// this blocked scan, or cdf minus the found masses -- gives the same bits, so the chosen indices are
// numpy's. probs itself depends on the fp32 order of sum(p**alpha) (torch's reduction order is its own).
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>

#include "../../include/tdmpc_hip.h"
#include "../../include/tdmpc_replay.h"

namespace tdmpc_internal {
void set_error(const char* msg);
}

namespace {

#define DEVI __device__ __forceinline__
constexpr int RB = 2048;   // elements per scan block
constexpr int RT = 256;    // threads per scan block (8 consecutive elements each)

#define RCHK(x)                                                                   \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            tdmpc_internal::set_error(hipGetErrorString(e_));                     \
            return TDMPC_E_HIP;                                                   \
        }                                                                         \
    } while (0)

inline size_t rup(size_t x, size_t a) { return (x + a - 1) / a * a; }

struct RWork {
    float* p;        // [cap] p**alpha
    double* cdf;     // [cap] in-block inclusive cdf
    float* probs;    // [cap]
    float* bsum;     // [nb] fp32 block sums of p
    double* btot;    // [nb] float64 block totals of probs
    double* boff;    // [nb] float64 block offsets
    double* scal;    // [0] S (sum of p, as float), [1] last = cdf[-1]
    float* part;     // [nb] partial maxima (add_priorities)
    int64_t* idx;    // [B] chosen indices (without replacement: the first round's draws first)
    unsigned long long* last;  // [cap] update_priorities: (generation << 32 | position) of the last writer
    unsigned* gen;   // [1] update_priorities: generation counter
    size_t total;
};

bool dims_ok(const tdmpc_replay_dims* d) {
    if (!d || d->capacity <= 0 || d->episode_length <= 0 || d->capacity % d->episode_length || d->horizon < 0 ||
        d->horizon >= d->episode_length || d->batch_size <= 0 || d->batch_size > 1024 || d->action_dim <= 0)
        return false;
    if (d->modality == 0) return d->obs_dim > 0;
    return d->modality == 1 && d->img_hw > 0 && d->frame_stack > 0;
}

void make_rwork(const tdmpc_replay_dims* d, char* base, RWork* w) {
    const size_t cap = d->capacity, nb = (cap + RB - 1) / RB, B = d->batch_size;
    size_t o = 0;
    auto take = [&](size_t bytes) { size_t r = o; o += rup(bytes, 256); return base ? base + r : nullptr; };
    w->p = (float*)take(cap * 4);
    w->cdf = (double*)take(cap * 8);
    w->probs = (float*)take(cap * 4);
    w->bsum = (float*)take(nb * 4);
    w->btot = (double*)take(nb * 8);
    w->boff = (double*)take(nb * 8);
    w->scal = (double*)take(64);
    w->part = (float*)take(nb * 4);
    w->idx = (int64_t*)take(B * 8);
    w->last = (unsigned long long*)take(cap * 8);
    w->gen = (unsigned*)take(64);
    w->total = o;
}

DEVI float nanmax(float a, float b) { return (a != a || b != b) ? NAN : fmaxf(a, b); }   // torch.max keeps NaN

// ------------------------------------------------------------------------------------------------ probs
__global__ void __launch_bounds__(RT) rp_pow_kernel(const float* prio, int total, float alpha, float* p, float* bsum) {
    __shared__ float red[RT];
    const int t = threadIdx.x, base = blockIdx.x * RB + t * 8;
    float s = 0.f;
    if (base + 8 <= total) {
        const float4 a = *(const float4*)(prio + base), b = *(const float4*)(prio + base + 4);
        float v[8] = {powf(a.x, alpha), powf(a.y, alpha), powf(a.z, alpha), powf(a.w, alpha),
                      powf(b.x, alpha), powf(b.y, alpha), powf(b.z, alpha), powf(b.w, alpha)};
        *(float4*)(p + base) = make_float4(v[0], v[1], v[2], v[3]);
        *(float4*)(p + base + 4) = make_float4(v[4], v[5], v[6], v[7]);
        for (int k = 0; k < 8; ++k) s += v[k];
    } else {
        for (int k = 0; k < 8; ++k)
            if (base + k < total) {
                const float v = powf(prio[base + k], alpha);
                p[base + k] = v;
                s += v;
            }
    }
    red[t] = s;
    __syncthreads();
    for (int off = RT / 2; off > 0; off >>= 1) {
        if (t < off) red[t] += red[t + off];
        __syncthreads();
    }
    if (t == 0) bsum[blockIdx.x] = red[0];
}

// S = sum of the fp32 block sums in a fixed order: slot i < 1024 holds bsum[i] + bsum[i + 1024] + ..., then a
// halving tree over the 1024 slots. Every scan block recomputes it from the ~nb / 1024 floats (the same bits in each
// block), so no separate launch is needed between the pow pass and the scan.
DEVI float total_of(const float* bsum, int nb, float* red, int t) {   // 256 threads, red[256]
    float v[4];
    for (int q = 0; q < 4; ++q) {
        float x = 0.f;
        for (int i = t + 256 * q; i < nb; i += 1024) x += bsum[i];
        v[q] = x;
    }
    v[0] += v[2];   // tree level 512: slot i += slot i + 512 (i = t, t + 256)
    v[1] += v[3];
    red[t] = v[0] + v[1];   // level 256
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if (t < off) red[t] += red[t + off];
        __syncthreads();
    }
    const float S = red[0];
    __syncthreads();
    return S;
}

// probs = p / S (fp32, like `probs /= probs.sum()`), then the float64 inclusive cdf of each 2048-block:
// 8 elements per thread sequentially, thread totals scanned across the block.
__global__ void __launch_bounds__(RT) rp_scan_kernel(const float* p, int total, const float* bsum, int nb,
                                                     float* probs, float* probs_out, double* cdf, double* btot) {
    __shared__ double ts[RT];
    __shared__ float red[RT];
    const int t = threadIdx.x, base = blockIdx.x * RB + t * 8;
    const float S = total_of(bsum, nb, red, t);
    double run = 0.0, loc[8];
    for (int k = 0; k < 8; ++k) {
        const int i = base + k;
        double v = 0.0;
        if (i < total) {
            const float q = __fdiv_rn(p[i], S);
            probs[i] = q;
            if (probs_out) probs_out[i] = q;
            v = (double)q;
        }
        run += v;
        loc[k] = run;
    }
    ts[t] = run;
    __syncthreads();
    // inclusive scan of the thread totals (Hillis-Steele; RT = 256)
    for (int off = 1; off < RT; off <<= 1) {
        const double add = t >= off ? ts[t - off] : 0.0;
        __syncthreads();
        ts[t] += add;
        __syncthreads();
    }
    const double excl = t ? ts[t - 1] : 0.0;
    for (int k = 0; k < 8; ++k)
        if (base + k < total) cdf[base + k] = excl + loc[k];
    if (t == RT - 1) btot[blockIdx.x] = ts[RT - 1];
}

// exclusive float64 scan of the block totals (chunks of 1024, Hillis-Steele), last = their sum
__global__ void __launch_bounds__(1024) rp_offsets_kernel(const double* btot, int nb, double* boff, double* scal) {
    __shared__ double ts[1024];
    const int t = threadIdx.x;
    double carry = 0.0;
    for (int c0 = 0; c0 < nb; c0 += 1024) {
        const double v = c0 + t < nb ? btot[c0 + t] : 0.0;
        ts[t] = v;
        __syncthreads();
        for (int off = 1; off < 1024; off <<= 1) {
            const double add = t >= off ? ts[t - off] : 0.0;
            __syncthreads();
            ts[t] += add;
            __syncthreads();
        }
        if (c0 + t < nb) boff[c0 + t] = carry + (t ? ts[t - 1] : 0.0);
        carry += ts[1023];
        __syncthreads();
    }
    if (t == 0) scal[1] = carry;
}

DEVI double cdf_at(const double* cdf, const double* boff, int i) { return cdf[i] + boff[i / RB]; }

// ------------------------------------------------------------------------------------------------ choice
// With replacement: draw b is searchsorted(cdf / last, u[b], side='right') -- the first i with
// u < cdf[i] / last -- by one wave: 64 probes per round narrow [lo, hi) 64-fold.
__global__ void __launch_bounds__(64) rp_choice_kernel(const double* cdf, const double* boff, const double* scal,
                                                       int total, const double* u, int64_t* idx, int32_t* n_used) {
    const int lane = threadIdx.x, b = blockIdx.x;
    if (b == 0 && lane == 0 && n_used) *n_used = gridDim.x;   // one uniform per draw
    const double x = u[b], last = scal[1];
    int lo = 0, hi = total;   // invariant: the answer is in [lo, hi) and cdf[hi - 1] / last > x
    while (hi - lo > 64) {
        const int step = (hi - lo + 63) / 64;
        const int i = min(lo + (lane + 1) * step - 1, hi - 1);
        const bool pred = x < cdf_at(cdf, boff, i) / last;
        const unsigned long long m = __ballot(pred);
        const int l = m ? __ffsll(m) - 1 : 63;
        const int il = min(lo + (l + 1) * step - 1, hi - 1);
        const int ip = l ? min(lo + l * step - 1, hi - 1) + 1 : lo;
        lo = ip;
        hi = il + 1;
    }
    const int i = lo + lane;
    const bool pred = i < hi && x < cdf_at(cdf, boff, i) / last;
    const unsigned long long m = __ballot(pred);
    if (lane == 0) idx[b] = m ? lo + __ffsll(m) - 1 : hi - 1;
}

// Ascending bitonic sort of 1024 keys, one per thread of a 1024-thread block, returned in the thread's register
// (thread t holds the t-th smallest). Partner distances below 64 run in the wave (xor shuffles, no barrier); only
// the 10 steps with j >= 64 go through LDS (`buf`, 1024 keys).
template <typename K>
DEVI K bitonic1024(K v, K* buf, int t) {
    for (int k = 2; k <= 1024; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            K o;
            if (j >= 64) {
                buf[t] = v;
                __syncthreads();
                o = buf[t ^ j];
                __syncthreads();
            } else {
                o = __shfl_xor(v, j, 64);
            }
            const bool lower = (t & j) == 0, up = (t & k) == 0;
            // the lower partner keeps the min when ascending, the max when descending
            v = (lower == up) ? (o < v ? o : v) : (o < v ? v : o);
        }
    return v;
}

// Inclusive prefix sum over a 1024-thread block: wave scans by shuffles, then the 16 wave totals (2 barriers).
template <typename T>
DEVI T block_scan1024(T v, T* wsum, int t) {
    const int lane = t & 63, w = t >> 6;
    for (int o = 1; o < 64; o <<= 1) {
        const T u = __shfl_up(v, o, 64);
        if (lane >= o) v += u;
    }
    if (lane == 63) wsum[w] = v;
    __syncthreads();
    T add = 0;
    for (int i = 0; i < w; ++i) add += wsum[i];
    __syncthreads();
    return v + add;
}

// Uniform number k >= n_u of a without-replacement sample whose caller-supplied stream ran out: a splitmix64 hash of
// the stream's last value and k, as a double in [0, 1) (53 bits). Deterministic, and only reached when numpy's
// rounds need more than n_u uniforms (n_used then reports the total consumed, > n_u).
DEVI double extra_uniform(const double* u, int n_u, int k) {
    unsigned long long z = (unsigned long long)__double_as_longlong(u[n_u - 1]) + 0x9e3779b97f4a7c15ull * (unsigned)(k + 1);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    z ^= z >> 31;
    return (double)(z >> 11) * 0x1.0p-53;
}

// Without replacement (numpy's rounds, RandomState.choice(replace=False, p)): round 1 has no found entries, so its
// draws are rp_choice_kernel's (one wave per draw, in idx on entry); this workgroup keeps their first occurrences and
// runs the later rounds -- usually zero or one, with a few draws -- itself: one wave per draw, 64-ary search of
// u < cdf'(i) / last' where cdf' = cdf - (mass of found entries <= i) and last' = last - (mass of all found), the
// found set kept sorted in LDS with float64 prefix masses. First occurrences per round (np.unique(return_index))
// come from an LDS hash set; the found set is re-sorted only when another round follows (a draw never repeats a
// found entry: those have no mass left). n_used: uniforms consumed;
// -2 when fewer than B entries have non-zero probability (numpy raises "Fewer non-zero entries in p than size";
// idx is then padded with 0).
__global__ void __launch_bounds__(1024) rp_norepl_kernel(const double* cdf, const double* boff, const double* scal,
                                                         const float* probs, int total, int B, const double* u,
                                                         int n_u, int64_t* idx, int32_t* n_used) {
    __shared__ int fs[1024];        // found indices, sorted ascending, [0, nf)
    __shared__ double fm[1024];     // fm[k] = mass of fs[0..k]
    __shared__ int order[1024];     // found indices in numpy's output order
    __shared__ int nv[1024];        // this round's draws
    __shared__ int newv[1024];      // this round's new found values
    __shared__ int hkey[2048];      // hash set of the round's values
    __shared__ int hpos[2048];      // smallest draw position per value
    __shared__ int sk[1024];        // sort exchange buffer
    __shared__ int iws[16];
    __shared__ double dws[16];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6, nw = blockDim.x >> 6;
    int n_uniq = 0, used = 0, nf = 0;
    const double last = scal[1];
    bool ok = true;
    if (t < B) nv[t] = (int)idx[t];   // round 1 (rp_choice_kernel)
    __syncthreads();
    for (int round = 0; n_uniq < B; ++round) {
        const int m = B - n_uniq;
        const double lastp = last - (nf ? fm[nf - 1] : 0.0);
        if (round > 0) {
            if (!(lastp > 0.0)) { ok = false; break; }   // every entry with mass is found already
            for (int j = wave; j < m; j += nw) {
                const int k = used + j;
                const double x = k < n_u ? u[k] : extra_uniform(u, n_u, k);
                int lo = 0, hi = total;   // answer in [lo, hi): the first i with x < cdf'(i) / last'
                while (hi > lo) {
                    const int len = hi - lo, step = (len + 63) / 64;
                    const int i = min(lo + (lane + 1) * step - 1, hi - 1);
                    int a = 0, bnd = nf;   // found entries <= i
                    while (a < bnd) {
                        const int c = (a + bnd) >> 1;
                        if (fs[c] <= i) a = c + 1; else bnd = c;
                    }
                    const bool pred = x < (cdf_at(cdf, boff, i) - (a ? fm[a - 1] : 0.0)) / lastp;
                    const unsigned long long bm = __ballot(pred);
                    if (step == 1) {   // the probes were lo .. hi - 1 themselves
                        lo = bm ? lo + __ffsll(bm) - 1 : hi - 1;
                        break;
                    }
                    const int l = bm ? __ffsll(bm) - 1 : 63;
                    const int il = min(lo + (l + 1) * step - 1, hi - 1);
                    lo = l ? min(lo + l * step - 1, hi - 1) + 1 : lo;
                    hi = il + 1;
                }
                if (lane == 0) nv[j] = min(lo, total - 1);
            }
            __syncthreads();
        }
        used += m;
        // first occurrences (np.unique(return_index)): an LDS hash set of the round's values, each slot keeping
        // the smallest draw position that holds its value
        hkey[t] = -1; hkey[t + 1024] = -1;
        hpos[t] = 0x7fffffff; hpos[t + 1024] = 0x7fffffff;
        __syncthreads();
        int slot = 0;
        if (t < m) {
            const int v = nv[t];
            slot = (int)(((unsigned)v * 2654435761u) >> 21);   // 11 bits
            while (true) {
                const int old = atomicCAS(&hkey[slot], -1, v);
                if (old == -1 || old == v) break;
                slot = (slot + 1) & 2047;
            }
            atomicMin(&hpos[slot], t);
        }
        __syncthreads();
        const bool first = t < m && hpos[slot] == t;
        const int rank = block_scan1024(first ? 1 : 0, iws, t) - (first ? 1 : 0);
        int nnew = 0;
        for (int i = 0; i < 16; ++i) nnew += iws[i];
        if (first) {
            order[n_uniq + rank] = nv[t];
            newv[rank] = nv[t];
        }
        n_uniq += nnew;
        __syncthreads();
        if (n_uniq >= B) break;
        // the next round searches cdf - (found masses): found set = previous found + this round's, sorted
        int v2 = t < nf ? fs[t] : (t < nf + nnew ? newv[t - nf] : 0x7fffffff);
        v2 = bitonic1024(v2, sk, t);
        fs[t] = v2;
        nf += nnew;
        const double fmv = block_scan1024(t < nf ? (double)probs[v2] : 0.0, dws, t);
        fm[t] = fmv;
        __syncthreads();
    }
    if (t < B) idx[t] = t < n_uniq ? order[t] : 0;
    if (t == 0 && n_used) *n_used = ok ? used : -2;
}

// ------------------------------------------------------------------------------------------------ gather
struct GatherArgs {
    int modality, F, S, fs, A, L, H, B;
    long cap;   // storage rows: action/reward [cap], obs [cap + 1]
    const void* obs; const void* last_obs; const float* action; const float* reward;
    const int64_t* idx;
    // importance weights (helper.py:518-519): weights[b] = (total * probs[idx[b]])**-beta / max over the batch
    const float* probs; int total; float beta; int64_t* idx_out; float* weights;
    float* o_obs; float* o_next; float* o_action; float* o_reward;
};

// stacked observation of storage index j into dst: state = row j; pixels = frame_stack frames back from j
// that do not cross the episode start (helper.py:490-502), oldest first, as floats.
DEVI void stacked_obs(const GatherArgs& a, long j, float* dst) {
    if (j > a.cap) {
        // a window past the storage end (only reachable when a caller gave a masked episode tail a non-zero
        // priority; the reference raises IndexError there): NaN rows instead of an out-of-bounds read
        const int F = a.modality == 0 ? a.F : a.fs * 3 * a.S * a.S;
        for (int k = threadIdx.x; k < F; k += blockDim.x) dst[k] = NAN;
        return;
    }
    if (a.modality == 0) {
        const float* src = (const float*)a.obs + (size_t)j * a.F;
        for (int k = threadIdx.x; k < a.F; k += blockDim.x) dst[k] = src[k];
        return;
    }
    const int plane = a.S * a.S, frame = 3 * plane;
    const long start = j - j % a.L;
    for (int k = threadIdx.x; k < a.fs * frame; k += blockDim.x) {
        const int c = k / plane, pix = k % plane;
        const int back = a.fs - 1 - c / 3;                 // 0 = newest frame (last 3 channels)
        const long src_j = max(j - back, start);
        dst[k] = (float)((const uint8_t*)a.obs)[(size_t)src_j * frame + (c % 3) * plane + pix];
    }
}

__global__ void __launch_bounds__(256) rp_gather_kernel(const GatherArgs a) {
    const int b = blockIdx.x, y = blockIdx.y;
    const long i = a.idx[b];
    const int F = a.modality == 0 ? a.F : a.fs * 3 * a.S * a.S;
    if (y == 0) {
        // the batch's largest weight (torch.max keeps NaN), recomputed by each row's block (B powf's from L2)
        __shared__ float red[256];
        const int t = threadIdx.x;
        float m = -INFINITY;
        for (int k = t; k < a.B; k += 256) m = nanmax(m, powf(__fmul_rn((float)a.total, a.probs[a.idx[k]]), -a.beta));
        red[t] = m;
        __syncthreads();
        for (int off = 128; off > 0; off >>= 1) {
            if (t < off) red[t] = nanmax(red[t], red[t + off]);
            __syncthreads();
        }
        if (t == 0) {
            a.weights[b] = __fdiv_rn(powf(__fmul_rn((float)a.total, a.probs[i]), -a.beta), red[0]);
            a.idx_out[b] = i;
        }
        stacked_obs(a, i, a.o_obs + (size_t)b * F);
        return;
    }
    const int t = y - 1;
    float* dst = a.o_next + ((size_t)t * a.B + b) * F;
    if (t == a.H && (i + a.H + 1) % a.L == 0 && i + a.H < a.cap) {
        // episode end: the stored final observation (helper.py:525-526)
        const long e = (i + a.H) / a.L;
        if (a.modality == 0) {
            const float* src = (const float*)a.last_obs + (size_t)e * F;
            for (int k = threadIdx.x; k < F; k += blockDim.x) dst[k] = src[k];
        } else {
            const uint8_t* src = (const uint8_t*)a.last_obs + (size_t)e * F;
            for (int k = threadIdx.x; k < F; k += blockDim.x) dst[k] = (float)src[k];
        }
    } else {
        stacked_obs(a, i + t + 1, dst);
    }
    const bool in = i + t < a.cap;
    for (int k = threadIdx.x; k < a.A; k += blockDim.x)
        a.o_action[((size_t)t * a.B + b) * a.A + k] = in ? a.action[(size_t)(i + t) * a.A + k] : NAN;
    if (threadIdx.x == 0) a.o_reward[(size_t)t * a.B + b] = in ? a.reward[i + t] : NAN;
}

// ------------------------------------------------------------------------------------------------ add
__global__ void __launch_bounds__(RT) rp_max_kernel(const float* prio, int n, float* part) {
    __shared__ float red[RT];
    const int t = threadIdx.x, base = blockIdx.x * RB + t * 8;
    float m = -INFINITY;
    for (int k = 0; k < 8; ++k)
        if (base + k < n) m = nanmax(m, prio[base + k]);
    red[t] = m;
    __syncthreads();
    for (int off = RT / 2; off > 0; off >>= 1) {
        if (t < off) red[t] = nanmax(red[t], red[t + off]);
        __syncthreads();
    }
    if (t == 0) part[blockIdx.x] = red[0];
}

__global__ void __launch_bounds__(1024) rp_add_prio_kernel(float* prio, const float* part, int nparts, int idx, int L,
                                                           int H, int first) {
    __shared__ float red[1024];
    const int t = threadIdx.x;
    float m = -INFINITY;
    for (int i = t; i < nparts; i += 1024) m = nanmax(m, part[i]);
    red[t] = m;
    __syncthreads();
    for (int off = 512; off > 0; off >>= 1) {
        if (t < off) red[t] = nanmax(red[t], red[t + off]);
        __syncthreads();
    }
    const float maxp = first ? 1.0f : red[0];
    for (int k = t; k < L; k += 1024) prio[idx + k] = k >= L - H ? 0.f : maxp;
}

// p[idxs[i]] = v[i] + eps; with duplicate indices the LAST occurrence wins, like a sequential index_put_ (the
// reference's CPU semantics; its GPU index_put_ leaves the winner unspecified). Last-writer-wins in O(n): every
// position i posts (generation << 32 | i) to last[idxs[i]] with a 64-bit atomicMax; the position that finds its own
// key there writes. The generation (a device counter bumped after each call) makes older calls' keys smaller, so
// `last` never needs clearing (it starts zeroed with the workspace).
__global__ void rp_update_post_kernel(unsigned long long* last, const unsigned* gen, const int64_t* idxs, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const unsigned long long key = ((unsigned long long)(*gen + 1u) << 32) | (unsigned)i;
    atomicMax(last + idxs[i], key);
}

__global__ void rp_update_write_kernel(float* prio, const unsigned long long* last, const unsigned* gen,
                                       const int64_t* idxs, const float* v, int n, float eps) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const unsigned long long key = ((unsigned long long)(*gen + 1u) << 32) | (unsigned)i;
    const int64_t k = idxs[i];
    if (last[k] == key) prio[k] = __fadd_rn(v[i], eps);
}

__global__ void rp_update_bump_kernel(unsigned* gen) { *gen += 1u; }

// n <= RP_UPD_ONE (a learner batch): the three kernels above as the phases of ONE workgroup, a barrier between them
// (the generation-tagged keys are the same, so the paths mix across calls)
constexpr int RP_UPD_ONE = 1024;
__global__ void __launch_bounds__(RP_UPD_ONE) rp_update_one_kernel(float* prio, unsigned long long* last,
                                                                   unsigned* gen, const int64_t* idxs, const float* v,
                                                                   int n, float eps) {
    const int i = threadIdx.x;
    const unsigned g = *gen + 1u;
    const unsigned long long key = ((unsigned long long)g << 32) | (unsigned)i;
    const int64_t k = i < n ? idxs[i] : 0;
    if (i < n) atomicMax(last + k, key);
    __syncthreads();
    if (i < n && __hip_atomic_load(last + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == key)
        prio[k] = __fadd_rn(v[i], eps);
    __syncthreads();
    if (i == 0) *gen = g;
}

}  // namespace

extern "C" {

size_t tdmpc_replay_workspace_bytes(const tdmpc_replay_dims* d) {
    if (!dims_ok(d)) return 0;
    RWork w;
    make_rwork(d, nullptr, &w);
    return w.total;
}

int tdmpc_replay_add_priorities(const tdmpc_replay_dims* d, float* prio, int32_t idx, int32_t full, void* ws,
                                size_t ws_bytes, void* stream) {
    if (!d || !prio || !ws) return TDMPC_E_NULL;
    if (!dims_ok(d)) return TDMPC_E_DIMS;
    if (idx < 0 || idx % d->episode_length || idx + d->episode_length > d->capacity) return TDMPC_E_DIMS;
    RWork w;
    make_rwork(d, nullptr, &w);
    if (ws_bytes < w.total) return TDMPC_E_SIZE;
    make_rwork(d, (char*)ws, &w);
    hipStream_t s = (hipStream_t)stream;
    const int n = full ? d->capacity : idx;   // running max over everything stored so far
    const int nb = std::max(1, (n + RB - 1) / RB);
    if (n > 0) hipLaunchKernelGGL(rp_max_kernel, dim3(nb), dim3(RT), 0, s, prio, n, w.part);
    RCHK(hipGetLastError());
    hipLaunchKernelGGL(rp_add_prio_kernel, dim3(1), dim3(1024), 0, s, prio, w.part, n > 0 ? nb : 0, idx,
                       d->episode_length, d->horizon, (int)(n == 0));
    RCHK(hipGetLastError());
    return 0;
}

int tdmpc_replay_update_priorities(const tdmpc_replay_dims* d, float* prio, const int64_t* idxs,
                                   const float* values, int32_t n, float eps, void* ws, size_t ws_bytes,
                                   void* stream) {
    if (!d || !prio || !idxs || !values || !ws) return TDMPC_E_NULL;
    if (!dims_ok(d) || n < 0) return TDMPC_E_DIMS;
    RWork w;
    make_rwork(d, nullptr, &w);
    if (ws_bytes < w.total) return TDMPC_E_SIZE;
    make_rwork(d, (char*)ws, &w);
    if (!n) return 0;
    hipStream_t s = (hipStream_t)stream;
    if (n <= RP_UPD_ONE) {
        hipLaunchKernelGGL(rp_update_one_kernel, dim3(1), dim3(RP_UPD_ONE), 0, s, prio, w.last, w.gen, idxs, values, n,
                           eps);
        RCHK(hipGetLastError());
        return 0;
    }
    const dim3 grid((n + 255) / 256);
    hipLaunchKernelGGL(rp_update_post_kernel, grid, dim3(256), 0, s, w.last, w.gen, idxs, n);
    RCHK(hipGetLastError());
    hipLaunchKernelGGL(rp_update_write_kernel, grid, dim3(256), 0, s, prio, w.last, w.gen, idxs, values, n, eps);
    RCHK(hipGetLastError());
    hipLaunchKernelGGL(rp_update_bump_kernel, dim3(1), dim3(1), 0, s, w.gen);
    RCHK(hipGetLastError());
    return 0;
}

int tdmpc_replay_sample(const tdmpc_replay_dims* d, const tdmpc_replay_store* st, int32_t total, int32_t full,
                        float alpha, float beta, const double* u, int32_t n_u, int64_t* idxs, float* weights,
                        float* obs, float* next_obs, float* action, float* reward, float* probs_out,
                        int32_t* n_used, void* ws, size_t ws_bytes, void* stream) {
    if (!d || !st || !u || !idxs || !weights || !obs || !next_obs || !action || !reward || !ws) return TDMPC_E_NULL;
    if (!st->obs || !st->last_obs || !st->action || !st->reward || !st->priorities) return TDMPC_E_NULL;
    if (!dims_ok(d) || total <= 0 || total > d->capacity) return TDMPC_E_DIMS;
    const int B = d->batch_size;
    if (n_u < B || (full && total < B)) return TDMPC_E_DIMS;
    RWork w;
    make_rwork(d, nullptr, &w);
    if (ws_bytes < w.total) return TDMPC_E_SIZE;
    make_rwork(d, (char*)ws, &w);
    hipStream_t s = (hipStream_t)stream;
    const int nb = (total + RB - 1) / RB;
    hipLaunchKernelGGL(rp_pow_kernel, dim3(nb), dim3(RT), 0, s, st->priorities, total, alpha, w.p, w.bsum);
    RCHK(hipGetLastError());
    hipLaunchKernelGGL(rp_scan_kernel, dim3(nb), dim3(RT), 0, s, w.p, total, w.bsum, nb, w.probs, probs_out, w.cdf,
                       w.btot);
    RCHK(hipGetLastError());
    hipLaunchKernelGGL(rp_offsets_kernel, dim3(1), dim3(1024), 0, s, w.btot, nb, w.boff, w.scal);
    RCHK(hipGetLastError());
    // round 1 of both forms: one wave per draw
    hipLaunchKernelGGL(rp_choice_kernel, dim3(B), dim3(64), 0, s, w.cdf, w.boff, w.scal, total, u, w.idx, n_used);
    RCHK(hipGetLastError());
    if (full) {
        hipLaunchKernelGGL(rp_norepl_kernel, dim3(1), dim3(1024), 0, s, w.cdf, w.boff, w.scal, w.probs, total, B, u,
                           n_u, w.idx, n_used);
        RCHK(hipGetLastError());
    }
    GatherArgs g;
    g.modality = d->modality; g.F = d->obs_dim; g.S = d->img_hw; g.fs = d->frame_stack; g.A = d->action_dim;
    g.L = d->episode_length; g.H = d->horizon; g.B = B;
    g.cap = d->capacity;
    g.obs = st->obs; g.last_obs = st->last_obs; g.action = st->action; g.reward = st->reward; g.idx = w.idx;
    g.probs = w.probs; g.total = total; g.beta = beta; g.idx_out = idxs; g.weights = weights;
    g.o_obs = obs; g.o_next = next_obs; g.o_action = action; g.o_reward = reward;
    hipLaunchKernelGGL(rp_gather_kernel, dim3(B, d->horizon + 2), dim3(256), 0, s, g);
    RCHK(hipGetLastError());
    return 0;
}

}  // extern "C"
