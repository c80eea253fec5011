/*
 * tdmpc_hip.h -- C ABI of libtdmpc_hip.so, the MI355X (gfx950) TD-MPC planner.
 *
 * This is the drop-in boundary of the planning hot path. The reference has no FFI: its
 * boundary is the Python method `TDMPC.plan(obs, eval_mode=False, step=None, t0=True)`
 * (/root/reference/src/algorithm/tdmpc.py:94-163). `tdmpc_amd.TDMPC.plan` keeps that signature and calls
 * the entry points below through ctypes; any other host (C, C++, a cgo/JNI stub) can call them directly.
 *
 * Conventions
 *   - Every pointer argument except `dims`, `params`, `layout` and the host-side arrays documented as such
 *     is a DEVICE pointer owned by the caller. No entry point allocates device memory or synchronises.
 *   - `stream` is a hipStream_t (NULL = default stream). Work is enqueued in stream order, so a call can be
 *     captured into a hipGraph.
 *   - Return 0 on success, a negative TDMPC_E* code otherwise. No exceptions cross the ABI.
 *   - fp32 everywhere except the elite-choice uniform `u` (float64, like numpy's random_sample).
 *   - Thread safety: no global mutable state; calls on distinct streams with distinct workspaces are safe.
 */
#ifndef TDMPC_HIP_H
#define TDMPC_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TDMPC_ABI_VERSION 8

#define TDMPC_OK 0
#define TDMPC_E_DIMS (-1)     /* unsupported or inconsistent dims / params */
#define TDMPC_E_HIP (-2)      /* a HIP runtime call failed (hipGetLastError after a launch) */
#define TDMPC_E_NULL (-3)     /* a required pointer is NULL */
#define TDMPC_E_SIZE (-4)     /* a caller buffer is smaller than tdmpc_sizes() says */

/* Static shape of one planner instance. Mirrors the cfg keys the reference reads
 * (cfgs/default.yaml:10-16,29,72-74; obs_shape/action_dim from envs/env.py:284-286). */
typedef struct tdmpc_dims {
    int32_t modality;      /* 0 = state, 1 = pixels (helper.enc, helper.py:119-133) */
    int32_t obs_dim;       /* state: obs_shape[0]; pixels: unused */
    int32_t img_c;         /* pixels: 3*frame_stack */
    int32_t img_hw;        /* pixels: img_size */
    int32_t num_channels;  /* pixels: conv channels */
    int32_t action_dim;    /* A */
    int32_t latent_dim;    /* L */
    int32_t mlp_dim;       /* M (hidden width of d, R, pi, Q); must be 512 or a multiple of 64 */
    int32_t enc_dim;       /* E (state encoder hidden width) */
    int32_t num_samples;   /* N  (cfg.num_samples) */
    int32_t num_pi;        /* P = int(mixture_coef * N) */
    int32_t num_elites;    /* K */
    int32_t max_horizon;   /* largest H any call will use (workspace is sized for it) */
    int32_t max_iterations;/* largest cfg.iterations any call will use */
    int32_t max_batch;     /* largest number of environments planned per call */
    int32_t enc_norm;      /* state encoder: 0 = Linear-ELU-Linear (helper.enc, helper.py:130-132); 1 = with a
                              LayerNorm after the first Linear (helper.dmlab_enc_norm for state with
                              norm_type 'ln', helper.py:156-166: the iCEM agent's cfg.normalize) */
} tdmpc_dims;

/* Per-call scalars (tdmpc.py:106-149). */
typedef struct tdmpc_plan_params {
    int32_t horizon;       /* H = int(min(cfg.horizon, linear_schedule(horizon_schedule, step))) */
    int32_t iterations;    /* cfg.iterations */
    int32_t batch;         /* number of environments in this call (<= max_batch) */
    int32_t warm_start;    /* 1: mean[:-1] = prev_mean[1:] (not t0 and prev_mean exists) */
    int32_t eval_mode;     /* 1: no final action noise (tdmpc.py:157) */
    float min_std;         /* cfg.min_std (TruncatedNormal scale for pi) */
    float temperature;     /* cfg.temperature */
    float momentum;        /* cfg.momentum, as float32 */
    float one_minus_momentum; /* float32(1 - momentum) computed in float64 like Python does */
    float std_floor;       /* self.std: lower clamp of the CEM std (tdmpc.py:148) */
    float discount_pow[17];/* float32(discount**t) for t = 0..H, the running Python-float product */
    int32_t path;          /* kernel path: 0 = auto by row count, 1 = layered GEMMs only, 2 = row-block chain
                              kernels wherever the shape allows (row block by launch size), 3 / 4 = chain
                              kernels on 32- / 16-row blocks only, 5 = TOLD.next on the column-split step kernel
                              (others layered), 6 = chain kernels with fp32 products from a three-way bf16
                              split (TDMPC_PATH_CHAIN_X6), 7 = path 5 with those products, 8 = path 6 (the retired
                              64-row blocks), 9 = the persistent one-env plan
                              (plan1: one launch after the encoder), 10 = the wide step kernel (TDMPC_PATH_WIDE);
                              results agree within the fp32 tolerance */
    /* ABI 5: per-call state read from device memory at run time, so one captured hipGraph serves every value */
    const int32_t* warm_flags; /* optional device int32 [batch]: per-env warm start (tdmpc.py:124-125, `not t0`
                                  for that env with a previous mean); NULL = warm_start for every env */
    const float* std_floor_dev;/* optional device float scalar: self.std (tdmpc.py:148), which update() moves
                                  every step during std_schedule (tdmpc.py:196); NULL = std_floor */
    /* ABI 6 */
    int32_t* status;           /* optional device int32, sticky: a plan that failed on the device ORs a nonzero
                                  TDMPC_STATUS_* code into it (its action / metrics are NaN then). The caller zeroes
                                  it once and checks it at its next host sync; the reference cannot fail this way,
                                  so a nonzero status must be raised, never ignored. NULL = not reported. */
} tdmpc_plan_params;

/* tdmpc_plan_params.status bits */
#define TDMPC_STATUS_P1_TIMEOUT 1   /* the persistent one-env plan (path 9 / auto at batch 1) gave up at a hand-off:
                                       not every workgroup of its grid was resident (e.g. other work held CUs) */
#define TDMPC_STATUS_PACK_STALE 2   /* ABI 8: a tdmpc_pack_weights launch found another job table in `packed` than the
                                       one it was issued for (the buffer was re-allocated or zeroed at a recorded
                                       address without tdmpc_pack_forget and packed under capture, or a captured
                                       graph's pack replayed after the buffer was re-keyed): it packed nothing and
                                       poisoned the weights with NaN. Sticky in the packed buffer until the next
                                       uncaptured pack; tdmpc_plan, tdmpc_plan_icem and tdmpc_cem_iter OR it into
                                       their status word and return NaN actions / metrics. */

#define TDMPC_PATH_AUTO 0
#define TDMPC_PATH_LAYERED 1
#define TDMPC_PATH_CHAIN 2
#define TDMPC_PATH_CHAIN32 3
#define TDMPC_PATH_CHAIN16 4
#define TDMPC_PATH_SPLIT 5
#define TDMPC_PATH_CHAIN_X6 6   /* chain kernels, fp32 products from a three-way bf16 split (M = 512) */
#define TDMPC_PATH_SPLIT_X6 7   /* the split path (5) with the x6 products (M = 512) */
#define TDMPC_PATH_CHAIN64 8    /* retired (64-row x6 blocks measured no faster): runs path 6 */
#define TDMPC_PATH_PERSIST 9    /* one env: the whole plan after the encoder as ONE persistent launch (x6 products,
                                   weight-stationary; batch 1, M = 512, >= 256 CUs; the auto path's choice there);
                                   calls it does not apply to run the auto path */
#define TDMPC_PATH_WIDE 10      /* TOLD.next on the 128-row wide step kernel (x6, weights streamed once per workgroup
                                   through an LDS ring) at every width it supports, x6 chain kernels elsewhere;
                                   the auto path picks it for launches with >= one 128-row block per CU and head */

/* Byte sizes the caller must allocate (all 256-byte aligned). */
typedef struct tdmpc_sizes {
    size_t packed_weight_bytes;  /* packed TOLD parameter buffer (tdmpc_pack_weights) */
    size_t workspace_bytes;      /* scratch for one tdmpc_plan call at max dims */
    size_t noise_floats_per_env; /* floats of the per-env noise stream at max horizon / iterations */
} tdmpc_sizes;

/* Returns TDMPC_ABI_VERSION. */
int tdmpc_abi_version(void);

/* Fill `out` for `dims`. */
int tdmpc_sizes_for(const tdmpc_dims* dims, tdmpc_sizes* out);

/* Number of floats of the per-env noise stream for a call with horizon H and I iterations:
 *   H*P*A  (pre-rollout TruncatedNormal eps, tdmpc.py:117 / helper.py:88)
 * + I*(H*N*A + T*A)  (per CEM iteration: torch.randn(H,N,A) tdmpc.py:131, then pi eps at the horizon
 *                     tdmpc.py:91), T = N+P
 * + A  (final action noise, tdmpc.py:158)
 * laid out in exactly that (reference draw) order. */
size_t tdmpc_noise_floats(const tdmpc_dims* dims, int32_t horizon, int32_t iterations);

/* Fill the noise streams of `batch` envs (env e at noise + e*env_stride floats, layout above) with exactly the
 * values the reference's per-env draw sequence takes from torch's device Philox generator (tdmpc.py:117, 131, 91,
 * 158 -- each a separate normal_/randn launch there), in ONE launch: element li of a draw of n values is
 * component (li / S) % 4 of the (li / S / 4 + 1)-th normal4 of Philox subsequence li % S at the draw's counter
 * offset, S = 256 * min(grid_cap, ceil(n / 256)) (ATen's distribution_elementwise_grid_stride_kernel, block
 * 256, unroll 4). Draw k of env e starts at `offset` + the counter advance of every earlier draw;
 * `*offset_advance` receives the total the caller adds to the generator. grid_cap = CUs * (max threads per
 * CU / 256), as ATen's calc_execution_policy. eval_mode skips the final action draw. gen_state: NULL, or a device
 * pointer to {seed, offset} read by the kernel when it runs instead of `seed` / `offset` -- so one captured graph
 * serves every call: the host stages the generator's state into it before each replay. */
int tdmpc_reference_normals(const tdmpc_dims* dims, float* noise, int32_t batch, int64_t env_stride,
                            int32_t horizon, int32_t iterations, int32_t eval_mode, uint64_t seed, uint64_t offset,
                            const uint64_t* gen_state, int32_t grid_cap, uint64_t* offset_advance, void* stream);

/* Number of parameter tensors tdmpc_pack_weights expects: the reference state_dict order
 * (TOLD, tdmpc.py:9-23): _encoder.*, _dynamics.{0,2,4}.{weight,bias}, _reward.{0,2,4}.*, _pi.{0,2,4}.*,
 * _Q1.{0,1,3,4,6}.*, _Q2.{0,1,3,4,6}.*  (state encoder: 4 tensors, 6 with enc_norm -- 0.w 0.b 1.w 1.b 3.w
 * 3.b --; pixel encoder: 10). */
int tdmpc_num_param_tensors(const tdmpc_dims* dims);

/* Pack the TOLD parameters (device pointers, reference state_dict order, fp32, contiguous nn.Linear
 * [out,in] / Conv2d [out,in,kh,kw] layout) into `packed` (replaces TDMPC.model for planning). ONE kernel
 * launch enqueued on `stream`. Its job table lives in `packed` itself (no library-global device memory): every
 * call outside a stream capture uploads it with a header naming it (a nonce); a call inside a capture uploads
 * nothing and requires the same tensors as this buffer's last uncaptured pack (pack once before capturing).
 * The kernel checks the header's nonce against the table the call was issued for: a mismatch (a buffer
 * re-allocated or zeroed at a known address and packed first under capture, a replayed graph whose buffer was
 * re-keyed since) packs nothing, NaN-poisons the weights and raises TDMPC_STATUS_PACK_STALE, which the next plan
 * passes on -- never silently zero or stale weights. Once a capture has packed into `packed`, an uncaptured pack
 * from OTHER tensors returns TDMPC_E_DIMS until tdmpc_pack_forget(packed). Re-run whenever the parameters change
 * (after TDMPC.update -- the learner does so from its flat parameter buffer inside its update graph). When
 * allocated, `packed` must be zero-filled once (every tensor's region is rewritten whole, padding included, but
 * the alignment gaps between regions are not, and padded vector reads may touch them); announcing it with
 * tdmpc_pack_forget is good practice (a skipped call is caught by the nonce check, not silently wrong). */
int tdmpc_pack_weights(const tdmpc_dims* dims, const float* const* tensors, int32_t n_tensors,
                       void* packed, size_t packed_bytes, void* stream);

/* A packed buffer was (re)allocated or is re-keyed at `packed`: forget the job table the library last uploaded at
 * that address (and free its pinned staging buffer). The next uncaptured pack uploads a table with a new nonce;
 * graphs captured over the old table then fail loudly (TDMPC_STATUS_PACK_STALE) if replayed. Returns 0. */
int tdmpc_pack_forget(const void* packed);

/* Diagnostic, host only (no HIP call): bounds-checks tdmpc_pack_weights' job table for these dims, given the
 * element count of each of the n reference tensors (state_dict order). Returns the number of jobs, or
 * TDMPC_E_SIZE naming the first job that would write outside the layout or read outside its tensor. */
int tdmpc_debug_pack_check(const tdmpc_dims* d, const int64_t* numel, int32_t n);

/* TOLD.h for `batch` observations (tdmpc.py:115,121 / helper.enc). obs: state fp32 [batch, obs_dim]; pixels
 * uint8 [batch, C, S, S] if obs_is_u8 else fp32 of the same shape (raw 0..255 values, /255 inside).
 * z0: fp32 [batch, L]. */
int tdmpc_encode(const tdmpc_dims* dims, const void* packed, const void* obs, int32_t obs_is_u8,
                 int32_t batch, void* workspace, float* z0, void* stream);

/* One full TDMPC.plan for `params->batch` independent environments (tdmpc.py:94-163 minus the seed-step
 * branch, which needs no model):
 *   obs        [batch, obs...]        observation (fp32, or uint8 pixels when obs_is_u8)
 *   noise      [batch, tdmpc_noise_floats(H, I)]  per-env noise streams in reference draw order
 *   u          [batch] float64        the uniform numpy draws inside np.random.choice (tdmpc.py:153)
 *   prev_mean  [batch, H, A] in/out   self._prev_mean (read when warm_start, always written)
 *   action     [batch, A]      out    the planned action a (tdmpc.py:155-158)
 *   metrics    [batch, 2]      out    {external_reward_mean, current_std} (tdmpc.py:160)
 *   elite_out  [batch, H, K, A] out   optional (NULL ok): last iteration's elite actions
 *   score_out  [batch, K]      out    optional: last iteration's softmax scores
 *   value_out  [batch, I, T]   out    optional: every iteration's estimate_value output (tdmpc.py:137)
 *   mean_out / std_out [batch, I, H, A] out optional: CEM mean/std after each iteration (tdmpc.py:149) */
int tdmpc_plan(const tdmpc_dims* dims, const tdmpc_plan_params* params, const void* packed,
               const void* obs, int32_t obs_is_u8, const float* noise, const double* u,
               float* prev_mean, float* action, float* metrics,
               float* elite_out, float* score_out, float* value_out, float* mean_out, float* std_out,
               void* workspace, size_t workspace_bytes, void* stream);

/* ---- iCEM planner: TdICemSimMlp.plan, /root/reference/src/algorithm/
 * tdmpc_icem_similarity_mlp.py:160-265, on the planner's kernels (chain or layered, `path`). Per-iteration candidate counts shrink
 * (N_i = max(2K, int(N_{i-1} / factor))), a fraction of the elites is reused (shifted in time from the previous
 * plan in the first iteration, carried over from the previous iteration afterwards), the last iteration's
 * sample 0 is the CEM mean, and the sample noise is the caller's (white / pink / brown thirds, coloured noise
 * from the powerlaw-PSD generator, drawn in the reference's order). Row layout per env: [sampled | reused] at
 * rows [0, N_i + E_i), the P0 policy rollouts at rows [N + K, N + K + P0) (dims.num_pi is the largest P0). */
typedef struct tdmpc_icem_params {
    int32_t horizon, iterations, batch, warm_start, eval_mode;
    int32_t has_elites;       /* the elite buffer holds the previous plan's elites (hasattr(self, '_elite_actions')) */
    int32_t elite_horizon;    /* their horizon: H, or H - 1 right after the horizon schedule grew */
    int32_t n_pi0;            /* P0 = int(mixture_coef * num_samples): policy rollouts of the pre-rollout */
    int32_t path;             /* TDMPC_PATH_*: kernel family (auto: chain kernels only for wide launches) */
    int32_t n_samples[16];    /* N_i (n_samples[0] == dims.num_samples) */
    int32_t n_pi[16];         /* P_i = int(mixture_coef * N_i) */
    int32_t n_elite[16];      /* E_i reused elite trajectories (0 when none) */
    int64_t samp_off[16];     /* per-env noise offsets (floats): iteration i's sample noise [H][N_i][A] */
    int64_t term_off[16];     /*   iteration i's terminal policy noise [N_i + E_i + P_i][A] */
    int64_t reuse_off;        /*   the reused elites' fresh coloured sequence [H][E_0][A] (first iteration) */
    int64_t pi_off;           /*   the pre-rollout policy noise [H][P0][A] */
    int64_t act_off;          /*   the final action noise [A] */
    int64_t env_stride;       /* floats per env noise stream */
    float min_std, temperature, momentum, one_minus_momentum, std_floor, init_std;
    float discount_pow[17];
    int32_t* status;          /* ABI 8: optional device int32, sticky (tdmpc_plan_params.status) */
} tdmpc_icem_params;

/* Sizes for tdmpc_plan_icem (the workspace holds N + K + num_pi rows per env). */
int tdmpc_icem_sizes_for(const tdmpc_dims* dims, tdmpc_sizes* out);

/*   elites   [batch, max_horizon, K, A] in/out: the previous plan's elites (read when has_elites), then every
 *            iteration's (`self._elite_actions`)
 *   value_out [batch, iterations, N + K + num_pi] optional: iteration i's values of its T_i candidates
 *   other arguments as tdmpc_plan. */
int tdmpc_plan_icem(const tdmpc_dims* dims, const tdmpc_icem_params* params, const void* packed,
                    const void* obs, int32_t obs_is_u8, const float* noise, const double* u, float* prev_mean,
                    float* elites, float* action, float* metrics, float* value_out, float* mean_out,
                    float* std_out, void* workspace, size_t workspace_bytes, void* stream);

/* Building blocks of tdmpc_plan, exposed for unit parity tests (each is one part of the reference):
 * rollout values for explicit candidate action sequences -- TDMPC.estimate_value (tdmpc.py:83-92) for
 * `batch` envs with T rows each starting from z0[env]:
 *   actions   [batch, H, T, A]   candidate actions (rows 0..T-1)
 *   eps_term  [batch, T, A]      TruncatedNormal eps of the pi call at the horizon
 *   value     [batch, T] out     G after nan_to_num
 *   reward_last [batch, T] out   reward at t = H-1 (its mean is estimate_value's second output)
 *   z_last    [batch, T, L] out  optional: latent after H steps */
int tdmpc_estimate_value(const tdmpc_dims* dims, const tdmpc_plan_params* params, const void* packed,
                         const float* z0, const float* actions, const float* eps_term, int32_t rows,
                         float* value, float* reward_last, float* z_last,
                         void* workspace, size_t workspace_bytes, void* stream);

/* The policy pre-rollout of TDMPC.plan (tdmpc.py:113-118) for `batch` envs: z = z0 repeated P times, then for
 * t < H: pi_actions[t] = TOLD.pi(z, min_std) with the caller's TruncatedNormal eps, z = TOLD.next(z, .)[0]
 * (the last step's next is not computed: its latent is unused).
 *   z0         [batch, L]
 *   eps_pi     [batch, H, P, A]   _standard_normal draws of the H pi calls (P = dims.num_pi)
 *   pi_actions [batch, H, P, A] out */
int tdmpc_pi_rollout(const tdmpc_dims* dims, const tdmpc_plan_params* params, const void* packed,
                     const float* z0, const float* eps_pi, float* pi_actions,
                     void* workspace, size_t workspace_bytes, void* stream);

/* One CEM iteration of TDMPC.plan (tdmpc.py:127-149) for `batch` envs: candidates
 * clamp(mean + std * eps_cem, -1, 1) followed by the P pi_actions, estimate_value (nan_to_num), top-K, softmax
 * refit; mean = momentum * mean + (1 - momentum) * _mean, std = _std.clamp(std_floor, 2).
 *   z0            [batch, L]
 *   pi_actions    [batch, H, P, A]   (tdmpc_pi_rollout's output; NULL when P == 0)
 *   eps_cem       [batch, H, N, A]   the torch.randn draw of the candidates
 *   eps_term      [batch, T, A]      the horizon pi call's eps (T = N + P)
 *   mean, std     [batch, H, A] in/out
 *   elite_actions [batch, H, K, A] out   (elite order = torch.topk order)
 *   score         [batch, K] out
 *   value         [batch, T] out     optional: estimate_value's output for the T candidates
 *   reward_mean   [batch] out        estimate_value's mean reward at t = H-1 (external_reward_mean) */
int tdmpc_cem_iter(const tdmpc_dims* dims, const tdmpc_plan_params* params, const void* packed,
                   const float* z0, const float* pi_actions, const float* eps_cem, const float* eps_term,
                   float* mean, float* std, float* elite_actions, float* score, float* value, float* reward_mean,
                   void* workspace, size_t workspace_bytes, void* stream);

/* Diagnostic kernel timer for the roofline report (bench.py). Arms a per-thread recorder: every later
 * launch issued from this thread that matches is bracketed by HIP events on its stream (at most
 * max_launches).
 *   cfg 0..3: linear_kernel / linear_lds_kernel launches of tile configuration `cfg` (1 = latency 32x32,
 *     2 = latency 32x64, 3 = throughput LDS tile, 0 = any) and prologue `pro` (0 plain, 1 LayerNorm, -1 any),
 *     restricted to K == N == kdim when kdim > 0 (the hidden kdim x kdim layers);
 *   cfg 4 / 5 / 6: chain_kernel launches of the TOLD.next step / pi / Q heads;
 * in both cases restricted to launches over exactly `rows` rows when rows > 0 (e.g. batch * num_samples:
 * the CEM rollout). tdmpc_profile_end waits for the events and returns the launch count, the summed kernel
 * time in ms and the summed algorithmic FLOPs (2*M*N*K per GEMM problem; for a chain launch 2 * rows * the
 * head's MACs per row at the real, unpadded widths). Eager use only (events are not graph-capturable). */
int tdmpc_profile_begin(int32_t cfg, int32_t pro, int32_t kdim, int32_t rows, int32_t max_launches);
int tdmpc_profile_end(int32_t* launches, double* total_ms, double* flops);
/* Name of the kernel (and its template arguments) of the last launch the armed profiler timed, "" if none. */
const char* tdmpc_profile_kernel(void);

/* Diagnostic: persistent one-env plans (TDMPC_PATH_PERSIST) launched after this call record, for workgroups 0 and
 * 255, the 100 MHz realtime clock at every hand-off's arrival and release into `dev` (device, 2048 uint64:
 * [workgroup 0: 1024][workgroup 255: 1024], entry 2*k / 2*k + 1 for hand-off k). NULL turns it off. */
int tdmpc_debug_plan1_stamps(void* dev);

/* Last HIP error string seen by this thread (for diagnostics). */
const char* tdmpc_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* TDMPC_HIP_H */
