/*
 * tdmpc_replay.h -- C ABI of the GPU prioritized replay buffer in libtdmpc_hip.so.
 *
 * Replaces the sampling hot spot of the reference's `ReplayBuffer` (/root/reference/src/algorithm/
 * helper.py:434-534): `sample()` computes probs = p**alpha / sum on the device, then copies them to the host
 * for `np.random.choice(total, batch, p=probs, replace=not full)` (a device->host sync and an O(capacity)
 * float64 cumsum on the CPU every update), then gathers H+1-step windows with ~4(H+1) small indexing ops.
 * Here the whole sample -- probabilities, float64 cdf, numpy's choice algorithm (with and without
 * replacement), importance weights and the window gather -- is five stream-ordered kernels (six without
 * replacement) with no host round trip; `add`'s running-max priority (a `.item()` sync in the reference) is a device reduction.
 *
 * Conventions as in tdmpc_hip.h: device pointers owned by the caller, stream-ordered, no allocation or
 * synchronisation, 0 or a negative TDMPC_E* code (declared there).
 */
#ifndef TDMPC_REPLAY_H
#define TDMPC_REPLAY_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct tdmpc_replay_dims {
    int32_t modality;       /* 0 = state (fp32 observations), 1 = pixels (uint8 3-channel frames) */
    int32_t obs_dim;        /* state: observation width */
    int32_t img_hw;         /* pixels: frame height = width */
    int32_t frame_stack;    /* pixels: frames per stacked observation (cfg.frame_stack) */
    int32_t action_dim;
    int32_t episode_length; /* cfg.episode_length; capacity is a multiple of it */
    int32_t capacity;       /* min(cfg.train_steps, cfg.max_buffer_size) (helper.py:443) */
    int32_t horizon;        /* window steps: cfg.horizon (latent_plan=True, train.py:80) or cfg.env_horizon */
    int32_t batch_size;     /* cfg.batch_size, <= 1024 */
} tdmpc_replay_dims;

/* The buffer's storage (helper.py:448-455), caller-owned device tensors. */
typedef struct tdmpc_replay_store {
    const void* obs;        /* [capacity + 1, frame]: state fp32 [obs_dim]; pixels uint8 [3, S, S] */
    const void* last_obs;   /* [capacity / L, obs]: state fp32 [obs_dim]; pixels uint8 [3 * frame_stack, S, S] */
    const float* action;    /* [capacity, A] */
    const float* reward;    /* [capacity] */
    const float* priorities;/* [capacity] */
} tdmpc_replay_store;

/* Workspace bytes tdmpc_replay_sample / tdmpc_replay_add_priorities need (256-byte aligned). */
size_t tdmpc_replay_workspace_bytes(const tdmpc_replay_dims* dims);

/* helper.py:477-485: the priorities of the episode just written at [idx, idx + L): the running maximum
 * (over all of them when `full`, else over [0, idx); 1.0 for the very first episode), with the last
 * `horizon` transitions of the episode set to 0. The storage copies themselves are plain device copies. */
int tdmpc_replay_add_priorities(const tdmpc_replay_dims* dims, float* priorities, int32_t idx, int32_t full,
                                void* workspace, size_t workspace_bytes, void* stream);

/* helper.py:487-488: priorities[idxs[i]] = values[i] + eps for i < n; with duplicate indices the last
 * occurrence wins (sequential index_put_ semantics, as the reference on the CPU). O(n): three small launches
 * (64-bit atomicMax of a generation-tagged position per index, the winners write, the generation advances).
 * `workspace` is the buffer's workspace (tdmpc_replay_workspace_bytes), ZERO-FILLED by the caller once when it
 * is allocated; it carries the per-slot last-writer keys from call to call. */
int tdmpc_replay_update_priorities(const tdmpc_replay_dims* dims, float* priorities, const int64_t* idxs,
                                   const float* values, int32_t n, float eps, void* workspace,
                                   size_t workspace_bytes, void* stream);

/* helper.py:504-528 for `total` valid transitions (idx, or capacity when full):
 *   u        [n_u] float64 uniforms in [0, 1), consumed in numpy's order (replace: the first batch_size;
 *            without replacement (full): successive rounds of batch_size - found). Should the rounds need more
 *            than n_u, they continue on a deterministic hash stream seeded by u[n_u - 1] (*n_used > n_u tells)
 *   idxs     [B] int64 out, weights [B] out  ((total * probs[idx])**-beta / max)
 *   obs      [B, obs] fp32 out (pixels: [B, 3 * frame_stack, S, S] as float values 0..255)
 *   next_obs [H + 1, B, obs] out, action [H + 1, B, A] out, reward [H + 1, B] out
 *   probs_out [total] fp32 optional (NULL ok), n_used int32 optional (device): uniforms consumed, or -2 when
 *            fewer than batch_size entries have non-zero probability without replacement (numpy raises
 *            ValueError there; idxs is padded with 0 -- check *n_used). */
int tdmpc_replay_sample(const tdmpc_replay_dims* dims, const tdmpc_replay_store* store, int32_t total,
                        int32_t full, float alpha, float beta, const double* u, int32_t n_u, int64_t* idxs,
                        float* weights, float* obs, float* next_obs, float* action, float* reward,
                        float* probs_out, int32_t* n_used, void* workspace, size_t workspace_bytes,
                        void* stream);

#ifdef __cplusplus
}
#endif
#endif /* TDMPC_REPLAY_H */
