"""`ReplayBuffer`: drop-in for the reference's prioritized replay buffer with device-side sampling.

Reference: `ReplayBuffer` in /root/reference/src/algorithm/helper.py:434-534 (constructed by
`src/train.py:80` as `ReplayBuffer(cfg, latent_plan=True)`). Same constructor, attributes (`capacity`,
`idx`, `_full`, `_obs`, `_last_obs`, `_action`, `_reward`, `_priorities`, `_eps`, `batch_size`, `horizon`),
`add(episode)` / `+=`, `update_priorities(idxs, priorities)` and `sample() -> (obs, next_obs, action,
reward, idxs, weights)` with the reference's shapes and dtypes. The storage lives on the GPU for both
modalities; `sample()` runs entirely in libtdmpc_hip.so (include/tdmpc_replay.h): no host round trip, no
`.item()` / `.cpu()` synchronisation (the reference syncs twice per sample and once per add).

Randomness: the reference draws np.random.choice's uniforms from numpy's global generator. Here they come
from torch's generator on the device (a float64 `uniform_()` buffer), consumed in numpy's order, so a
given uniform stream selects exactly numpy's indices (tests/test_replay.py) -- but the stream itself is not
numpy's. Pass `u=` to `sample` to supply it (parity tests).
"""
from __future__ import annotations

import ctypes as C
import warnings
from copy import deepcopy

import torch

from . import _lib


class ReplayBuffer:
    graph_safe = True   # sample() / update_priorities() are sync-free and capturable (tdmpc_amd.learner)

    def __init__(self, cfg, latent_plan: bool = False):
        self.cfg = deepcopy(cfg)
        self.device = torch.device(cfg.device)
        self.capacity = int(min(cfg.train_steps, cfg.max_buffer_size))
        L = int(cfg.episode_length)
        if self.capacity % L:
            raise ValueError("capacity must be a multiple of episode_length")
        pixels = cfg.modality != "state"
        dtype = torch.uint8 if pixels else torch.float32
        frame = (3, *cfg.obs_shape[-2:]) if pixels else tuple(cfg.obs_shape)
        dev = self.device
        self._obs = torch.empty((self.capacity + 1, *frame), dtype=dtype, device=dev)
        self._last_obs = torch.empty((self.capacity // L, *cfg.obs_shape), dtype=dtype, device=dev)
        self._action = torch.empty((self.capacity, cfg.action_dim), dtype=torch.float32, device=dev)
        self._reward = torch.empty((self.capacity,), dtype=torch.float32, device=dev)
        self._priorities = torch.ones((self.capacity,), dtype=torch.float32, device=dev)
        self._eps = 1e-6
        self._full = False
        self.idx = 0
        self.batch_size = int(cfg.batch_size)
        self.horizon = int(cfg.horizon if latent_plan else cfg.env_horizon)
        d = _lib.ReplayDims()
        d.modality = 1 if pixels else 0
        d.obs_dim = 0 if pixels else int(cfg.obs_shape[0])
        d.img_hw = int(cfg.obs_shape[-1]) if pixels else 0
        d.frame_stack = int(cfg.frame_stack) if pixels else 1
        d.action_dim = int(cfg.action_dim)
        d.episode_length = L
        d.capacity = self.capacity
        d.horizon = self.horizon
        d.batch_size = self.batch_size
        self._dims = d
        self._L = _lib.lib()
        ws = self._L.tdmpc_replay_workspace_bytes(C.byref(d))
        if ws == 0:
            raise ValueError("unsupported replay buffer dims")
        self._ws = torch.zeros(ws, dtype=torch.uint8, device=dev)   # zero-filled once (update_priorities' keys)
        B, H = self.batch_size, self.horizon
        obs_shape = tuple(cfg.obs_shape)
        self._out_idx = torch.empty(B, dtype=torch.int64, device=dev)
        self._out_w = torch.empty(B, dtype=torch.float32, device=dev)
        self._out_obs = torch.empty((B, *obs_shape), dtype=torch.float32, device=dev)
        self._out_next = torch.empty((H + 1, B, *obs_shape), dtype=torch.float32, device=dev)
        self._out_action = torch.empty((H + 1, B, cfg.action_dim), dtype=torch.float32, device=dev)
        self._out_reward = torch.empty((H + 1, B), dtype=torch.float32, device=dev)
        self._n_used = torch.zeros(1, dtype=torch.int32, device=dev)
        self._ubuf = torch.empty(4 * B, dtype=torch.float64, device=dev)
        self._store = _lib.ReplayStore(self._obs.data_ptr(), self._last_obs.data_ptr(), self._action.data_ptr(),
                                       self._reward.data_ptr(), self._priorities.data_ptr())
        self.last_probs = None

    def _stream(self):
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def __add__(self, episode):
        self.add(episode)
        return self

    def add(self, episode):
        """helper.py:467-485. `episode` has obs [L+1, *obs_shape], action [L, A], reward [L] (the reference
        `Episode`, or any object with those attributes)."""
        L = int(self.cfg.episode_length)
        obs = torch.as_tensor(episode.obs).to(self.device)
        self._obs[self.idx:self.idx + L] = obs[:-1] if self.cfg.modality == "state" else obs[:-1, -3:]
        self._last_obs[self.idx // L] = obs[-1]
        self._action[self.idx:self.idx + L] = torch.as_tensor(episode.action).to(self.device)
        self._reward[self.idx:self.idx + L] = torch.as_tensor(episode.reward).to(self.device)
        _lib.check(self._L.tdmpc_replay_add_priorities(
            C.byref(self._dims), C.c_void_p(self._priorities.data_ptr()), self.idx, int(self._full),
            C.c_void_p(self._ws.data_ptr()), self._ws.numel(), self._stream()), "tdmpc_replay_add_priorities")
        self.idx = (self.idx + L) % self.capacity
        self._full = self._full or self.idx == 0

    def update_priorities(self, idxs, priorities):
        """helper.py:487-488: p[idxs] = priorities + 1e-6."""
        idxs = torch.as_tensor(idxs).to(self.device, torch.int64).contiguous().view(-1)
        vals = torch.as_tensor(priorities).to(self.device, torch.float32).contiguous().view(-1)
        if vals.numel() != idxs.numel():
            raise ValueError("priorities and idxs differ in length")
        _lib.check(self._L.tdmpc_replay_update_priorities(
            C.byref(self._dims), C.c_void_p(self._priorities.data_ptr()), C.c_void_p(idxs.data_ptr()),
            C.c_void_p(vals.data_ptr()), idxs.numel(), C.c_float(self._eps), C.c_void_p(self._ws.data_ptr()),
            self._ws.numel(), self._stream()), "tdmpc_replay_update_priorities")
        self._keep_upd = (idxs, vals)   # read asynchronously by the kernels

    def sample(self, u=None, keep_probs: bool = False):
        """helper.py:504-528 -> (obs, next_obs, action, reward [H+1, B, 1], idxs, weights). The returned
        tensors are this buffer's output buffers (overwritten by the next sample)."""
        cfg, B = self.cfg, self.batch_size
        total = self.capacity if self._full else self.idx
        if total <= 0:
            raise RuntimeError("sample() on an empty buffer")
        if u is None:
            u = self._ubuf.uniform_()
            self._n_u_last = None   # own draws: no caller stream whose numpy draw could be departed from
        else:
            u = torch.as_tensor(u, dtype=torch.float64).to(self.device).contiguous()
            self._n_u_last = u.numel()
        probs = torch.empty(total, dtype=torch.float32, device=self.device) if keep_probs else None
        _lib.check(self._L.tdmpc_replay_sample(
            C.byref(self._dims), C.byref(self._store), total, int(self._full), C.c_float(cfg.per_alpha),
            C.c_float(cfg.per_beta), C.c_void_p(u.data_ptr()), u.numel(), C.c_void_p(self._out_idx.data_ptr()),
            C.c_void_p(self._out_w.data_ptr()), C.c_void_p(self._out_obs.data_ptr()),
            C.c_void_p(self._out_next.data_ptr()), C.c_void_p(self._out_action.data_ptr()),
            C.c_void_p(self._out_reward.data_ptr()), C.c_void_p(_lib.ptr(probs)),
            C.c_void_p(self._n_used.data_ptr()), C.c_void_p(self._ws.data_ptr()), self._ws.numel(),
            self._stream()), "tdmpc_replay_sample")
        self._u_keep = u   # the kernels read it asynchronously
        self.last_probs = probs
        return (self._out_obs, self._out_next, self._out_action, self._out_reward.unsqueeze(2), self._out_idx,
                self._out_w)

    @property
    def uniforms_used(self) -> int:
        """Uniforms the last sample consumed (> the supplied count: the rounds continued on the hash stream;
        -2: fewer than batch_size non-zero priorities without replacement). Synchronises."""
        return int(self._n_used.item())

    def check_sample(self):
        """Raise like the reference's np.random.choice(replace=False) when the last sample could not find
        batch_size distinct non-zero-probability transitions (device flag; synchronises). Warn when numpy's
        rounds needed more uniforms than were supplied: the kernel then continued on its own hash stream, so
        the draw is still a valid without-replacement sample but no longer numpy's for the supplied stream."""
        used = self.uniforms_used
        if used == -2:
            raise ValueError("Fewer non-zero entries in p than size")
        n_u = getattr(self, "_n_u_last", None)
        if n_u is not None and used > n_u:
            warnings.warn(f"replay sample consumed {used} uniforms, {n_u} supplied: the rounds past the supplied "
                          "stream used the kernel's hash stream (not numpy's draw for this stream)", RuntimeWarning)
        return used
