"""ORACLE -- test infrastructure only. CPU restatement of the reference's prioritized replay buffer.

Only `tests/` and `bench.py`'s CPU-baseline leg may import this module (as the checker / the timed CPU
path); the product (`tdmpc_amd.replay`) never does.

Restates `ReplayBuffer` of /root/reference/src/algorithm/helper.py:434-534 (snapshot 2025-01-17):
  * `add(episode)`             helper.py:467-485  storage writes; new priorities = the running max (1.0 for
                               the first episode), the last `horizon` transitions of the episode set to 0
  * `update_priorities`        helper.py:487-488  p[idxs] = priority + 1e-6
  * `_get_obs`                 helper.py:490-502  pixels: frame_stack frames back from idx, not crossing the
                               episode start
  * `sample()`                 helper.py:504-528  probs = p**alpha / sum (fp32, torch), np.random.choice
                               (replace = not full) with p=probs, IS weights (total * probs[idx])**-beta / max,
                               H+1 step windows, last next_obs from _last_obs at episode ends
with every uniform numpy's `np.random.choice` would draw taken from an explicit stream `u` (float64),
consumed in numpy's order: replace=True -> `random_sample(size)` once; replace=False -> rounds of
`random_sample(size - n_found)` (numpy/random/mtrand.pyx `RandomState.choice`). `choice` below restates that
algorithm on float64 cdf = cumsum(p) / cdf[-1] and searchsorted(side='right').

Pinning: tests/golden/make_replay_golden.py ran the reference ReplayBuffer in the build container (cfg.device
= 'cpu'; `Tensor.cuda` made a no-op for the pixel path) from fixed seeds and recorded its samples;
tests/test_replay.py checks this restatement against them (indices / windows bit-exact).
"""
from __future__ import annotations

import numpy as np
import torch


def choice(probs32: np.ndarray, size: int, replace: bool, u: np.ndarray):
    """np.random.choice(len(p), size, p=probs32, replace=replace) with numpy's uniforms taken from `u`.
    Returns (indices int64 [size], number of uniforms consumed)."""
    p = probs32.astype(np.float64)
    if replace:
        cdf = np.cumsum(p)
        cdf /= cdf[-1]
        x = u[:size]
        return cdf.searchsorted(x, side="right").astype(np.int64), size
    p = p.copy()
    found = np.zeros(size, dtype=np.int64)
    n_uniq, used = 0, 0
    while n_uniq < size:
        x = u[used:used + size - n_uniq]
        used += size - n_uniq
        if n_uniq > 0:
            p[found[:n_uniq]] = 0
        cdf = np.cumsum(p)
        cdf /= cdf[-1]
        new = cdf.searchsorted(x, side="right")
        _, first = np.unique(new, return_index=True)
        first.sort()
        new = new.take(first)
        found[n_uniq:n_uniq + new.size] = new
        n_uniq += new.size
    return found, used


class RefReplay:
    """cfg keys: modality, obs_shape, action_dim, episode_length, capacity, batch_size, horizon, per_alpha,
    per_beta, frame_stack (pixels)."""

    def __init__(self, cfg):
        self.cfg = cfg
        self.capacity = int(cfg.capacity)
        L = int(cfg.episode_length)
        pixels = cfg.modality == "pixels"
        dtype = torch.uint8 if pixels else torch.float32
        frame = (3, *cfg.obs_shape[-2:]) if pixels else tuple(cfg.obs_shape)
        self._obs = torch.zeros((self.capacity + 1, *frame), dtype=dtype)
        self._last_obs = torch.zeros((self.capacity // L, *cfg.obs_shape), dtype=dtype)
        self._action = torch.zeros((self.capacity, cfg.action_dim), dtype=torch.float32)
        self._reward = torch.zeros((self.capacity,), dtype=torch.float32)
        self._priorities = torch.ones((self.capacity,), dtype=torch.float32)
        self._eps = 1e-6
        self._full = False
        self.idx = 0

    def add(self, ep_obs, ep_action, ep_reward):
        cfg, L = self.cfg, int(self.cfg.episode_length)
        ep_obs = torch.as_tensor(ep_obs)
        self._obs[self.idx:self.idx + L] = ep_obs[:-1] if cfg.modality != "pixels" else ep_obs[:-1, -3:]
        self._last_obs[self.idx // L] = ep_obs[-1]
        self._action[self.idx:self.idx + L] = torch.as_tensor(ep_action)
        self._reward[self.idx:self.idx + L] = torch.as_tensor(ep_reward)
        if self._full:
            max_priority = self._priorities.max().item()
        else:
            max_priority = 1.0 if self.idx == 0 else self._priorities[:self.idx].max().item()
        mask = torch.arange(L) >= L - cfg.horizon
        new = torch.full((L,), max_priority)
        new[mask] = 0
        self._priorities[self.idx:self.idx + L] = new
        self.idx = (self.idx + L) % self.capacity
        self._full = self._full or self.idx == 0

    def update_priorities(self, idxs, priorities):
        self._priorities[torch.as_tensor(idxs)] = torch.as_tensor(priorities).reshape(-1) + self._eps

    def _get_obs(self, arr, idxs):
        cfg = self.cfg
        if cfg.modality != "pixels":
            return arr[idxs]
        B, L, fs = len(idxs), int(cfg.episode_length), int(cfg.frame_stack)
        obs = torch.empty((B, 3 * fs, *arr.shape[-2:]), dtype=arr.dtype)
        obs[:, -3:] = arr[idxs]
        _idxs = idxs.clone()
        mask = torch.ones_like(_idxs, dtype=torch.bool)
        for i in range(1, fs):
            mask[_idxs % L == 0] = False
            _idxs[mask] -= 1
            obs[:, -(i + 1) * 3:-i * 3] = arr[_idxs]
        return obs.float()

    def probs(self):
        pr = (self._priorities if self._full else self._priorities[:self.idx]) ** self.cfg.per_alpha
        return pr / pr.sum()

    def sample(self, u, probs=None):
        """u: float64 uniform stream (numpy order). probs: optional float32 probabilities to use instead of
        this restatement's own (to check a device sampler's choice given ITS probabilities)."""
        cfg = self.cfg
        if probs is None:
            probs = self.probs()
        probs = torch.as_tensor(probs, dtype=torch.float32)
        total = len(probs)
        idx_np, used = choice(probs.numpy(), int(cfg.batch_size), not self._full, np.asarray(u, dtype=np.float64))
        idxs = torch.from_numpy(idx_np)
        weights = (total * probs[idxs]) ** (-cfg.per_beta)
        weights /= weights.max()
        obs = self._get_obs(self._obs, idxs)
        H = int(cfg.horizon)
        nxt_shape = self._last_obs.shape[1:]
        next_obs = torch.empty((H + 1, len(idxs), *nxt_shape), dtype=obs.dtype)
        action = torch.empty((H + 1, len(idxs), cfg.action_dim), dtype=torch.float32)
        reward = torch.empty((H + 1, len(idxs)), dtype=torch.float32)
        for t in range(H + 1):
            _idxs = idxs + t
            next_obs[t] = self._get_obs(self._obs, _idxs + 1)
            action[t] = self._action[_idxs]
            reward[t] = self._reward[_idxs]
        mask = (_idxs + 1) % int(cfg.episode_length) == 0
        next_obs[-1, mask] = self._last_obs[_idxs[mask] // int(cfg.episode_length)].float()
        return obs, next_obs, action, reward.unsqueeze(2), idxs, weights, used
