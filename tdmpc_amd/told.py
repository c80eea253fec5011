"""TOLD parameter container with the reference's module tree and state_dict key names.

Reference: `TOLD` in `src/algorithm/tdmpc.py:9-50`, built from `helper.enc` (`helper.py:119-133`),
`helper.mlp` (`helper.py:169-176`) and `helper.q` (`helper.py:197-201`).

The module exists so that a reference checkpoint (`{'model': sd, 'model_target': sd}`, `tdmpc.py:68-81`)
loads with `load_state_dict` unchanged and so that `TDMPC.model` exposes the same attributes. Planning does
NOT run these modules: `TDMPC.plan` packs the parameters into one device buffer and runs the HIP kernels.
The `forward`-style helpers (`h`, `next`, `pi`, `Q`) are what the learner (tdmpc_amd.learner) differentiates.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn


def _enc(cfg, enc_norm=False) -> nn.Sequential:
    if cfg.modality == "pixels":
        c = int(3 * cfg.frame_stack)
        nc = cfg.num_channels
        layers = [nn.Identity(),  # NormalizeImg (x/255) is parameter-free; index 0 like the reference
                  nn.Conv2d(c, nc, 7, stride=2), nn.ReLU(),
                  nn.Conv2d(nc, nc, 5, stride=2), nn.ReLU(),
                  nn.Conv2d(nc, nc, 3, stride=2), nn.ReLU(),
                  nn.Conv2d(nc, nc, 3, stride=2), nn.ReLU()]
        s = cfg.img_size
        for k in (7, 5, 3, 3):
            s = (s - k) // 2 + 1
        # the reference sizes the flatten by running the convs on torch.randn(C, S, S) (helper.py:28-31,
        # :129): draw (and drop) the same tensor so the default init of the layers built after it consumes
        # torch's generator exactly as in the reference (seeded inits then agree bit for bit)
        torch.randn(c, cfg.img_size, cfg.img_size)
        layers += [nn.Flatten(), nn.Linear(nc * s * s, cfg.latent_dim)]
        return nn.Sequential(*layers)
    if enc_norm:
        # helper.dmlab_enc_norm for state observations with norm_type 'ln' (helper.py:156-166, the iCEM agent's
        # encoder): Linear, LayerNorm, ELU, Linear -- keys _encoder.{0,1,3}
        return nn.Sequential(nn.Linear(cfg.obs_shape[0], cfg.enc_dim), nn.LayerNorm(cfg.enc_dim), nn.ELU(),
                             nn.Linear(cfg.enc_dim, cfg.latent_dim))
    return nn.Sequential(nn.Linear(cfg.obs_shape[0], cfg.enc_dim), nn.ELU(),
                         nn.Linear(cfg.enc_dim, cfg.latent_dim))


def _mlp(in_dim, mlp_dim, out_dim) -> nn.Sequential:
    return nn.Sequential(nn.Linear(in_dim, mlp_dim), nn.ELU(),
                         nn.Linear(mlp_dim, mlp_dim), nn.ELU(),
                         nn.Linear(mlp_dim, out_dim))


def _q(cfg) -> nn.Sequential:
    m = cfg.mlp_dim
    return nn.Sequential(nn.Linear(cfg.latent_dim + cfg.action_dim, m), nn.LayerNorm(m), nn.Tanh(),
                         nn.Linear(m, m), nn.LayerNorm(m), nn.ELU(),
                         nn.Linear(m, 1))


def pixel_enc_out_hw(cfg) -> int:
    s = cfg.img_size
    for k in (7, 5, 3, 3):
        s = (s - k) // 2 + 1
    return s


class TOLD(nn.Module):
    """Task-Oriented Latent Dynamics: encoder h, dynamics d, reward R, policy pi, twin Q."""

    def __init__(self, cfg, init: str = "reference", enc_norm: bool = False):
        super().__init__()
        self.cfg = cfg
        self._encoder = _enc(cfg, enc_norm)
        self._dynamics = _mlp(cfg.latent_dim + cfg.action_dim, cfg.mlp_dim, cfg.latent_dim)
        self._reward = _mlp(cfg.latent_dim + cfg.action_dim, cfg.mlp_dim, 1)
        self._pi = _mlp(cfg.latent_dim, cfg.mlp_dim, cfg.action_dim)
        self._Q1, self._Q2 = _q(cfg), _q(cfg)
        if init == "reference":
            # tdmpc.py:20-23: orthogonal init (helper.py:35-45), then zero the last layer of R, Q1, Q2.
            self.apply(_orthogonal_init)
            for m in (self._reward, self._Q1, self._Q2):
                m[-1].weight.data.fill_(0)
                m[-1].bias.data.fill_(0)

    def track_q_grad(self, enable=True):
        """tdmpc.py:25-28 (helper.set_requires_grad on Q1, Q2)."""
        for m in (self._Q1, self._Q2):
            for p in m.parameters():
                p.requires_grad_(enable)

    # Eager forms of the heads (tdmpc.py:30-50): the learner (tdmpc_amd/learner.py) differentiates through
    # them; the HIP planner does not use them.
    def h(self, obs):
        if self.cfg.modality == "pixels":
            obs = obs / 255.0
        return self._encoder(obs)

    def next(self, z, a):
        x = torch.cat([z, a], dim=-1)
        return self._dynamics(x), self._reward(x)

    def Q(self, z, a):
        x = torch.cat([z, a], dim=-1)
        return self._Q1(x), self._Q2(x)

    def pi(self, z, std=0, eps=None):
        """tdmpc.py:39-45: tanh(pi(z)), plus a TruncatedNormal(mu, std).sample(clip=0.3) when std > 0
        (`eps`: the N(0, 1) draw to use instead of drawing one -- parity tests)."""
        mu = torch.tanh(self._pi(z))
        if std > 0:
            return truncated_normal_sample(mu, torch.ones_like(mu) * std, clip=0.3, noise=eps)
        return mu


def truncated_normal_sample(loc, scale, clip=None, low=-1.0, high=1.0, eps=1e-6, noise=None):
    """helper.TruncatedNormal.sample (helper.py:71-96): eps ~ N(0, 1) drawn like torch.distributions'
    `_standard_normal` (an empty tensor filled by normal_), scaled, clipped to +-clip, added to loc, then
    clamped to (low + eps, high - eps) with a straight-through gradient."""
    if noise is None:
        noise = torch.empty(loc.shape, dtype=loc.dtype, device=loc.device).normal_()
    else:
        noise = noise.to(loc.device, loc.dtype).clone()
    noise *= scale
    if clip is not None:
        noise = torch.clamp(noise, -clip, clip)
    x = loc + noise
    clamped = torch.clamp(x, low + eps, high - eps)
    return x - x.detach() + clamped.detach()


def _orthogonal_init(m):
    if isinstance(m, nn.Linear):
        nn.init.orthogonal_(m.weight.data)
        if m.bias is not None:
            nn.init.zeros_(m.bias)
    elif isinstance(m, nn.Conv2d):
        nn.init.orthogonal_(m.weight.data, nn.init.calculate_gain("relu"))
        if m.bias is not None:
            nn.init.zeros_(m.bias)


def synthetic_state_dict(cfg, seed: int = 0, enc_norm: bool = False) -> dict:
    """Deterministic non-degenerate TOLD weights (BASELINE.md "Inputs"): every tensor of the reference
    state_dict drawn from `np.random.RandomState(seed + i)` in key order. Linear/conv weights are
    N(0, 1/fan_in) -- including the last layers of R/Q1/Q2, which the reference zero-inits and which would
    make every candidate's value identical (SURVEY.md §5 "Zero-init makes values degenerate"). Biases are
    N(0, 0.05^2); LayerNorm gains 1 + N(0, 0.1^2), shifts N(0, 0.1^2)."""
    model = TOLD(cfg, init="none", enc_norm=enc_norm)
    sd = {}
    for i, (k, v) in enumerate(model.state_dict().items()):
        rs = np.random.RandomState(seed * 1000 + i)
        shape = tuple(v.shape)
        is_ln = any(k.startswith(f"_Q{j}.{li}.") for j in (1, 2) for li in (1, 4)) or (
            enc_norm and k.startswith("_encoder.1."))
        if is_ln and k.endswith("weight"):
            arr = 1.0 + 0.1 * rs.standard_normal(shape)
        elif is_ln:
            arr = 0.1 * rs.standard_normal(shape)
        elif k.endswith("weight"):
            fan_in = int(np.prod(shape[1:]))
            arr = rs.standard_normal(shape) / np.sqrt(fan_in)
        else:
            arr = 0.05 * rs.standard_normal(shape)
        sd[k] = torch.from_numpy(arr.astype(np.float32))
    return sd
