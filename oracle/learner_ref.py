"""ORACLE -- test infrastructure only. CPU restatement of the reference learner.

Only `tests/` and `bench.py`'s CPU-baseline leg may import this module; the product (`tdmpc_amd.learner`)
never does.

Restates, on CPU torch with the same ATen ops in the same order (functional forms of the TOLD heads over a
dict of leaf tensors in state_dict order):
  * `TDMPC.update`      /root/reference/src/algorithm/tdmpc.py:192-245  (losses, clamp, IS-weighted mean --
                        including its [B, 1] x [B] -> [B, B] broadcast --, the 1/H gradient hook, grad-norm
                        clipping, Adam, the new priorities, update_pi, EMA every update_freq steps)
  * `TDMPC._td_target`  tdmpc.py:184-190  (online encoder and pi, target Q)
  * `TDMPC.update_pi`   tdmpc.py:165-182  (Q gradients off, rho-weighted -min(Q) over the latent rollout)
  * `helper.mse / l1 / ema`  helper.py:19-26, 48-52; `TruncatedNormal.sample`  helper.py:71-96
Random numbers: torch's global generator in the reference's order (per horizon step one TruncatedNormal draw
[B, A] in `_td_target`, then H+1 in `update_pi`), so on the CPU it reproduces the reference from the same seed.

Pinning: tests/golden/make_learner_golden.py ran the reference `TDMPC.update` here (two updates, EMA on the
second); tests/test_learner.py requires this restatement to match it bit for bit.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F


def _lin(p, x, name):
    return F.linear(x, p[name + ".weight"], p[name + ".bias"])


def _mlp(p, x, pre):
    x = F.elu(_lin(p, x, pre + ".0"))
    x = F.elu(_lin(p, x, pre + ".2"))
    return _lin(p, x, pre + ".4")


def _q(p, x, pre, m):
    x = _lin(p, x, pre + ".0")
    x = torch.tanh(F.layer_norm(x, (m,), p[pre + ".1.weight"], p[pre + ".1.bias"], 1e-5))
    x = _lin(p, x, pre + ".3")
    x = F.elu(F.layer_norm(x, (m,), p[pre + ".4.weight"], p[pre + ".4.bias"], 1e-5))
    return _lin(p, x, pre + ".6")


def h(p, cfg, obs):
    if cfg.modality == "pixels":
        x = obs.div(255.)
        for i in (1, 3, 5, 7):
            x = F.relu(F.conv2d(x, p[f"_encoder.{i}.weight"], p[f"_encoder.{i}.bias"], stride=2))
        return _lin(p, x.view(x.size(0), -1), "_encoder.10")
    return _lin(p, F.elu(_lin(p, obs, "_encoder.0")), "_encoder.2")


def nxt(p, z, a):
    x = torch.cat([z, a], dim=-1)
    return _mlp(p, x, "_dynamics"), _mlp(p, x, "_reward")


def Q(p, cfg, z, a):
    x = torch.cat([z, a], dim=-1)
    return _q(p, x, "_Q1", cfg.mlp_dim), _q(p, x, "_Q2", cfg.mlp_dim)


def pi(p, z, std):
    mu = torch.tanh(_mlp(p, z, "_pi"))
    if std > 0:
        scale = torch.ones_like(mu) * std
        eps = torch.empty(mu.shape, dtype=mu.dtype, device=mu.device).normal_()
        eps *= scale
        eps = torch.clamp(eps, -0.3, 0.3)
        x = mu + eps
        clamped = torch.clamp(x, -1.0 + 1e-6, 1.0 - 1e-6)
        return x - x.detach() + clamped.detach()
    return mu



def _clip_grad_norm_19(params, max_norm):
    """torch 1.9's clip_grad_norm_ (the reference pins pytorch=1.9, environment.yaml:6; called at tdmpc.py:178, 228):
    total = ||stack(||g||)||, clip_coef = max_norm / (total + 1e-6), grads scaled only `if clip_coef < 1` (a NaN norm
    scales nothing). The norm is reduced as the installed torch's clip_grad_norm_ reduces it (_foreach_norm per tensor,
    then the norm of their stack), so finite norms stay bitwise equal to the reference-generated fixtures."""
    grads = [p.grad for p in params if p.grad is not None]
    total = torch.linalg.vector_norm(torch.stack(torch._foreach_norm([g.detach() for g in grads], 2.0)), 2.0)
    clip_coef = max_norm / (total + 1e-6)
    if clip_coef < 1:
        for g in grads:
            g.detach().mul_(clip_coef)
    return total

class RefLearner:
    """model / target parameters as leaf tensors in state_dict order; Adam like the reference (tdmpc.py:62-63)."""

    def __init__(self, cfg, sd_model, sd_target):
        self.cfg = cfg
        self.p = {k: v.detach().clone().float().requires_grad_(True) for k, v in sd_model.items()}
        self.pt = {k: v.detach().clone().float() for k, v in sd_target.items()}
        self.params = list(self.p.values())
        self.pi_params = [v for k, v in self.p.items() if k.startswith("_pi.")]
        self.q_params = [v for k, v in self.p.items() if k.startswith("_Q1.") or k.startswith("_Q2.")]
        self.optim = torch.optim.Adam(self.params, lr=cfg.lr)
        self.pi_optim = torch.optim.Adam(self.pi_params, lr=cfg.lr)

    @torch.no_grad()
    def _td_target(self, next_obs, reward):
        cfg = self.cfg
        next_z = h(self.p, cfg, next_obs)
        return reward + cfg.discount * torch.min(*Q(self.pt, cfg, next_z, pi(self.p, next_z, cfg.min_std)))

    def update_pi(self, zs):
        cfg = self.cfg
        self.pi_optim.zero_grad(set_to_none=True)
        for v in self.q_params:
            v.requires_grad_(False)
        pi_loss = 0
        for t, z in enumerate(zs):
            a = pi(self.p, z, cfg.min_std)
            q = torch.min(*Q(self.p, cfg, z, a))
            pi_loss += -q.mean() * (cfg.rho ** t)
        pi_loss.backward()
        _clip_grad_norm_19(self.pi_params, cfg.grad_clip_norm)
        self.pi_optim.step()
        for v in self.q_params:
            v.requires_grad_(True)
        return pi_loss.item()

    def update(self, batch, step):
        """One reference `TDMPC.update` on a sampled batch -> (metrics dict, new priorities [B, 1])."""
        cfg = self.cfg
        obs, next_obses, action, reward, idxs, weights = batch
        self.optim.zero_grad(set_to_none=True)
        z = h(self.p, cfg, obs)
        zs = [z.detach()]
        consistency_loss, reward_loss, value_loss, priority_loss = 0, 0, 0, 0
        for t in range(cfg.horizon):
            Q1, Q2 = Q(self.p, cfg, z, action[t])
            z, reward_pred = nxt(self.p, z, action[t])
            with torch.no_grad():
                next_obs = next_obses[t]
                next_z = h(self.pt, cfg, next_obs)
                td_target = self._td_target(next_obs, reward[t])
            zs.append(z.detach())
            rho = cfg.rho ** t
            consistency_loss += rho * torch.mean(F.mse_loss(z, next_z, reduction="none"), dim=1, keepdim=True)
            reward_loss += rho * F.mse_loss(reward_pred, reward[t], reduction="none")
            value_loss += rho * (F.mse_loss(Q1, td_target, reduction="none") + F.mse_loss(Q2, td_target, reduction="none"))
            priority_loss += rho * (F.l1_loss(Q1, td_target, reduction="none") + F.l1_loss(Q2, td_target, reduction="none"))
        total_loss = cfg.consistency_coef * consistency_loss.clamp(max=1e4) + \
            cfg.reward_coef * reward_loss.clamp(max=1e4) + \
            cfg.value_coef * value_loss.clamp(max=1e4)
        weighted_loss = (total_loss * weights).mean()
        weighted_loss.register_hook(lambda grad: grad * (1 / cfg.horizon))
        weighted_loss.backward()
        grad_norm = _clip_grad_norm_19(self.params, cfg.grad_clip_norm)
        self.optim.step()
        new_prio = priority_loss.clamp(max=1e4).detach()
        pi_loss = self.update_pi(zs)
        if step % cfg.update_freq == 0:
            with torch.no_grad():
                for k, v in self.p.items():
                    self.pt[k].lerp_(v, cfg.tau)
        return {"consistency_loss": float(consistency_loss.mean().item()),
                "reward_loss": float(reward_loss.mean().item()),
                "value_loss": float(value_loss.mean().item()),
                "pi_loss": pi_loss,
                "total_loss": float(total_loss.mean().item()),
                "weighted_loss": float(weighted_loss.mean().item()),
                "grad_norm": float(grad_norm)}, new_prio

    def state_dicts(self):
        return {k: v.detach() for k, v in self.p.items()}, dict(self.pt)


def random_shift(x: np.ndarray, shift: np.ndarray, pad: int) -> np.ndarray:
    """RandomShiftsAug's arithmetic (helper.py:262-283) restated: replicate-pad by `pad`, then sample the padded
    frame at base_grid + shift. linspace(-1 + 1/n, 1 - 1/n, n)[:h] unnormalises (align_corners=False) to the pixel
    centres 0..h-1 and shift s * 2/n to s pixels, so the bilinear sample is the padded pixel (i + s_y, j + s_x).
    The reference evaluates those coordinates in fp32 and lands within ~1e-5 px of them (its output blends that
    much of a neighbour: <= 2.5e-3 on 0..255 frames, tests/test_learner.py against its recorded outputs).
    x: [n, c, h, w] float32; shift: [n, 2] integers (x, y)."""
    n, c, h, w = x.shape
    xp = np.pad(x, ((0, 0), (0, 0), (pad, pad), (pad, pad)), mode="edge")
    out = np.empty_like(x)
    for k in range(n):
        sx, sy = int(shift[k, 0]), int(shift[k, 1])
        out[k] = xp[k, :, sy:sy + h, sx:sx + w]
    return out
