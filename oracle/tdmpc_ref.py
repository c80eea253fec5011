"""ORACLE -- test infrastructure only. CPU restatement of the reference planner.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import this module, and
only as the checker / the timed CPU baseline. The product path (`tdmpc_amd`) never imports it: the HIP
planner fails loudly when its extension is missing.

What it restates (reference `/root/reference`, snapshot 2025-01-17):
  * `TOLD.h / next / pi / Q`          src/algorithm/tdmpc.py:30-50
  * `helper.mlp / q / enc`            src/algorithm/helper.py:119-133, 169-176, 197-201
  * `TruncatedNormal.sample(clip)`    src/algorithm/helper.py:71-96
  * `TDMPC.estimate_value`            src/algorithm/tdmpc.py:83-92
  * `TDMPC.plan`                      src/algorithm/tdmpc.py:94-163
with every random draw taken from an explicit `NoiseBundle` instead of the global generators.
`draw_noise` reproduces the reference's draw order on the torch / numpy global generators (SURVEY.md §8a
A10), so `plan(..., draw_noise(...))` equals the reference `plan()` run from the same seeds.

Pinning: tests/golden/make_golden.py imported the reference itself in the build container (shims: a stub
`rlpyt` module, a no-op `Module.cuda`, a namespace cfg) and recorded its outputs; tests/test_oracle.py checks
this restatement against those fixtures (bit-exact: same ATen CPU ops in the same order).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional

import numpy as np
import torch
import torch.nn.functional as F


# ----------------------------------------------------------------------------- schedule
def linear_schedule(schdl, step):
    """helper.py:639-652."""
    import re
    try:
        return float(schdl)
    except (TypeError, ValueError):
        m = re.match(r"linear\((.+),(.+),(.+),(.+)\)", schdl)
        if m:
            init, final, duration, start = [float(g) for g in m.groups()]
            mix = np.clip((step - start) / duration, 0.0, 1.0)
            return (1.0 - mix) * init + mix * final
    raise NotImplementedError(schdl)


# ----------------------------------------------------------------------------- noise
@dataclass
class NoiseBundle:
    """Every random number one `plan()` call consumes, in reference draw order."""
    eps_pi: Optional[torch.Tensor]          # [H, P, A]  H x normal_([P,A])   (TruncatedNormal in pre-rollout)
    eps_cem: list = field(default_factory=list)   # I x [H, N, A]  torch.randn(H, N, A)
    eps_term: list = field(default_factory=list)  # I x [T, A]     normal_([T,A]) (pi at the horizon)
    u: float = 0.0                          # numpy random_sample() inside np.random.choice
    eps_act: Optional[torch.Tensor] = None  # [A] torch.randn(A) (train mode only)
    seed_action: Optional[torch.Tensor] = None  # [A] uniform_(-1,1) (seed-step branch only)


def plan_horizon(cfg, step):
    return int(min(cfg.horizon, linear_schedule(cfg.horizon_schedule, step)))


def draw_noise(cfg, step, eval_mode=False, device="cpu") -> NoiseBundle:
    """Draw from torch's / numpy's global generators exactly as `TDMPC.plan` does."""
    A = cfg.action_dim
    if step < cfg.seed_steps and not eval_mode:
        return NoiseBundle(eps_pi=None, seed_action=torch.empty(A, dtype=torch.float32,
                                                                 device=device).uniform_(-1, 1))
    H = plan_horizon(cfg, step)
    N = cfg.num_samples
    P = int(cfg.mixture_coef * N)
    T = N + P
    nb = NoiseBundle(eps_pi=None)
    if P > 0:
        nb.eps_pi = torch.stack([torch.empty(P, A, device=device).normal_() for _ in range(H)])
    for _ in range(cfg.iterations):
        nb.eps_cem.append(torch.randn(H, N, A, device=device))
        nb.eps_term.append(torch.empty(T if P > 0 else N, A, device=device).normal_())
    nb.u = float(np.random.random_sample())
    if not eval_mode:
        nb.eps_act = torch.randn(A, device=device)
    return nb


# ----------------------------------------------------------------------------- TOLD heads
class RefTOLD:
    """Functional TOLD over a reference-layout state_dict (fp32, CPU)."""

    def __init__(self, sd: dict, cfg):
        self.sd = {k: v.detach().to("cpu", torch.float32) for k, v in sd.items()}
        self.cfg = cfg

    def _lin(self, x, name):
        return F.linear(x, self.sd[name + ".weight"], self.sd[name + ".bias"])

    def _mlp(self, x, pre):
        x = F.elu(self._lin(x, pre + ".0"))
        x = F.elu(self._lin(x, pre + ".2"))
        return self._lin(x, pre + ".4")

    def _q(self, x, pre):
        m = self.cfg.mlp_dim
        x = self._lin(x, pre + ".0")
        x = torch.tanh(F.layer_norm(x, (m,), self.sd[pre + ".1.weight"], self.sd[pre + ".1.bias"], 1e-5))
        x = self._lin(x, pre + ".3")
        x = F.elu(F.layer_norm(x, (m,), self.sd[pre + ".4.weight"], self.sd[pre + ".4.bias"], 1e-5))
        return self._lin(x, pre + ".6")

    def h(self, obs):
        """helper.enc (helper.py:119-133)."""
        if self.cfg.modality == "pixels":
            x = obs.div(255.)
            for i in (1, 3, 5, 7):
                x = F.relu(F.conv2d(x, self.sd[f"_encoder.{i}.weight"], self.sd[f"_encoder.{i}.bias"], stride=2))
            x = x.view(x.size(0), -1)
            return self._lin(x, "_encoder.10")
        x = self._lin(obs, "_encoder.0")
        if "_encoder.3.weight" in self.sd:
            # helper.dmlab_enc_norm, state, norm_type 'ln' (helper.py:156-166): Linear, LayerNorm, ELU, Linear
            x = F.layer_norm(x, (x.shape[-1],), self.sd["_encoder.1.weight"], self.sd["_encoder.1.bias"], 1e-5)
            return self._lin(F.elu(x), "_encoder.3")
        return self._lin(F.elu(x), "_encoder.2")

    def next(self, z, a):
        x = torch.cat([z, a], dim=-1)
        return self._mlp(x, "_dynamics"), self._mlp(x, "_reward")

    def pi_mu(self, z):
        return torch.tanh(self._mlp(z, "_pi"))

    def pi(self, z, std, eps):
        """TOLD.pi + TruncatedNormal(mu, std).sample(clip=0.3) with eps supplied (helper.py:86-96)."""
        mu = self.pi_mu(z)
        if std > 0:
            scale = torch.ones_like(mu) * std
            eps = eps.clone()
            eps *= scale
            eps = torch.clamp(eps, -0.3, 0.3)
            x = mu + eps
            clamped = torch.clamp(x, -1.0 + 1e-6, 1.0 - 1e-6)
            return x - x.detach() + clamped.detach()
        return mu

    def Q(self, z, a):
        x = torch.cat([z, a], dim=-1)
        return self._q(x, "_Q1"), self._q(x, "_Q2")


# ----------------------------------------------------------------------------- planner
class PlanState:
    """Mutable planner state the reference keeps on `self`: `_prev_mean` and `std` (tdmpc.py:59,154,196)."""

    def __init__(self, std):
        self.std = std
        self.prev_mean = None


@torch.no_grad()
def estimate_value(told, cfg, z, actions, horizon, eps_term, trace=None):
    """tdmpc.py:83-92."""
    G, discount = 0, 1
    for t in range(horizon):
        z, reward = told.next(z, actions[t])
        G += discount * reward
        discount *= cfg.discount
    q1, q2 = told.Q(z, told.pi(z, cfg.min_std, eps_term))
    G += discount * torch.min(q1, q2)
    if trace is not None:
        trace.setdefault("q1", []).append(q1.clone())
        trace.setdefault("q2", []).append(q2.clone())
        trace.setdefault("z_H", []).append(z.clone())
    return G.nan_to_num_(0), float(reward.mean().item())


@torch.no_grad()
def plan(told: RefTOLD, cfg, state: PlanState, obs, noise: NoiseBundle, eval_mode=False, step=None,
         t0=True, trace: Optional[dict] = None):
    """tdmpc.py:94-163 with explicit noise. Returns (action[A], metrics dict)."""
    plan_metrics = {"external_reward_mean": 0.0, "current_std": 0.0}
    if step < cfg.seed_steps and not eval_mode:
        return noise.seed_action.clone(), plan_metrics

    obs = torch.tensor(np.asarray(obs), dtype=torch.float32).unsqueeze(0)
    horizon = int(min(cfg.horizon, linear_schedule(cfg.horizon_schedule, step)))
    num_pi_trajs = int(cfg.mixture_coef * cfg.num_samples)
    A = cfg.action_dim
    if num_pi_trajs > 0:
        pi_actions = torch.empty(horizon, num_pi_trajs, A)
        z = told.h(obs).repeat(num_pi_trajs, 1)
        for t in range(horizon):
            pi_actions[t] = told.pi(z, cfg.min_std, noise.eps_pi[t])
            z, _ = told.next(z, pi_actions[t])

    z = told.h(obs).repeat(cfg.num_samples + num_pi_trajs, 1)
    mean = torch.zeros(horizon, A)
    std = 2 * torch.ones(horizon, A)
    if not t0 and state.prev_mean is not None:
        mean[:-1] = state.prev_mean[1:]
    if trace is not None:
        trace["z0"] = z[0].clone()
        trace["mean_init"] = mean.clone()
        if num_pi_trajs > 0:
            trace["pi_actions"] = pi_actions.clone()

    for i in range(cfg.iterations):
        actions = torch.clamp(mean.unsqueeze(1) + std.unsqueeze(1) * noise.eps_cem[i], -1, 1)
        if num_pi_trajs > 0:
            actions = torch.cat([actions, pi_actions], dim=1)
        value, reward_mean = estimate_value(told, cfg, z, actions, horizon, noise.eps_term[i], trace)
        elite_idxs = torch.topk(value.squeeze(1), cfg.num_elites, dim=0).indices
        elite_value, elite_actions = value[elite_idxs], actions[:, elite_idxs]
        max_value = elite_value.max(0)[0]
        score = torch.exp(cfg.temperature * (elite_value - max_value))
        score /= score.sum(0)
        _mean = torch.sum(score.unsqueeze(0) * elite_actions, dim=1) / (score.sum(0) + 1e-9)
        _std = torch.sqrt(torch.sum(score.unsqueeze(0) * (elite_actions - _mean.unsqueeze(1)) ** 2, dim=1) /
                          (score.sum(0) + 1e-9))
        _std = _std.clamp_(state.std, 2)
        mean, std = cfg.momentum * mean + (1 - cfg.momentum) * _mean, _std
        if trace is not None:
            trace.setdefault("actions", []).append(actions.clone())
            trace.setdefault("value", []).append(value.clone())
            trace.setdefault("elite_idxs", []).append(elite_idxs.clone())
            trace.setdefault("mean", []).append(mean.clone())
            trace.setdefault("std", []).append(std.clone())
            trace.setdefault("score", []).append(score.clone())
            trace.setdefault("reward_mean", []).append(reward_mean)

    score = score.squeeze(1).cpu().numpy()
    j = choice_index(score, noise.u)
    actions = elite_actions[:, j]
    state.prev_mean = mean
    mean, std = actions[0], _std[0]
    a = mean
    if not eval_mode:
        a += std * noise.eps_act
    plan_metrics.update({"current_std": std.mean().item(), "external_reward_mean": reward_mean})
    if trace is not None:
        trace["j"] = j
    return a, plan_metrics


def choice_index(p_f32: np.ndarray, u: float) -> int:
    """`np.random.choice(len(p), p=p)` given its one uniform draw u (numpy legacy RandomState.choice:
    cdf = cumsum(float64 p); cdf /= cdf[-1]; searchsorted(cdf, u, side='right'))."""
    cdf = np.cumsum(p_f32.astype(np.float64))
    cdf /= cdf[-1]
    return int(np.searchsorted(cdf, u, side="right"))
