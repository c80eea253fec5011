"""Planner configuration: the subset of the reference cfg that `TDMPC.plan` reads.

The reference builds its cfg with OmegaConf (`src/cfg.py:6-48`): `cfgs/default.yaml` <- CLI <-
`cfgs/{modality}.yaml` <- `cfgs/tasks/{domain}.yaml`. OmegaConf is not a dependency here, and only
attribute access is needed on the hot path, so the cfg is a plain namespace. `make_cfg(task)` resolves
the same precedence for the keys `plan()` touches; the values are cited below so they can be checked.

`obs_shape` / `action_dim` are injected at runtime by the reference's `make_env` (`envs/env.py:284-286`);
dm_control is not installed here, so the DMControl task dims are listed in `TASK_DIMS`.
"""
from __future__ import annotations

import re
from types import SimpleNamespace

# cfgs/default.yaml values used by TDMPC / TOLD (line numbers in that file).
DEFAULTS = dict(
    modality="state",            # :3
    discount=0.99,               # :4
    iterations=6,                # :10
    num_samples=512,             # :11 says 256 ("256 for icem, 512 default"); 512 is the TD-MPC default the
                                 #     north-star metric is quoted on (BASELINE.json metric: N=512)
    num_elites=64,               # :12 says 32 ("32 for icem, 64 default"); 64 at N=512
    mixture_coef=0.5,            # :13
    min_std=0.05,                # :14
    temperature=0.5,             # :15
    momentum=0.1,                # :16
    horizon=5,                   # :29 is 6; BASELINE.json pins H=5 for every config
    std_schedule="linear(0.5, 0.05, 25000, 0)",      # :45 (min_std substituted)
    horizon_schedule="linear(2, 5, 25000, 0)",       # :46 (horizon substituted)
    seed_steps=5000,             # :48
    enc_dim=256,                 # :72
    mlp_dim=512,                 # :73
    latent_dim=50,               # :74
    # learning (TDMPC.update / update_pi / ReplayBuffer, tdmpc.py:165-245, helper.py:434-534)
    lr=1e-3,                     # :64
    batch_size=512,              # :27
    max_buffer_size=1000000,     # :28
    rho=1.0,                     # :37
    reward_coef=0.5,             # :32
    value_coef=0.1,              # :33
    consistency_coef=0.5,        # :34
    per_alpha=0.6,               # :40
    per_beta=0.4,                # :41
    grad_clip_norm=10,           # :42
    update_freq=2,               # :43
    tau=0.01,                    # :44
    # iCEM planner (TdICemSimMlp, tdmpc_icem_similarity_mlp.py; cfgs/default.yaml)
    factor_decrease_num=1.25,    # :20
    shift_elites_over_time=True, # :21
    fraction_elites_reused=0.25, # :22
    keep_previous_elites=True,   # :23
    noise_beta=2.5,              # :24
    regularization_schedule="linear(0.05, 0.5, 1, 5000)",  # :47 (mixture_coef substituted)
    normalize=True,              # :97 (DSSM encoder: helper.dmlab_enc_norm; TOLD ignores it)
    norm_type="ln",              # :98
    # pixels.yaml
    frame_stack=3,               # cfgs/pixels.yaml:2
    num_channels=32,             # cfgs/pixels.yaml:3
    img_size=84,                 # cfgs/pixels.yaml:4
)

# obs_dim / action_dim of the DMControl tasks the configs name (dm_control task specs).
TASK_DIMS = {
    "cartpole": (5, 1),
    "cheetah": (17, 6),
    "humanoid": (67, 21),
    "dog": (223, 38),
    "quadruped": (78, 12),
}

# cfgs/tasks/{domain}.yaml overrides of keys the planner reads.
TASK_OVERRIDES = {
    "humanoid": dict(latent_dim=100,    # cfgs/tasks/humanoid.yaml:6 (iterations:3 / num_samples:4 are
                                        # overridden by BASELINE.json's N=512, iters=6)
                     regularization_schedule="linear(0.05, 0.5, 1, 50000)",     # :9
                     batch_size=512, lr=1e-3),                                    # :7
    "dog": dict(latent_dim=100, batch_size=2048, lr=3e-4),                        # cfgs/tasks/dog.yaml:4-6
    "cartpole": dict(regularization_schedule="linear(0.05, 0.5, 10000, 2500)",  # cfgs/tasks/cartpole.yaml:3
                     lr=3e-4),                                                    # :4
}

# The BASELINE.json configs (name -> overrides). N/H/I come from BASELINE.json itself.
BENCH_CONFIGS = {
    "cartpole-swingup": dict(task="cartpole", num_samples=64, num_elites=32, iterations=3, horizon=5),
    "cheetah-run": dict(task="cheetah", num_samples=512, num_elites=64, iterations=6, horizon=5),
    "humanoid-run": dict(task="humanoid", num_samples=512, num_elites=64, iterations=6, horizon=5),
    "humanoid-run-l512": dict(task="humanoid", num_samples=512, num_elites=64, iterations=6, horizon=5,
                              latent_dim=512),
    "dog-run": dict(task="dog", num_samples=512, num_elites=64, iterations=6, horizon=5),
    "quadruped-run-pixels": dict(task="quadruped", modality="pixels", num_samples=512, num_elites=64,
                                 iterations=6, horizon=5),
}


def make_cfg(task: str = "humanoid", **overrides) -> SimpleNamespace:
    """Resolve a planner cfg: defaults <- task yaml <- overrides (mirrors `src/cfg.py:8-32` precedence)."""
    d = dict(DEFAULTS)
    d.update(TASK_OVERRIDES.get(task, {}))
    d.update(overrides)
    obs_dim, act_dim = TASK_DIMS[task]
    if d["modality"] == "pixels":
        d["obs_shape"] = (3 * d["frame_stack"], d["img_size"], d["img_size"])
    else:
        d["obs_shape"] = (obs_dim,)
    d["action_dim"] = act_dim
    d["task"] = task
    d["device"] = "cuda"
    # schedules are written with the resolved min_std / horizon, as OmegaConf interpolation would.
    if "std_schedule" not in overrides:
        d["std_schedule"] = f"linear(0.5, {d['min_std']}, 25000, 0)"
    if "horizon_schedule" not in overrides:
        d["horizon_schedule"] = f"linear(2, {d['horizon']}, 25000, 0)"
    return SimpleNamespace(**d)


def bench_cfg(name: str, **overrides) -> SimpleNamespace:
    spec = dict(BENCH_CONFIGS[name])
    spec.update(overrides)
    task = spec.pop("task")
    return make_cfg(task, **spec)


def linear_schedule(schdl, step) -> float:
    """Reference `helper.linear_schedule` (`src/algorithm/helper.py:639-652`).

    A float (or float string) is returned as is; `linear(init,final,duration,start)` mixes linearly
    with mix = clip((step-start)/duration, 0, 1), computed in float64 like numpy does there.
    """
    try:
        return float(schdl)
    except (TypeError, ValueError):
        m = re.match(r"linear\((.+),(.+),(.+),(.+)\)", schdl)
        if m:
            init, final, duration, start = [float(g) for g in m.groups()]
            mix = min(max((step - start) / duration, 0.0), 1.0)
            return (1.0 - mix) * init + mix * final
    raise NotImplementedError(schdl)
