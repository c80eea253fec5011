"""Shared by tests/golden/make_replay_golden.py and tests/test_replay.py: the replay-buffer golden cases and
their deterministic episode / priority data (regenerated from seeds, so the fixture stores only outputs)."""
from types import SimpleNamespace

import numpy as np

CASES = {
    # state: 4 episodes of 50 fill the buffer; the schedule wraps around once
    "state": dict(modality="state", obs_shape=(5,), action_dim=2, episode_length=50, capacity=200, batch_size=32,
                  horizon=5, per_alpha=0.6, per_beta=0.4, frame_stack=1),
    # pixels: 3-channel 8x8 frames, frame_stack 3 (stacked obs 9x8x8)
    "pixels": dict(modality="pixels", obs_shape=(9, 8, 8), action_dim=3, episode_length=20, capacity=60,
                   batch_size=16, horizon=3, per_alpha=0.6, per_beta=0.4, frame_stack=3),
}
# operations: ("add", ep_seed) | ("sample", np_seed) | ("prio", seed)  (priorities for the last sample's idxs)
SCHEDULES = {
    "state": [("add", 1), ("add", 2), ("sample", 101), ("prio", 7), ("sample", 102), ("add", 3), ("add", 4),
              ("sample", 103), ("prio", 8), ("sample", 104), ("add", 5), ("sample", 105)],
    "pixels": [("add", 1), ("add", 2), ("sample", 201), ("prio", 9), ("add", 3), ("sample", 202), ("add", 4),
               ("sample", 203)],
}


def case_cfg(name):
    return SimpleNamespace(**CASES[name])


def episode(cfg, seed):
    """(obs [L+1, *obs_shape], action [L, A], reward [L]) of one synthetic episode."""
    rs = np.random.RandomState(seed)
    L = cfg.episode_length
    if cfg.modality == "pixels":
        obs = rs.randint(0, 256, size=(L + 1,) + tuple(cfg.obs_shape)).astype(np.uint8)
    else:
        obs = rs.standard_normal((L + 1,) + tuple(cfg.obs_shape)).astype(np.float32)
    action = rs.uniform(-1, 1, size=(L, cfg.action_dim)).astype(np.float32)
    reward = rs.standard_normal(L).astype(np.float32)
    return obs, action, reward


def priorities(cfg, seed):
    return (np.random.RandomState(seed).rand(cfg.batch_size, 1) * 3).astype(np.float32)


def uniforms(cfg, seed):
    """The stream np.random.choice reads after np.random.seed(seed) (4x batch: enough for the rounds of the
    no-replacement path in these cases)."""
    return np.random.RandomState(seed).random_sample(4 * cfg.batch_size)
