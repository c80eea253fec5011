"""Shared by tests/golden/make_learner_golden.py and tests/test_learner.py: the learner golden case."""
import numpy as np
import torch

from tdmpc_amd.config import make_cfg

METRICS = ("consistency_loss", "reward_loss", "value_loss", "pi_loss", "total_loss", "weighted_loss", "grad_norm")


def learner_cfg():
    """cartpole dims, a 64-transition batch, horizon 5, the reference's learning defaults
    (cfgs/default.yaml: lr 1e-3, rho 1.0, coefs 0.5 / 0.5 / 0.1, grad_clip 10, update_freq 2, tau 0.01)."""
    return make_cfg("cartpole", num_samples=64, num_elites=32, iterations=3, horizon=5, batch_size=64)


def batch(cfg, seed=5):
    """(obs [B, obs], next_obses [H+1, B, obs], action [H+1, B, A], reward [H+1, B, 1], idxs [B], weights [B])"""
    rs = np.random.RandomState(seed)
    B, H, O, A = cfg.batch_size, cfg.horizon, cfg.obs_shape[0], cfg.action_dim
    f = lambda *s: torch.from_numpy(rs.standard_normal(s).astype(np.float32))  # noqa: E731
    obs = f(B, O)
    next_obses = f(H + 1, B, O)
    action = torch.from_numpy(rs.uniform(-1, 1, (H + 1, B, A)).astype(np.float32))
    reward = f(H + 1, B, 1)
    idxs = torch.arange(B, dtype=torch.int64)
    weights = torch.from_numpy(rs.uniform(0.5, 1.0, B).astype(np.float32))
    return obs, next_obses, action, reward, idxs, weights


def probe(n_elems, k=64, seed=0):
    return np.random.RandomState(seed).randint(0, n_elems, size=k)


def summarize(sd):
    """per tensor: float64 sum, sum of squares, and 64 fixed elements (one row per tensor)."""
    s, ss, pr = [], [], []
    for i, v in enumerate(sd.values()):
        v = v.detach().double().reshape(-1).cpu()
        s.append(float(v.sum()))
        ss.append(float((v ** 2).sum()))
        pr.append(v[torch.from_numpy(probe(v.numel(), seed=i))].numpy())
    return np.array(s), np.array(ss), np.stack(pr)
