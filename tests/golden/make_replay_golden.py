"""Generate tests/golden/replay_{state,pixels}.npz by running the REFERENCE ReplayBuffer in this container.

Run once in the build container (where /root/reference exists):   python tests/golden/make_replay_golden.py
The reference buffer (helper.py:434-534) runs on the CPU: cfg.device = 'cpu', `torch.Tensor.cuda` is made a
no-op and `torch.empty(device='cuda')` allocates on the CPU, because the pixel path of `_get_obs` / `sample`
places tensors on the GPU explicitly (helper.py:494-528); only placement changes, not the arithmetic. The reference is
imported like make_golden.py does (rlpyt stub, no bytecode). Each case follows tests/replay_io.py's schedule:
episodes and priorities come from seeds, and every sample() runs right after np.random.seed(s) so that
np.random.choice's uniforms are `RandomState(s).random_sample(...)`. The .npz holds each sample's outputs.
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np
import torch

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

from make_golden import import_reference  # noqa: E402
from replay_io import CASES, SCHEDULES, case_cfg, episode, priorities  # noqa: E402


def ref_cfg(c):
    return types.SimpleNamespace(device="cpu", train_steps=c.capacity, max_buffer_size=10**9,
                                 modality=c.modality, obs_shape=c.obs_shape, episode_length=c.episode_length,
                                 action_dim=c.action_dim, batch_size=c.batch_size, env_horizon=c.horizon,
                                 horizon=c.horizon, per_alpha=c.per_alpha, per_beta=c.per_beta,
                                 frame_stack=c.frame_stack)


def main():
    import_reference()
    import algorithm.helper as h
    torch.Tensor.cuda = lambda self, *a, **k: self
    # the pixel path also allocates with device=torch.device('cuda') (helper.py:495): place it on the CPU
    _empty = torch.empty

    def empty_cpu(*a, device=None, **k):
        return _empty(*a, device="cpu" if device is not None and str(device).startswith("cuda") else device, **k)
    torch.empty = empty_cpu
    for name in CASES:
        c = case_cfg(name)
        rc = ref_cfg(c)
        buf = h.ReplayBuffer(rc, latent_plan=True)
        out, k, last_idxs = {}, 0, None
        for op, seed in SCHEDULES[name]:
            if op == "add":
                obs, act, rew = episode(c, seed)
                ep = h.Episode(rc, obs[0])
                ep.obs[:] = torch.from_numpy(obs)
                ep.action[:] = torch.from_numpy(act)
                ep.reward[:] = torch.from_numpy(rew)
                buf.add(ep)
            elif op == "prio":
                buf.update_priorities(last_idxs, torch.from_numpy(priorities(c, seed)))
            else:
                np.random.seed(seed)
                obs, next_obs, action, reward, idxs, weights = buf.sample()
                last_idxs = idxs
                for key, v in dict(obs=obs, next_obs=next_obs, action=action, reward=reward, idxs=idxs,
                                   weights=weights).items():
                    out[f"s{k}_{key}"] = v.numpy()
                out[f"s{k}_probs"] = ((buf._priorities if buf._full else buf._priorities[:buf.idx])
                                      ** c.per_alpha / ((buf._priorities if buf._full else
                                                         buf._priorities[:buf.idx]) ** c.per_alpha).sum()).numpy()
                k += 1
        out["nsamples"] = np.array(k)
        path = os.path.join(HERE, f"replay_{name}.npz")
        np.savez_compressed(path, **out)
        print(f"wrote {path}: {k} samples, {os.path.getsize(path)} bytes")


if __name__ == "__main__":
    main()
