"""Prioritized replay: the oracle restatement against the reference's own samples
(tests/golden/replay_*.npz from make_replay_golden.py) and the GPU sampler against both.

Parity bar: sampled indices and every gathered window (obs, next_obs, action, reward) bit-exact; IS weights
bit-exact given the same float32 probabilities. The device computes probs = p**alpha / sum(p**alpha) with its
own fp32 reduction order, so its probabilities may differ from torch's in the last bits (checked to 2e-6
relative); indices then still agree unless a uniform falls within that rounding of a cdf boundary, which the
golden cases do not hit.
"""
import os
import warnings

import numpy as np
import pytest
import torch

from oracle.replay_ref import RefReplay, choice
from replay_io import CASES, SCHEDULES, case_cfg, episode, priorities, uniforms

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _golden(name):
    return np.load(os.path.join(GOLDEN, f"replay_{name}.npz"))


def _replay_schedule(name, buf, on_sample):
    c = case_cfg(name)
    k, last = 0, None
    for op, seed in SCHEDULES[name]:
        if op == "add":
            buf.add(*episode(c, seed))
        elif op == "prio":
            buf.update_priorities(last, priorities(c, seed))
        else:
            last = on_sample(k, seed)
            k += 1
    return k


@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_matches_reference_replay(name):
    c = case_cfg(name)
    g = _golden(name)
    ref = RefReplay(c)

    def on_sample(k, seed):
        obs, next_obs, action, reward, idxs, weights, used = ref.sample(uniforms(c, seed))
        assert np.array_equal(idxs.numpy(), g[f"s{k}_idxs"])
        for key, v in dict(obs=obs, next_obs=next_obs, action=action, reward=reward, weights=weights).items():
            assert np.array_equal(v.numpy(), g[f"s{k}_{key}"]), (k, key)
        return idxs

    n = _replay_schedule(name, ref, on_sample)
    assert n == int(g["nsamples"])


def test_choice_without_replacement_rounds():
    """numpy's no-replacement rounds: heavy mass on few items forces collisions and several rounds."""
    rs = np.random.RandomState(0)
    p = np.full(100, 1e-3, dtype=np.float32)
    p[:5] = 10.0
    p /= p.sum()
    np.random.seed(5)
    want = np.random.choice(100, 20, replace=False, p=p)
    got, used = choice(p, 20, False, np.random.RandomState(5).random_sample(400))
    assert np.array_equal(got, want) and used > 20


# ------------------------------------------------------------------------------------------------ GPU
def _gpu_cfg(c, device="cuda"):
    from types import SimpleNamespace
    return SimpleNamespace(**{**vars(c), "device": device, "train_steps": c.capacity, "max_buffer_size": 10**9,
                              "env_horizon": c.horizon})


class _Ep:
    def __init__(self, obs, action, reward):
        self.obs, self.action, self.reward = torch.from_numpy(obs), torch.from_numpy(action), torch.from_numpy(reward)


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(CASES))
def test_gpu_replay_matches_reference(name):
    """The device buffer through the golden schedule: indices and windows bit-exact to the reference's."""
    from tdmpc_amd.replay import ReplayBuffer
    c = case_cfg(name)
    g = _golden(name)
    buf = ReplayBuffer(_gpu_cfg(c), latent_plan=True)
    k, last = 0, None
    for op, seed in SCHEDULES[name]:
        if op == "add":
            buf.add(_Ep(*episode(c, seed)))
        elif op == "prio":
            buf.update_priorities(last, torch.from_numpy(priorities(c, seed)))
        else:
            obs, next_obs, action, reward, idxs, weights = buf.sample(u=uniforms(c, seed), keep_probs=True)
            np.testing.assert_allclose(buf.last_probs.cpu().numpy(), g[f"s{k}_probs"], rtol=2e-6, atol=0)
            assert np.array_equal(idxs.cpu().numpy(), g[f"s{k}_idxs"]), k
            for key, v in dict(obs=obs, next_obs=next_obs, action=action, reward=reward).items():
                assert np.array_equal(v.cpu().numpy(), g[f"s{k}_{key}"]), (k, key)
            np.testing.assert_allclose(weights.cpu().numpy(), g[f"s{k}_weights"], rtol=2e-6, atol=0)
            assert buf.uniforms_used > 0
            last = idxs.clone()
            k += 1
    # priorities after the schedule equal the oracle's (max, masks, updates are exact float ops)
    ref = RefReplay(c)
    _replay_schedule(name, ref, lambda kk, seed: ref.sample(uniforms(c, seed))[4])
    assert np.array_equal(buf._priorities.cpu().numpy(), ref._priorities.numpy())


@pytest.mark.gpu
@pytest.mark.parametrize("full", [False, True])
def test_gpu_choice_large_buffer(full):
    """A 250k-transition buffer (humanoid: 500000 / action_repeat 2) with random priorities: given the device's
    own float32 probabilities, numpy's choice algorithm (the oracle) picks exactly the device's indices."""
    from types import SimpleNamespace
    from tdmpc_amd.replay import ReplayBuffer
    L, cap = 500, 250_000
    c = SimpleNamespace(modality="state", obs_shape=(67,), action_dim=21, episode_length=L, capacity=cap,
                        batch_size=512, horizon=5, per_alpha=0.6, per_beta=0.4, frame_stack=1)
    buf = ReplayBuffer(_gpu_cfg(c), latent_plan=True)
    rs = np.random.RandomState(0)
    n_ep = cap // L if full else (cap // L) // 2 + 3
    ep = _Ep(rs.standard_normal((L + 1, 67)).astype(np.float32), rs.uniform(-1, 1, (L, 21)).astype(np.float32),
             rs.standard_normal(L).astype(np.float32))
    for _ in range(n_ep):
        buf.add(ep)
    total = cap if full else buf.idx
    idx = rs.randint(0, total, size=20000)
    buf.update_priorities(torch.from_numpy(idx), torch.from_numpy(rs.exponential(1.0, size=(20000, 1)).astype(np.float32)))
    u = rs.random_sample(4 * 512)
    obs, next_obs, action, reward, idxs, weights = buf.sample(u=u, keep_probs=True)
    probs = buf.last_probs.cpu().numpy()
    want, used = choice(probs, 512, not full, u)
    assert np.array_equal(idxs.cpu().numpy(), want)
    assert buf.uniforms_used == used
    w = (total * torch.from_numpy(probs)[torch.from_numpy(want)]) ** (-0.4)
    np.testing.assert_allclose(weights.cpu().numpy(), (w / w.max()).numpy(), rtol=2e-6)
    if full:
        assert len(set(want.tolist())) == 512
    # windows: rows of the storage
    st = buf._obs.cpu()
    assert torch.equal(obs.cpu(), st[idxs.cpu()])
    assert torch.equal(next_obs[2].cpu(), st[idxs.cpu() + 3])


def _big_buffer(full, cap=250_000, L=500):
    from types import SimpleNamespace
    from tdmpc_amd.replay import ReplayBuffer
    c = SimpleNamespace(modality="state", obs_shape=(67,), action_dim=21, episode_length=L, capacity=cap,
                        batch_size=512, horizon=5, per_alpha=0.6, per_beta=0.4, frame_stack=1)
    buf = ReplayBuffer(_gpu_cfg(c), latent_plan=True)
    rs = np.random.RandomState(1)
    ep = _Ep(rs.standard_normal((L + 1, 67)).astype(np.float32), rs.uniform(-1, 1, (L, 21)).astype(np.float32),
             rs.standard_normal(L).astype(np.float32))
    for _ in range(cap // L if full else cap // L // 2):
        buf.add(ep)
    return buf


@pytest.mark.gpu
def test_gpu_update_priorities_last_writer_wins():
    """helper.py:487-488 with duplicate indices, at the bench's size (50k updates): the last occurrence wins,
    as a sequential index_put_ on the CPU; repeated calls (generation-tagged keys, never cleared) included."""
    buf = _big_buffer(False)
    total = buf.idx
    rs = np.random.RandomState(5)
    ref = buf._priorities.cpu().numpy().copy()
    for n, span in ((50_000, 3000), (700, 50), (50_000, total)):
        idx = rs.randint(0, span, size=n)
        v = rs.exponential(1.0, size=(n, 1)).astype(np.float32)
        buf.update_priorities(torch.from_numpy(idx), torch.from_numpy(v))
        for i, k in enumerate(idx):   # the reference's CPU index_put_: sequential
            ref[k] = np.float32(v[i, 0] + np.float32(1e-6))
        assert np.array_equal(buf._priorities.cpu().numpy(), ref)


@pytest.mark.gpu
def test_gpu_norepl_concentrated_priorities():
    """Without replacement on a full buffer whose mass sits on a few hundred transitions (one of them 1e6 times
    the rest): several of numpy's rounds, each after zeroing the found masses -- the device's picks equal the
    oracle's choice on the device's probabilities and the same uniforms, and the uniforms consumed agree."""
    buf = _big_buffer(True)
    rs = np.random.RandomState(2)
    buf._priorities.zero_()
    hot = rs.choice(buf.capacity, 700, replace=False)
    p = rs.exponential(1.0, size=700).astype(np.float32)
    p[0] = 1e6
    buf.update_priorities(torch.from_numpy(hot), torch.from_numpy(p[:, None]))
    u = rs.random_sample(64 * 512)
    *_, idxs, weights = buf.sample(u=u, keep_probs=True)
    probs = buf.last_probs.cpu().numpy()
    want, used = choice(probs, 512, False, u)
    assert np.array_equal(idxs.cpu().numpy(), want)
    assert buf.uniforms_used == used and used > 512   # more than one round
    # the same with only batch_size uniforms: the rounds continue on the hash stream, still distinct picks
    *_, idxs, _ = buf.sample(u=u[:512])
    got = idxs.cpu().numpy()
    assert len(set(got.tolist())) == 512 and (probs[got] > 0).all() and buf.uniforms_used > 512
    with pytest.warns(RuntimeWarning, match="uniforms"):   # past the supplied stream: no longer numpy's draw
        buf.check_sample()
    # enough uniforms supplied: no warning
    buf.sample(u=u)
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        assert buf.check_sample() == used
    # the buffer's own draws (u=None, as TDMPC.update samples): no caller stream, so no warning however many
    # uniforms the rounds took
    buf.sample()
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        assert buf.check_sample() > 0


@pytest.mark.gpu
def test_gpu_norepl_fewer_nonzero_than_batch_raises():
    """numpy's choice(replace=False) raises when fewer than `size` entries have mass; the device flags it and
    check_sample() raises the same ValueError."""
    buf = _big_buffer(True)
    buf._priorities.zero_()
    hot = torch.arange(0, 300, dtype=torch.int64) * 7
    buf.update_priorities(hot, torch.ones(300, 1))
    *_, idxs, _ = buf.sample()
    with pytest.raises(ValueError, match="Fewer non-zero"):
        buf.check_sample()
    assert set(idxs.cpu().numpy().tolist()[:300]) == set(hot.tolist())
