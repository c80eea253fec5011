"""Learner: `TDMPC.update / update_pi / _td_target`.

* The oracle (oracle/learner_ref.py) reproduces the reference `TDMPC.update` bit for bit on the CPU
  (tests/golden/learner_cartpole.npz, recorded from the reference by make_learner_golden.py).
* The GPU learner (tdmpc_amd.learner, eager and HIP-graph replay) against the oracle on the same batch and the
  same TruncatedNormal draws. Tolerance (fp32, stated here): losses / grad norm rtol 2e-5; parameters after
  an update |gpu - ref| <= 1e-6 + 1e-4 |ref| for >= 99.9 % of the elements and <= 2 lr everywhere (Adam
  turns a last-bit gradient difference on an element whose gradient is ~0 into a different step of size
  <= lr); priorities rtol 2e-5. Graph replay equals eager bitwise.
"""
import os

import numpy as np
import pytest
import torch

from learner_io import METRICS, batch, learner_cfg, summarize
from oracle.learner_ref import RefLearner
from tdmpc_amd.told import synthetic_state_dict

G = np.load(os.path.join(os.path.dirname(__file__), "golden", "learner_cartpole.npz"))


def test_oracle_learner_matches_reference():
    cfg = learner_cfg()
    lr = RefLearner(cfg, synthetic_state_dict(cfg, 21), synthetic_state_dict(cfg, 22))
    b = batch(cfg)
    torch.manual_seed(0)
    for k, step in enumerate((1, 2)):
        m, prio = lr.update(b, step)
        assert np.array_equal(np.array([m[n] for n in METRICS]), G[f"u{k}_metrics"]), k
        assert np.array_equal(prio.numpy(), G[f"u{k}_prio"]), k
        sd, sdt = lr.state_dicts()
        for tag, d in (("model", sd), ("target", sdt)):
            s, ss, pr = summarize(d)
            assert np.array_equal(s, G[f"u{k}_{tag}_sum"]), (k, tag)
            assert np.array_equal(ss, G[f"u{k}_{tag}_sumsq"]), (k, tag)
            assert np.array_equal(pr, G[f"u{k}_{tag}_probe"]), (k, tag)


# ------------------------------------------------------------------------------------------------ GPU
class _DeviceBatchBuffer:
    """Hands out one fixed batch (already on the device) and keeps the priorities it is given."""

    def __init__(self, b, device="cuda"):
        self.b = tuple(x.to(device) for x in b)
        self.prio = torch.zeros(self.b[0].shape[0], 1, device=device)

    def sample(self):
        return self.b

    def update_priorities(self, idxs, p):
        self.prio.copy_(p)


def _params_close(got, want, lr):
    """|got - want| <= 1e-6 + 1e-4 |want| on >= 99.9 % of the elements, <= 2 lr + 1e-6 everywhere."""
    for k in want:
        g, w = got[k].detach().double().cpu(), want[k].detach().double()
        d = (g - w).abs()
        assert (d <= 2 * lr + 1e-6).all(), (k, float(d.max()))
        frac = float((d <= 1e-6 + 1e-4 * w.abs()).double().mean())
        assert frac >= 0.999, (k, frac)


@pytest.mark.gpu
def test_gpu_update_matches_oracle():
    from tdmpc_amd.tdmpc import TDMPC
    cfg = learner_cfg()
    agent = TDMPC(cfg)
    agent.model.load_state_dict(synthetic_state_dict(cfg, 21))
    agent.model_target.load_state_dict(synthetic_state_dict(cfg, 22))
    ref = RefLearner(cfg, synthetic_state_dict(cfg, 21), synthetic_state_dict(cfg, 22))
    b = batch(cfg)
    buf = _DeviceBatchBuffer(b)
    H, B, A = cfg.horizon, cfg.batch_size, cfg.action_dim
    torch.manual_seed(0)   # the oracle draws the same 2H+1 normals per update from this generator
    noise = [[torch.empty(B, A).normal_() for _ in range(2 * H + 1)] for _ in range(2)]
    torch.manual_seed(0)
    for k, step in enumerate((1, 2)):
        m = agent.update(buf, step, noise=noise[k])
        rm, rprio = ref.update(b, step)
        np.testing.assert_allclose([m[n] for n in METRICS], [rm[n] for n in METRICS], rtol=2e-5, atol=1e-7)
        np.testing.assert_allclose(buf.prio.cpu().numpy(), rprio.numpy(), rtol=2e-5, atol=1e-6)
        sd, sdt = ref.state_dicts()
        _params_close(agent.model.state_dict(), sd, cfg.lr)
        _params_close(agent.model_target.state_dict(), sdt, cfg.lr)


@pytest.mark.gpu
@pytest.mark.parametrize("task", ["humanoid", "dog", "cheetah"])
def test_gpu_update_matches_oracle_full_size(task):
    """The bench's learner shape (batch 512, horizon 5, mlp 512; humanoid L100 A21 / dog L100 A38 obs 223 / cheetah L50 A6):
    two updates (EMA on the second) against the oracle, same batch and TruncatedNormal draws, same tolerances."""
    from tdmpc_amd.config import make_cfg
    from tdmpc_amd.tdmpc import TDMPC
    cfg = make_cfg(task, num_samples=64, num_elites=32, iterations=3, horizon=5, batch_size=512)
    agent = TDMPC(cfg)
    agent.model.load_state_dict(synthetic_state_dict(cfg, 31))
    agent.model_target.load_state_dict(synthetic_state_dict(cfg, 32))
    assert agent.learner().engine is not None
    ref = RefLearner(cfg, synthetic_state_dict(cfg, 31), synthetic_state_dict(cfg, 32))
    b = batch(cfg, seed=9)
    buf = _DeviceBatchBuffer(b)
    H, B, A = cfg.horizon, cfg.batch_size, cfg.action_dim
    torch.manual_seed(1)
    noise = [[torch.empty(B, A).normal_() for _ in range(2 * H + 1)] for _ in range(2)]
    torch.manual_seed(1)
    for k, step in enumerate((1, 2)):
        m = agent.update(buf, step, noise=noise[k])
        rm, rprio = ref.update(b, step)
        np.testing.assert_allclose([m[n] for n in METRICS], [rm[n] for n in METRICS], rtol=2e-5, atol=1e-7)
        np.testing.assert_allclose(buf.prio.cpu().numpy(), rprio.numpy(), rtol=2e-5, atol=1e-6)
        sd, sdt = ref.state_dicts()
        _params_close(agent.model.state_dict(), sd, cfg.lr)
        _params_close(agent.model_target.state_dict(), sdt, cfg.lr)


@pytest.mark.gpu
def test_graph_replay_equals_eager():
    """6 updates from a device replay buffer: 3 eager warm-ups + 3 graph replays == 6 eager updates, bitwise
    (same kernels, same philox offsets), including the buffer's priorities and the EMA target."""
    from types import SimpleNamespace
    from tdmpc_amd.replay import ReplayBuffer
    from tdmpc_amd.tdmpc import TDMPC
    cfg = learner_cfg()
    rc = SimpleNamespace(**{**vars(cfg), "device": "cuda", "train_steps": 2000, "max_buffer_size": 10**6,
                            "episode_length": 200, "env_horizon": cfg.horizon})
    rs = np.random.RandomState(0)
    ep = SimpleNamespace(obs=torch.from_numpy(rs.standard_normal((201, 5)).astype(np.float32)),
                         action=torch.from_numpy(rs.uniform(-1, 1, (200, 1)).astype(np.float32)),
                         reward=torch.from_numpy(rs.standard_normal(200).astype(np.float32)))
    runs = []
    for warm in (3, 100):
        agent = TDMPC(cfg)
        agent.model.load_state_dict(synthetic_state_dict(cfg, 21))
        agent.model_target.load_state_dict(synthetic_state_dict(cfg, 22))
        agent.learner(graph=True, warmup=warm)
        buf = ReplayBuffer(rc, latent_plan=True)
        for _ in range(3):
            buf.add(ep)
        torch.manual_seed(7)
        ms = [agent.update(buf, s + 1, sync_metrics=False).clone() for s in range(6)]
        runs.append((agent, buf, torch.stack(ms)))
    (a1, b1, m1), (a2, b2, m2) = runs
    assert a1.learner()._graphs and not a2.learner()._graphs
    assert torch.equal(m1, m2)
    assert torch.equal(b1._priorities, b2._priorities)
    for x, y in zip(list(a1.model.parameters()) + list(a1.model_target.parameters()),
                    list(a2.model.parameters()) + list(a2.model_target.parameters())):
        assert torch.equal(x, y)


class _CpuAgent:
    """The attributes Learner reads from a TDMPC agent, on the CPU (no planner, no HIP library)."""

    def __init__(self, cfg, sd, sdt):
        from tdmpc_amd.learner import RandomShiftsAug
        from tdmpc_amd.told import TOLD
        self.cfg, self.device = cfg, torch.device("cpu")
        self.model, self.model_target = TOLD(cfg), TOLD(cfg)
        self.model.load_state_dict(sd)
        self.model_target.load_state_dict(sdt)
        self.aug = RandomShiftsAug(cfg)
        self.planner = type("P", (), {"_packed_key": None})()


def test_cpu_batched_learner_matches_oracle():
    """The learner's horizon-batched formulation (TD targets, Q / reward heads and the policy update as one
    pass over H*B rows; only the dynamics chain loops) against the oracle's per-step reference order, run on
    the CPU with the same draws: same tolerance as the GPU test."""
    from tdmpc_amd.learner import Learner
    cfg = learner_cfg()
    agent = _CpuAgent(cfg, synthetic_state_dict(cfg, 21), synthetic_state_dict(cfg, 22))
    ln = Learner(agent, graph=False)
    ref = RefLearner(cfg, synthetic_state_dict(cfg, 21), synthetic_state_dict(cfg, 22))
    b = batch(cfg)
    buf = _DeviceBatchBuffer(b, device="cpu")
    H, B, A = cfg.horizon, cfg.batch_size, cfg.action_dim
    torch.manual_seed(0)
    noise = [[torch.empty(B, A).normal_() for _ in range(2 * H + 1)] for _ in range(2)]
    torch.manual_seed(0)
    for k, step in enumerate((1, 2)):
        m = ln.update(buf, step, noise=noise[k])
        rm, rprio = ref.update(b, step)
        np.testing.assert_allclose(m.numpy(), [rm[n] for n in METRICS], rtol=2e-5, atol=1e-7)
        np.testing.assert_allclose(buf.prio.numpy(), rprio.numpy(), rtol=2e-5, atol=1e-6)
        sd, sdt = ref.state_dicts()
        _params_close(agent.model.state_dict(), sd, cfg.lr)
        _params_close(agent.model_target.state_dict(), sdt, cfg.lr)


AUG_ATOL = 2.5e-3   # the reference's fp32 grid coordinates sit within ~1e-5 px of the pixel centres


def _aug_golden():
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "learner_aug_pixels.npz"))
    for k in ("4", "5"):
        x = g["x" + k].astype(np.float32)
        n = x.shape[0] * x.shape[1] if x.ndim == 5 else x.shape[0]
        torch.manual_seed(11)   # the reference's draw in make_aug_golden.py
        shift = torch.randint(0, 9, size=(n, 1, 1, 2), dtype=torch.float32).view(n, 2).numpy()
        yield k, x, g["y" + k], shift


def test_random_shift_oracle_matches_reference():
    """oracle.learner_ref.random_shift (the integer-shift restatement of RandomShiftsAug, helper.py:250-283) against
    the reference module's recorded outputs (tests/golden/learner_aug_pixels.npz, make_aug_golden.py): 4-D and 5-D
    (horizon) batches, within AUG_ATOL."""
    from oracle.learner_ref import random_shift
    for k, x, y, shift in _aug_golden():
        xs = x.reshape(-1, *x.shape[-3:])
        r = random_shift(xs, shift, 4).reshape(y.shape)
        assert np.abs(r - y).max() <= AUG_ATOL, k


@pytest.mark.gpu
def test_gpu_random_shifts_aug_matches_reference():
    """tdmpc_amd.learner.RandomShiftsAug on the device (tdmpc_random_shift gather kernel): same torch draw as the
    reference module, output equal to the oracle's integer shift bitwise and within AUG_ATOL of the reference's
    recorded outputs, 4-D and 5-D batches."""
    from types import SimpleNamespace
    from oracle.learner_ref import random_shift
    from tdmpc_amd.learner import RandomShiftsAug
    aug = RandomShiftsAug(SimpleNamespace(img_size=84, modality="pixels"))
    for k, x, y, shift in _aug_golden():
        # the golden's shifts came from the CPU generator (make_aug_golden.py); on the GPU the module draws from
        # torch's CUDA generator with the reference's call (shape, dtype, device), checked below
        out = aug(torch.from_numpy(x).cuda(), shift=shift).cpu().numpy()
        assert out.shape == y.shape
        assert np.abs(out - y).max() <= AUG_ATOL, k
        xs = x.reshape(-1, *x.shape[-3:])
        assert np.array_equal(out.reshape(xs.shape), random_shift(xs, shift, 4)), k
        n = xs.shape[0]
        torch.manual_seed(12)
        out = aug(torch.from_numpy(x).cuda()).cpu().numpy()
        torch.manual_seed(12)
        drawn = torch.randint(0, 9, size=(n, 1, 1, 2), device="cuda", dtype=torch.float32).view(n, 2).cpu().numpy()
        assert np.array_equal(out.reshape(xs.shape), random_shift(xs, drawn, 4)), k


@pytest.mark.gpu
def test_gpu_pixel_update_graph_equals_eager():
    """Pixel TOLD (quadruped frames, conv encoder, RandomShiftsAug on the device) on the learner engine (the conv
    stack's forward / backward as learner_conv.hip kernels, every sum in a fixed order): 4 updates from a fixed
    batch, 3 eager warm-ups + 1 graph replay vs 4 eager updates, bitwise."""
    from tdmpc_amd.config import make_cfg
    from tdmpc_amd.tdmpc import TDMPC
    cfg = make_cfg("quadruped", modality="pixels", num_samples=32, num_elites=8, iterations=2, horizon=3,
                   batch_size=16)
    rs = np.random.RandomState(1)
    B, H, A = cfg.batch_size, cfg.horizon, cfg.action_dim
    obs_shape = tuple(cfg.obs_shape)
    b = (torch.from_numpy(rs.randint(0, 256, (B,) + obs_shape).astype(np.float32)),
         torch.from_numpy(rs.randint(0, 256, (H + 1, B) + obs_shape).astype(np.float32)),
         torch.from_numpy(rs.uniform(-1, 1, (H + 1, B, A)).astype(np.float32)),
         torch.from_numpy(rs.standard_normal((H + 1, B, 1)).astype(np.float32)),
         torch.arange(B), torch.ones(B))

    class Buf(_DeviceBatchBuffer):
        graph_safe, idx, _full = True, 0, False

    outs = []
    det = torch.backends.cudnn.deterministic
    torch.backends.cudnn.deterministic = True
    for warm in (3, 100):
        agent = TDMPC(cfg)
        agent.model.load_state_dict(synthetic_state_dict(cfg, 4))
        agent.model_target.load_state_dict(synthetic_state_dict(cfg, 5))
        agent.learner(graph=True, warmup=warm)
        buf = Buf(b)
        torch.manual_seed(9)
        ms = [agent.update(buf, s + 1, sync_metrics=False).clone() for s in range(4)]
        outs.append((agent, torch.stack(ms)))
    torch.backends.cudnn.deterministic = det
    (a1, m1), (a2, m2) = outs
    assert a1.learner().engine is not None and a1.learner()._graphs and not a2.learner()._graphs
    assert torch.isfinite(m1).all()
    assert torch.equal(m1, m2)
    for x, y in zip(a1.model.parameters(), a2.model.parameters()):
        assert torch.equal(x, y)


@pytest.mark.gpu
def test_gpu_pixel_update_matches_oracle():
    """Pixel TOLD at the learner's full shape (quadruped-run pixels: 9 x 84 x 84 frame stacks, conv encoder, batch
    512, horizon 5): two updates (EMA on the second) against the oracle (oracle/learner_ref.py, the reference's
    tdmpc.py:192-245 op for op), same batch and TruncatedNormal draws, on the learner engine (no autograd, no MIOpen:
    learner_conv.hip's conv kernels). RandomShiftsAug draws its shifts on the
    device (its own parity: test_gpu_random_shifts_aug_matches_reference), so the device's augmented frames are
    recorded and handed to the oracle as its observations -- the reference feeds the same augmented next_obs to
    the target encoder and to the TD target (tdmpc.py:207-208), as the learner does. Metrics and priorities at the
    state learner tests' tolerances; the first update's gradients (after clip_grad_norm_) within 1e-4 of each
    tensor's largest |gradient|, 1e-3 for the conv layers' weights and biases (an element of the first conv's
    gradients sums B x 39 x 39 = 779k products that largely cancel: the CPU's and the GPU's fp32 summation orders differ by up to
    ~2e-4 of the largest element, measured); parameters as _params_close, except the conv kernels: a conv weight's gradient sums
    B x 39 x 39 (first layer) products, and in an output channel whose ReLU is nearly dead that sum is decided by
    rounding, where Adam's first step (+-lr sign(g)) turns a different summation order into a step of the other sign
    -- so for the conv layers' weights and biases <= 2 lr everywhere (the bound Adam guarantees) and >= 90 % of the elements within the tight bound."""
    from tdmpc_amd.config import make_cfg
    from tdmpc_amd.tdmpc import TDMPC
    cfg = make_cfg("quadruped", modality="pixels", num_samples=64, num_elites=32, iterations=3, horizon=5,
                   batch_size=512)
    agent = TDMPC(cfg)
    agent.model.load_state_dict(synthetic_state_dict(cfg, 41))
    agent.model_target.load_state_dict(synthetic_state_dict(cfg, 42))
    assert agent.learner().engine is not None   # (the hand-written engine, not autograd + MIOpen)
    ref = RefLearner(cfg, synthetic_state_dict(cfg, 41), synthetic_state_dict(cfg, 42))
    B, H, A = cfg.batch_size, cfg.horizon, cfg.action_dim
    shape = tuple(cfg.obs_shape)
    rs = np.random.RandomState(3)
    b = (torch.from_numpy(rs.randint(0, 256, (B,) + shape).astype(np.float32)),
         torch.from_numpy(rs.randint(0, 256, (H + 1, B) + shape).astype(np.float32)),
         torch.from_numpy(rs.uniform(-1, 1, (H + 1, B, A)).astype(np.float32)),
         torch.from_numpy(rs.standard_normal((H + 1, B, 1)).astype(np.float32)),
         torch.arange(B), torch.ones(B))
    buf = _DeviceBatchBuffer(b)
    rec, aug = [], agent.aug

    def recording_aug(x, div=0.0):
        # (the engine augments straight into normalised frames, div = 255: the integer frames are recovered for the
        # oracle, which normalises them itself -- and torch's own x / 255 of them must be the kernel's output)
        y = aug(x, div=div)
        r = y.detach().cpu()
        if div:
            raw = torch.round(r * div)
            assert torch.equal(raw / div, r)
            r = raw
        rec.append(r)
        return y

    agent.aug = recording_aug
    torch.manual_seed(2)
    noise = [[torch.empty(B, A).normal_() for _ in range(2 * H + 1)] for _ in range(2)]
    torch.manual_seed(2)
    det = torch.backends.cudnn.deterministic
    torch.backends.cudnn.deterministic = True
    try:
        for k, step in enumerate((1, 2)):
            rec.clear()
            m = agent.update(buf, step, noise=noise[k])
            nxt_aug, obs_aug = rec   # the learner augments the H next-observation stacks first, then obs
            assert not torch.equal(obs_aug, b[0])   # (the augmentation ran)
            rb = (obs_aug, nxt_aug.view(H, B, *shape), b[2], b[3], b[4], b[5])
            rm, rprio = ref.update(rb, step)
            np.testing.assert_allclose([m[n] for n in METRICS], [rm[n] for n in METRICS], rtol=2e-5, atol=1e-7)
            np.testing.assert_allclose(buf.prio.cpu().numpy(), rprio.numpy(), rtol=2e-5, atol=1e-6)
            conv = [n for n in ref.p if n.startswith("_encoder.") and n.rsplit(".", 2)[1] in "1357"]
            assert len(conv) == 8   # the four conv layers' weights and biases
            if k == 0:
                for (name, pg), (rname, rp) in zip(agent.model.named_parameters(), ref.p.items()):
                    assert name == rname
                    g, r = pg.grad.detach().double().cpu(), rp.grad.detach().double()
                    tol = 1e-3 if name in conv else 1e-4   # (conv layers: sums of up to B x 41 x 41 products)
                    assert float((g - r).abs().max()) <= tol * float(r.abs().max()) + 1e-9, name
            sd, sdt = ref.state_dicts()
            _params_close(agent.model.state_dict(), {n: v for n, v in sd.items() if n not in conv}, cfg.lr)
            _params_close(agent.model_target.state_dict(), sdt, cfg.lr)
            for n in conv:
                d = (agent.model.state_dict()[n].double().cpu() - sd[n].double()).abs()
                assert (d <= 2 * cfg.lr + 1e-6).all(), n
                assert float((d <= 1e-6 + 1e-4 * sd[n].double().abs()).double().mean()) >= 0.9, n
    finally:
        torch.backends.cudnn.deterministic = det


@pytest.mark.gpu
def test_gpu_fused_loss_matches_aten():
    """The fused HIP loss (include/tdmpc_learner.h) against the reference's ATen composition on the same tensors:
    per-row losses, means, weighted loss and every input gradient (rtol 1e-5), with some rows past the 1e4 clamp."""
    from tdmpc_amd.learner import _FusedLoss, _l1, _mse
    g = torch.Generator().manual_seed(3)
    H, B, L = 5, 96, 50
    mk = lambda *s, sc=1.0: (torch.randn(*s, generator=g) * sc).cuda()  # noqa: E731
    zp, nz = mk(H, B, L).requires_grad_(), mk(H, B, L)
    q1, q2, rp = mk(H, B, sc=30).requires_grad_(), mk(H, B, sc=30).requires_grad_(), mk(H, B).requires_grad_()
    rw, td = mk(H, B), mk(H, B, sc=30)
    q1.data[:, :5] += 300.0                      # value loss of rows 0-4 above 1e4: clamped, no gradient
    w = torch.rand(B, generator=g).cuda() + 0.5
    rho = torch.tensor([0.5 ** t for t in range(H)], device="cuda")
    coefs = (2.0, 0.5, 0.1)
    scal, rows = _FusedLoss.apply(zp, nz, q1, q2, rp, rw, td, w, rho, coefs)
    (scal[4] * 0.2).backward()
    got = [zp.grad.clone(), q1.grad.clone(), q2.grad.clone(), rp.grad.clone()]
    for t in (zp, q1, q2, rp):
        t.grad = None
    r = rho.view(H, 1)
    cons = (r * _mse(zp, nz).mean(dim=2)).sum(0)
    rew = (r * _mse(rp, rw)).sum(0)
    val = (r * (_mse(q1, td) + _mse(q2, td))).sum(0)
    pri = (r * (_l1(q1, td) + _l1(q2, td))).sum(0).clamp(max=1e4)
    tot = coefs[0] * cons.clamp(max=1e4) + coefs[1] * rew.clamp(max=1e4) + coefs[2] * val.clamp(max=1e4)
    wl = (tot.view(B, 1) * w).mean()
    (wl * 0.2).backward()
    assert (val[:5] > 1e4).all()
    for x, y in zip(rows, (cons, rew, val, pri, tot)):
        torch.testing.assert_close(x, y.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(scal[:5], torch.stack([cons.mean(), rew.mean(), val.mean(), tot.mean(), wl]).detach(),
                               rtol=1e-5, atol=1e-6)
    for x, y in zip(got, (zp.grad, q1.grad, q2.grad, rp.grad)):
        torch.testing.assert_close(x, y, rtol=1e-5, atol=1e-9)


@pytest.mark.gpu
@pytest.mark.parametrize("layer", [0, 1, 2, 3])
def test_gpu_conv_kernels_match_torch(layer):
    """learner_conv.hip against torch's fp32 convolution on the CPU (float64 sums as the reference), per layer of
    the pixel encoder (quadruped: 9 x 84 x 84 -> 32 x 39 x 39 -> 18 -> 8 -> 3), a batch of 6: the forward with its
    ReLU (and the first layer's NormalizeImg / 255), the data gradient masked by the layer below's ReLU, and the
    weight / bias gradient slices (summed here). Tolerance: 1e-5 of each output's largest magnitude (fp32 sums of up
    to 6 x 39 x 39 products)."""
    import ctypes as C
    import torch.nn.functional as F
    from tdmpc_amd import _lib
    L = _lib.lib()
    ks, hw, cins = (7, 5, 3, 3), (84, 39, 18, 8, 3), (9, 32, 32, 32)
    k, hin, ho, cin, n = ks[layer], hw[layer], hw[layer + 1], cins[layer], 6
    g = torch.Generator().manual_seed(layer)
    x = torch.rand(n, cin, hin, hin, generator=g, dtype=torch.float64)
    if layer == 0:
        x = torch.floor(x * 256).clamp(max=255)     # raw frames, NormalizeImg inside
    else:
        x = torch.relu(x - 0.3)                      # a ReLU output (zeros included: the mask below)
    w = torch.randn(32, cin, k, k, generator=g, dtype=torch.float64) / (cin * k * k) ** 0.5
    bias = torch.randn(32, generator=g, dtype=torch.float64) * 0.1
    dy = torch.randn(n, 32, ho, ho, generator=g, dtype=torch.float64)
    xin = x / 255.0 if layer == 0 else x
    y_ref = torch.relu(F.conv2d(xin, w, bias, stride=2))
    dy_pre = dy * (y_ref > 0)
    dx_ref = torch.nn.grad.conv2d_input(x.shape, w, dy_pre, stride=2) * (x > 0)
    dw_ref = torch.nn.grad.conv2d_weight(xin, w.shape, dy_pre, stride=2)
    db_ref = dy_pre.sum((0, 2, 3))
    dev = "cuda"
    f = lambda t: t.float().contiguous().to(dev)   # noqa: E731
    xd, wd, bd, dyd = f(x), f(w), f(bias), f(dy_pre)
    y = torch.zeros(n, 32, ho, ho, device=dev)
    a = _lib.LgConv()
    a.x, a.nprob, a.n, a.cin, a.hin, a.k, a.in_div = xd.data_ptr(), 1, n, cin, hin, k, 255.0 if layer == 0 else 0.0
    a.w[0], a.b[0], a.y[0] = wd.data_ptr(), bd.data_ptr(), y.data_ptr()
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    _lib.check(L.tdmpc_lg_conv_fwd(C.byref(a), st), "conv_fwd")
    # the large layers run the LDS-staged forward; the direct kernel (TDMPC_CONV_DIRECT) must give the same bits
    y_direct = torch.full_like(y, float("nan"))
    a.y[0] = y_direct.data_ptr()
    os.environ["TDMPC_CONV_DIRECT"] = "1"
    try:
        _lib.check(L.tdmpc_lg_conv_fwd(C.byref(a), st), "conv_fwd direct")
    finally:
        del os.environ["TDMPC_CONV_DIRECT"]
    a.y[0] = y.data_ptr()
    torch.cuda.synchronize()
    assert torch.equal(y, y_direct), float((y - y_direct).abs().max())
    ips = 4
    nsl = -(-n // ips)
    K = cin * k * k
    part = torch.zeros(nsl, 32, K + 1, device=dev)
    _lib.check(L.tdmpc_lg_conv_bwd_weight(dyd.data_ptr(), xd.data_ptr(), 255.0 if layer == 0 else 0.0, part.data_ptr(),
                                          n, cin, hin, k, ips, st), "conv_bwd_weight")
    # (the LDS-staged weight gradient; the direct kernel must give the same bits)
    part_direct = torch.full_like(part, float("nan"))
    os.environ["TDMPC_CONV_DIRECT"] = "1"
    try:
        _lib.check(L.tdmpc_lg_conv_bwd_weight(dyd.data_ptr(), xd.data_ptr(), 255.0 if layer == 0 else 0.0,
                                              part_direct.data_ptr(), n, cin, hin, k, ips, st), "conv_bwd_weight direct")
    finally:
        del os.environ["TDMPC_CONV_DIRECT"]
    torch.cuda.synchronize()
    assert torch.equal(part, part_direct), float((part - part_direct).abs().max())
    if layer > 0:
        dx = torch.zeros(n, cin, hin, hin, device=dev)
        _lib.check(L.tdmpc_lg_conv_bwd_data(dyd.data_ptr(), wd.data_ptr(), xd.data_ptr(), dx.data_ptr(), n, cin, hin, k,
                                            st), "conv_bwd_data")
    torch.cuda.synchronize()

    def close(got, ref, what):
        ref = ref.double()
        err = float((got.double().cpu() - ref).abs().max())
        assert err <= 1e-5 * float(ref.abs().max()) + 1e-7, (what, err, float(ref.abs().max()))

    close(y, y_ref, "forward")
    s = part.double().sum(0).cpu()
    close(s[:, :K].reshape(w.shape), dw_ref, "weight gradient")
    close(s[:, K], db_ref, "bias gradient")
    if layer > 0:
        close(dx, dx_ref, "data gradient")

