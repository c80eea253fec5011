"""GPU parity: the HIP planner (through the C ABI) against the reference's golden vectors and the oracle.

Tolerances (fp32, stated here as the parity contract):
  * per-row estimate_value outputs (G, reward, z_H): |gpu - ref| <= 1e-5 + 1e-4 * |ref|
    (fp32 MFMA k-order vs MKL k-order; measured fp32-vs-fp64 error on G is ~2e-6);
  * CEM mean/std/action: atol 2e-5 while the elite index sets agree;
  * elite sets must agree except for swaps of candidates whose values are within 1e-4 (relative) of the
    cut-off value -- then the trajectories legitimately diverge and later iterations are not compared.
"""
import numpy as np
import pytest
import torch

from golden_io import call_noise, case_names, load_case
from oracle import tdmpc_ref
from tdmpc_amd.config import make_cfg
from tdmpc_amd.tdmpc import TDMPC
from tdmpc_amd.told import synthetic_state_dict

pytestmark = pytest.mark.gpu

from parity_util import ATOL, RTOL, compare_iterations as _compare_iterations, close as _close, \
    elites as _elites, near_tie as _near_tie, record

PATHS = ["layered", "chain16", "chain32", "split", "chain_x6", "split_x6", "chain", "persist", "wide"]


def _agent(cfg, wseed, B=1, path="auto"):
    agent = TDMPC(cfg, max_batch=B, path=path)
    agent.model.load_state_dict(synthetic_state_dict(cfg, wseed))
    agent.std = 0.05
    return agent


@pytest.mark.parametrize("path", PATHS)
@pytest.mark.parametrize("name", case_names())
def test_plan_matches_reference_golden(name, path):
    """Replay every golden call (reference outputs recorded from /root/reference's TDMPC.plan) on the GPU
    with the very same noise, on both kernel paths."""
    cfg, wseed, d = load_case(name)
    agent = _agent(cfg, wseed, path=path)
    for ci in range(int(d["ncalls"])):
        step, t0, ev = [int(x) for x in d[f"c{ci}_call"]]
        nb = call_noise(d, ci)
        if nb.seed_action is not None:
            a, m = agent.plan(d[f"c{ci}_obs"], eval_mode=bool(ev), step=step, t0=bool(t0))
            assert a.shape == (cfg.action_dim,) and (a.abs() <= 1).all()
            continue
        trace = {}
        a, m = agent._plan_envs(d[f"c{ci}_obs"][None], bool(ev), step, [bool(t0)], trace=trace, noise=[nb])
        gv = trace["value"][0].cpu().numpy()
        all_same = _compare_iterations(gv, d[f"c{ci}_values"], cfg.num_elites)
        if all_same:
            np.testing.assert_allclose(a[0].cpu().numpy(), d[f"c{ci}_action"], atol=2e-5, rtol=0)
            np.testing.assert_allclose(agent._prev_mean.cpu().numpy(), d[f"c{ci}_prev_mean"], atol=2e-5, rtol=0)
            rm, cs = m[0]["external_reward_mean"], m[0]["current_std"]
            np.testing.assert_allclose([rm, cs], d[f"c{ci}_metrics"], atol=2e-5, rtol=1e-4)
        record(all_same, f"{name}/{path}/call{ci}")
        if not all_same:
            break   # near-tie swap: this and the later (warm-started) calls diverge legitimately


@pytest.mark.parametrize("task,ov", [
    ("humanoid", dict(num_samples=512, num_elites=64)),
    ("cheetah", dict(num_samples=512, num_elites=64)),
    ("humanoid", dict(num_samples=512, num_elites=64, latent_dim=512)),
    ("dog", dict(num_samples=512, num_elites=64)),
])
@pytest.mark.parametrize("path", PATHS)
def test_estimate_value_fullsize(task, ov, path):
    """TDMPC.estimate_value at BASELINE sizes (T=768, H=5) vs the oracle's CPU fp32 TOLD, both kernel paths."""
    cfg = make_cfg(task, **ov)
    agent = _agent(cfg, 7, path=path)
    pl = agent.planner
    pl.pack(agent.model)
    H, T, A, L = 5, pl.T, cfg.action_dim, cfg.latent_dim
    g = torch.Generator().manual_seed(3)
    z0 = torch.randn(1, L, generator=g)
    actions = torch.rand(1, H, T, A, generator=g) * 2 - 1
    eps = torch.randn(1, T, A, generator=g)
    v, rl, zl = pl.estimate_value(z0, actions, eps, H)
    told = tdmpc_ref.RefTOLD(synthetic_state_dict(cfg, 7), cfg)
    G, ref_r = tdmpc_ref.estimate_value(told, cfg, z0.repeat(T, 1), actions[0], H, eps[0])[0], None
    z = z0.repeat(T, 1)
    for t in range(H):
        z, r = told.next(z, actions[0, t])
    np.testing.assert_array_less(np.abs(zl[0].cpu().numpy() - z.numpy()), ATOL + RTOL * np.abs(z.numpy()) + 1e-12)
    np.testing.assert_array_less(np.abs(rl[0].cpu().numpy() - r[:, 0].numpy()), ATOL + RTOL * np.abs(r[:, 0].numpy()))
    gv, rv = v[0].cpu().numpy(), G[:, 0].numpy()
    assert _close(gv, rv).all(), f"max |dG| {np.abs(gv - rv).max():.3e}"


@pytest.mark.parametrize("task,ov", [("humanoid", {}), ("quadruped", dict(modality="pixels"))])
def test_encoder(task, ov):
    cfg = make_cfg(task, num_samples=64, num_elites=8, **ov)
    agent = _agent(cfg, 11, B=3)
    pl = agent.planner
    pl.pack(agent.model)
    rs = np.random.RandomState(0)
    if cfg.modality == "pixels":
        obs = torch.from_numpy(rs.randint(0, 256, size=(3,) + tuple(cfg.obs_shape)).astype(np.uint8))
        ref_in = obs.float()
    else:
        obs = torch.from_numpy(rs.standard_normal((3,) + tuple(cfg.obs_shape)).astype(np.float32))
        ref_in = obs
    z = pl.encode(obs).cpu().numpy()
    told = tdmpc_ref.RefTOLD(synthetic_state_dict(cfg, 11), cfg)
    zr = told.h(ref_in).numpy()
    assert _close(z, zr, atol=1e-5, rtol=1e-4).all(), np.abs(z - zr).max()


@pytest.mark.parametrize("path", PATHS)
def test_batched_equals_single(path):
    """plan_batch over B envs: an env's result does not depend on its slot in the batch (bitwise, permuted
    envs), and equals a single-env plan of it up to the GEMM tile's summation order (tile shapes are chosen
    by row count, tdmpc_kernels.hip pick_cfg, so B=1 and B=3 may accumulate in different orders)."""
    cfg = make_cfg("humanoid", num_samples=128, num_elites=16, iterations=3)
    B = 3
    agent_b = _agent(cfg, 5, B=B, path=path)
    agent_1 = _agent(cfg, 5, B=1, path=path)
    rs = np.random.RandomState(1)
    obs = rs.standard_normal((B, cfg.obs_shape[0])).astype(np.float32)
    torch.manual_seed(0)
    noises = []
    for e in range(B):
        nb = tdmpc_ref.draw_noise(cfg, 10**6, False)
        noises.append(nb)
    ab, mb = agent_b._plan_envs(obs, False, 10**6, [True] * B, noise=noises)
    ab = ab.cpu()  # (the returned tensors are views of the planner's output buffers)
    perm = [2, 0, 1]
    ap, mp = agent_b._plan_envs(obs[perm], False, 10**6, [True] * B, noise=[noises[e] for e in perm])
    ap = ap.cpu()
    for k, e in enumerate(perm):
        assert torch.equal(ap[k], ab[e]), e
        assert mp[k] == mb[e], e
    for e in range(B):
        a1, _ = agent_1._plan_envs(obs[e:e + 1], False, 10**6, [True], noise=[noises[e]])
        assert torch.allclose(ab[e], a1[0].cpu(), atol=2e-5, rtol=0), e


def test_reference_rng_order_on_device():
    """The drop-in draws its noise from torch's CUDA generator with the reference's call sequence: the same
    seed gives the same stream as separate randn / normal_ calls of the reference's shapes."""
    cfg = make_cfg("cartpole", num_samples=64, num_elites=32, iterations=3)
    agent = _agent(cfg, 1)
    pl = agent.planner
    torch.manual_seed(123)
    np.random.seed(5)
    u = pl.draw_reference_noise(0, 5, 3, False)
    torch.manual_seed(123)
    np.random.seed(5)
    nb = tdmpc_ref.draw_noise(cfg, 10**6, False, device="cuda")
    lay = pl.noise_layout(5, 3)
    buf = pl.noise_view(5, 3, 1)[0]
    P, N, A, T = pl.P, pl.N, pl.A, pl.T
    assert torch.equal(buf[:5 * P * A].view(5, P, A), nb.eps_pi)
    for i in range(3):
        o = lay["cem_off"] + i * lay["iter"]
        assert torch.equal(buf[o:o + 5 * N * A].view(5, N, A), nb.eps_cem[i])
        assert torch.equal(buf[o + 5 * N * A:o + 5 * N * A + T * A].view(T, A), nb.eps_term[i])
    assert u == nb.u
    assert torch.equal(buf[lay["act_off"]:lay["act_off"] + A], nb.eps_act)


@pytest.mark.parametrize("task,ov,B,ev", [
    ("cartpole", dict(num_samples=64, num_elites=32, iterations=3), 1, False),
    ("humanoid", dict(num_samples=512, num_elites=64, iterations=6, horizon=5), 3, False),
    ("humanoid", dict(num_samples=512, num_elites=64, iterations=6, horizon=5), 2, True),
    ("dog", dict(num_samples=77, num_elites=13, iterations=3, horizon=4), 3, False),
    # no pi trajectories, and a randn(H,N,A) of 622,592 > 2048 x 256 values: ATen's grid-stride loop takes
    # two passes, elements past the first pass come from the 2nd normal4 and its components .y/.z/.w
    ("dog", dict(num_samples=2048, num_elites=64, mixture_coef=0.0, iterations=2, horizon=8), 2, False),
])
def test_reference_normals_one_launch(task, ov, B, ev):
    """tdmpc_reference_normals (one kernel for all of a call's draws, every env) writes bitwise the values of the
    reference's separate normal_ launches, and leaves torch's generator where those launches leave it."""
    cfg = make_cfg(task, **ov)
    pl = TDMPC(cfg, max_batch=B).planner
    H, I = cfg.horizon, cfg.iterations
    gen = torch.cuda.default_generators[0]
    torch.manual_seed(77)
    torch.randn(5, device="cuda")   # a nonzero starting offset
    for e in range(B):
        pl.draw_reference_torch(e, H, I, ev)
    want = pl.noise_view(H, I, B).clone()
    off_want = gen.get_offset()
    next_want = torch.randn(1000, device="cuda")
    pl.noise_flat.fill_(7.0)
    torch.manual_seed(77)
    torch.randn(5, device="cuda")
    pl.draw_reference_device(B, H, I, ev)
    got = pl.noise_view(H, I, B)
    assert gen.get_offset() == off_want
    assert torch.equal(torch.randn(1000, device="cuda"), next_want)
    if ev:   # the final action draw is not taken in eval mode: the slot is left alone
        A = pl.A
        assert (got[:, -A:] == 7.0).all()
        got, want = got[:, :-A], want[:, :-A]
    bad = (got != want).nonzero()
    assert bad.numel() == 0, f"{bad.shape[0]} of {got.numel()} differ, first at {bad[0].tolist()}"


@pytest.mark.parametrize("graph,B", [(True, 1), (False, 1), (True, 3)])
def test_plan_reference_draws_device_equals_torch(monkeypatch, graph, B):
    """plan() / plan_batch with the one-launch draws (the default: in the captured graph, the generator state
    staged through device memory) equals the same calls with the reference's own normal_ launches, bitwise, over
    warm-started calls, eval-mode calls and a reseed between calls; the generator ends in the same state."""
    cfg = make_cfg("humanoid", num_samples=512, num_elites=64, iterations=6, horizon=5)
    obs = np.random.RandomState(4).standard_normal((4, B, cfg.obs_shape[0])).astype(np.float32)
    outs = []
    for mode in ("device", "torch"):
        monkeypatch.setenv("TDMPC_REF_DRAWS", mode)
        agent = TDMPC(cfg, max_batch=B, graph=graph)
        agent.model.load_state_dict(synthetic_state_dict(cfg, 2))
        agent.std = 0.05
        assert agent.planner.ref_draws == mode
        torch.manual_seed(11)
        np.random.seed(11)
        res = []
        for k in range(4):
            if k == 2:
                torch.manual_seed(5)   # a new seed between calls reaches the staged generator state
            ev = k == 3
            if B == 1:
                a, m = agent.plan(obs[k, 0], eval_mode=ev, step=10**6, t0=(k == 0))
                res += [a.clone(), torch.tensor([m["external_reward_mean"], m["current_std"]])]
            else:
                a, m = agent.plan_batch(obs[k], eval_mode=ev, step=10**6, t0=(k == 0), sync_metrics=False)
                res += [a.clone(), m.clone()]
        res.append(torch.randn(4, device="cuda"))
        outs.append(res)
    for i, (x, y) in enumerate(zip(*outs)):
        assert torch.equal(x.cpu(), y.cpu()), f"output {i}: device {x[:3].tolist()} vs torch {y[:3].tolist()}"


@pytest.mark.parametrize("path", PATHS)
def test_plan_fullsize_vs_oracle(path):
    """Full humanoid-run plan (N=512, H=5, 6 iterations, T=768): GPU vs oracle on identical noise, warm
    start on the second call."""
    cfg = make_cfg("humanoid", num_samples=512, num_elites=64, iterations=6, horizon=5)
    agent = _agent(cfg, 9, path=path)
    told = tdmpc_ref.RefTOLD(synthetic_state_dict(cfg, 9), cfg)
    st = tdmpc_ref.PlanState(0.05)
    rs = np.random.RandomState(2)
    torch.manual_seed(4)
    np.random.seed(4)
    for call, t0 in enumerate([True, False]):
        obs = rs.standard_normal(cfg.obs_shape).astype(np.float32)
        nb = tdmpc_ref.draw_noise(cfg, 10**6, False)
        tr, rtr = {}, {}
        a, m = agent._plan_envs(obs[None], False, 10**6, [t0], trace=tr, noise=[nb])
        ra, rm = tdmpc_ref.plan(told, cfg, st, obs, nb, eval_mode=False, step=10**6, t0=t0, trace=rtr)
        ref_vals = torch.stack(rtr["value"]).squeeze(-1).numpy()
        same = _compare_iterations(tr["value"][0].cpu().numpy(), ref_vals, cfg.num_elites)
        record(same, f"fullsize/{path}/call{call}")
        if not same:
            break
        np.testing.assert_allclose(a[0].cpu().numpy(), ra.numpy(), atol=2e-5, rtol=0)
        np.testing.assert_allclose(tr["mean"][0, -1].cpu().numpy(), rtr["mean"][-1].numpy(), atol=2e-5, rtol=0)
        np.testing.assert_allclose(tr["std"][0, -1].cpu().numpy(), rtr["std"][-1].numpy(), atol=2e-5, rtol=0)


@pytest.mark.parametrize("path", PATHS)
def test_plan_ragged_vs_oracle(path):
    """Ragged shapes: N = 77 candidates (P = 38, T = 115 rows: partial 16- and 32-row blocks), K = 13, 3 envs in
    one call (rows of env e at e*T: blocks straddle envs), dog dims (A = 38: 10 action quads), vs the oracle."""
    cfg = make_cfg("dog", num_samples=77, num_elites=13, iterations=3, horizon=4)
    B = 3
    agent = _agent(cfg, 17, B=B, path=path)
    told = tdmpc_ref.RefTOLD(synthetic_state_dict(cfg, 17), cfg)
    rs = np.random.RandomState(8)
    obs = rs.standard_normal((B, cfg.obs_shape[0])).astype(np.float32)
    torch.manual_seed(3)
    np.random.seed(3)
    noises = [tdmpc_ref.draw_noise(cfg, 10**6, False) for _ in range(B)]
    tr = {}
    a, m = agent._plan_envs(obs, False, 10**6, [True] * B, trace=tr, noise=noises)
    for e in range(B):
        st, rtr = tdmpc_ref.PlanState(0.05), {}
        ra, rm = tdmpc_ref.plan(told, cfg, st, obs[e], noises[e], eval_mode=False, step=10**6, t0=True, trace=rtr)
        ref_vals = torch.stack(rtr["value"]).squeeze(-1).numpy()
        same = _compare_iterations(tr["value"][e].cpu().numpy(), ref_vals, cfg.num_elites)
        record(same, f"ragged/{path}/env{e}")
        if same:
            np.testing.assert_allclose(a[e].cpu().numpy(), ra.numpy(), atol=2e-5, rtol=0)


def test_bench_batch_vs_oracle():
    """The bench workload's shape: 8 humanoid envs in one plan_batch call (auto path: the row-block chain
    kernels at 4096 / 6144 rows), every env against the oracle on its own noise."""
    cfg = make_cfg("humanoid", num_samples=512, num_elites=64, iterations=6, horizon=5)
    B = 8
    agent = _agent(cfg, 13, B=B)
    told = tdmpc_ref.RefTOLD(synthetic_state_dict(cfg, 13), cfg)
    rs = np.random.RandomState(3)
    obs = rs.standard_normal((B, cfg.obs_shape[0])).astype(np.float32)
    torch.manual_seed(6)
    np.random.seed(6)
    noises = [tdmpc_ref.draw_noise(cfg, 10**6, False) for _ in range(B)]
    tr = {}
    a, m = agent._plan_envs(obs, False, 10**6, [True] * B, trace=tr, noise=noises)
    compared = 0
    for e in range(B):
        st = tdmpc_ref.PlanState(0.05)
        rtr = {}
        ra, rm = tdmpc_ref.plan(told, cfg, st, obs[e], noises[e], eval_mode=False, step=10**6, t0=True, trace=rtr)
        ref_vals = torch.stack(rtr["value"]).squeeze(-1).numpy()
        same = _compare_iterations(tr["value"][e].cpu().numpy(), ref_vals, cfg.num_elites)
        record(same, f"bench_batch/env{e}")
        if same:
            np.testing.assert_allclose(a[e].cpu().numpy(), ra.numpy(), atol=2e-5, rtol=0)
            compared += 1
    assert compared >= B // 2, "too many near-tie elite swaps to compare actions"


def test_bench_shape_b32_vs_oracle():
    """The bench line's exact workload: humanoid-run (N=512, H=5, 6 iterations) at 32 envs in one plan_batch call
    (auto path: 512 x6 chain workgroups per head, two co-resident per CU, the z0c first layer at t = 0, the cached
    pi-row terminal means), a cold call then a warm-started one, every env against the oracle on its own noise.
    At least B - 2 envs must run every comparison to the end on each call (near-tie escapes are counted too)."""
    cfg = make_cfg("humanoid", num_samples=512, num_elites=64, iterations=6, horizon=5)
    B = 32
    agent = _agent(cfg, 13, B=B)
    told = tdmpc_ref.RefTOLD(synthetic_state_dict(cfg, 13), cfg)
    states = [tdmpc_ref.PlanState(0.05) for _ in range(B)]
    rs = np.random.RandomState(31)
    torch.manual_seed(32)
    np.random.seed(32)
    live = list(range(B))                       # envs whose every comparison so far ran to the end
    for call, t0 in enumerate([True, False]):
        obs = rs.standard_normal((B, cfg.obs_shape[0])).astype(np.float32)
        noises = [tdmpc_ref.draw_noise(cfg, 10**6, False) for _ in range(B)]
        tr = {}
        a, m = agent._plan_envs(obs, False, 10**6, [t0] * B, trace=tr, noise=noises)
        a = a.cpu().numpy()
        pm = agent.planner.prev_mean_view(5, B).cpu().numpy()
        full = []
        for e in range(B):
            rtr = {}
            ra, rm = tdmpc_ref.plan(told, cfg, states[e], obs[e], noises[e], eval_mode=False, step=10**6, t0=t0,
                                    trace=rtr)
            if e not in live:
                continue
            ref_vals = torch.stack(rtr["value"]).squeeze(-1).numpy()
            same = _compare_iterations(tr["value"][e].cpu().numpy(), ref_vals, cfg.num_elites)
            record(same, f"bench_b32/call{call}/env{e}")
            if not same:
                continue
            np.testing.assert_allclose(a[e], ra.numpy(), atol=2e-5, rtol=0, err_msg=f"call {call} env {e}")
            np.testing.assert_allclose(tr["mean"][e, -1].cpu().numpy(), rtr["mean"][-1].numpy(), atol=2e-5, rtol=0)
            np.testing.assert_allclose(tr["std"][e, -1].cpu().numpy(), rtr["std"][-1].numpy(), atol=2e-5, rtol=0)
            np.testing.assert_allclose([m[e]["external_reward_mean"], m[e]["current_std"]],
                                       [rm["external_reward_mean"], rm["current_std"]], atol=2e-5, rtol=1e-4)
            np.testing.assert_allclose(pm[e], states[e].prev_mean.numpy(), atol=2e-5, rtol=0)
            full.append(e)
        need = len(live) - 2
        assert len(full) >= need, f"call {call}: {len(full)} of {len(live)} envs compared to the end"
        live = full


def test_graph_replay_equals_eager_batched():
    """B=8 humanoid through a captured HIP graph (the bench's mode: chain kernels on two streams, the side
    stream joining the capture through events) equals the same calls issued eagerly, bitwise."""
    cfg = make_cfg("humanoid", num_samples=512, num_elites=64, iterations=6, horizon=5)
    B = 8
    obs = np.random.RandomState(4).standard_normal((B, cfg.obs_shape[0])).astype(np.float32)
    outs = []
    for graph in (True, False):
        agent = TDMPC(cfg, max_batch=B, rng="fused", graph=graph)
        agent.model.load_state_dict(synthetic_state_dict(cfg, 2))
        agent.std = 0.05
        torch.manual_seed(11)
        res = []
        for call in range(3):
            a, m = agent.plan_batch(obs, step=10**6, t0=(call == 0), sync_metrics=False)
            res.append((a.clone(), m.clone()))
        outs.append(res)
    for (a1, m1), (a2, m2) in zip(*outs):
        assert torch.equal(a1, a2) and torch.equal(m1, m2)


def test_c_host_example():
    """examples/plan_c (built by __graft_entry__.build()): the C ABI from a plain C++ host -- sizes, packing,
    cold and warm tdmpc_plan on 32 humanoid envs -- runs and returns finite actions, inside [-1, 1] in eval mode."""
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples", "plan_c")
    assert os.path.exists(exe), "examples/plan_c missing: run __graft_entry__.build()"
    r = subprocess.run([exe, "32", "5"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "plan-steps/s" in r.stdout and "bad 0" in r.stdout, r.stdout


@pytest.mark.parametrize("path", ["layered", "chain32", "split"])
@pytest.mark.parametrize("task,ov", [("humanoid", dict(num_samples=128, num_elites=16, iterations=3)),
                                     ("cheetah", dict(num_samples=64, num_elites=8, iterations=2, mixture_coef=0.0))])
def test_building_blocks_compose_plan(task, ov, path):
    """The SURVEY §8b building blocks -- tdmpc_encode, tdmpc_pi_rollout, I x tdmpc_cem_iter, then the
    np.random.choice pick on the host -- reproduce the oracle's TDMPC.plan trace (tdmpc.py:113-163) for 2 envs:
    pi actions, per-iteration values, elite sets, scores, mean/std, reward mean and the action."""
    cfg = make_cfg(task, **ov)
    B, H = 2, 5
    agent = _agent(cfg, 9, B=B, path=path)
    pl = agent.planner
    pl.pack(agent.model)
    N, P, A, K, I = pl.N, pl.P, pl.A, cfg.num_elites, cfg.iterations
    T = N + P
    g = torch.Generator().manual_seed(4)
    obs = torch.randn(B, cfg.obs_shape[0], generator=g)
    eps_pi = torch.randn(B, H, P, A, generator=g)
    eps_cem = torch.randn(B, I, H, N, A, generator=g)
    eps_term = torch.randn(B, I, T, A, generator=g)
    eps_act = torch.randn(B, A, generator=g)
    us = [0.3, 0.85]
    told = tdmpc_ref.RefTOLD(synthetic_state_dict(cfg, 9), cfg)
    traces, refs = [], []
    for e in range(B):
        nb = tdmpc_ref.NoiseBundle(eps_pi=eps_pi[e] if P > 0 else None, eps_cem=list(eps_cem[e]),
                                   eps_term=list(eps_term[e]), u=us[e], eps_act=eps_act[e])
        tr = {}
        a, m = tdmpc_ref.plan(told, cfg, tdmpc_ref.PlanState(0.05), obs[e].numpy(), nb, step=10**6, t0=True, trace=tr)
        traces.append(tr)
        refs.append((a, m))

    z0 = pl.encode(obs)
    for e in range(B):
        assert _close(z0[e].cpu().numpy(), traces[e]["z0"].numpy()).all()
    pi = None
    if P > 0:
        pi = pl.pi_rollout(z0, eps_pi, H)
        for e in range(B):
            assert _close(pi[e].cpu().numpy(), traces[e]["pi_actions"].numpy()).all(), \
                np.abs(pi[e].cpu().numpy() - traces[e]["pi_actions"].numpy()).max()
    mean = torch.zeros(B, H, A, device=pl.device)
    std = torch.full((B, H, A), 2.0, device=pl.device)
    diverged = [False] * B
    for i in range(I):
        elite, score, value, rmean = pl.cem_iter(z0, pi, eps_cem[:, i], eps_term[:, i], mean, std, H)
        for e in range(B):
            if diverged[e]:
                continue
            tr = traces[e]
            rv = tr["value"][i][:, 0].numpy()
            gv = value[e].cpu().numpy()
            assert _close(gv, rv).all(), f"env {e} iteration {i}: max |dG| {np.abs(gv - rv).max():.3e}"
            ref_idx = tr["elite_idxs"][i].numpy()
            eg, er = _elites(gv, K), set(ref_idx.tolist())
            if eg != er:
                assert _near_tie(rv, eg, er, K)
                diverged[e] = True
                record(False, f"blocks/{task}/{path}/env{e}/iter{i}")
                continue
            ref_elite = tr["actions"][i][:, ref_idx].numpy()
            np.testing.assert_allclose(elite[e].cpu().numpy(), ref_elite, atol=2e-5, rtol=0)
            np.testing.assert_allclose(score[e].cpu().numpy(), tr["score"][i][:, 0].numpy(), atol=2e-5, rtol=1e-4)
            np.testing.assert_allclose(mean[e].cpu().numpy(), tr["mean"][i].numpy(), atol=2e-5, rtol=0)
            np.testing.assert_allclose(std[e].cpu().numpy(), tr["std"][i].numpy(), atol=2e-5, rtol=0)
            np.testing.assert_allclose(float(rmean[e]), tr["reward_mean"][i], atol=2e-5, rtol=1e-4)
    for e in range(B):
        if diverged[e]:
            continue
        record(True)
        # the output pick of tdmpc.py:152-158 on the host from the last iteration's score / elites / std
        j = tdmpc_ref.choice_index(score[e].cpu().numpy(), us[e])
        a = elite[e, 0, j].cpu() + std[e, 0].cpu() * eps_act[e]
        np.testing.assert_allclose(a.numpy(), refs[e][0].numpy(), atol=2e-5, rtol=0)


def test_x6_accuracy_matches_f32_mfma():
    """The x6 products (three-way bf16 split, fp32 accumulation) are as accurate as the exact f32 MFMA: at
    BASELINE size (humanoid, T = 768, H = 5) both paths' estimate_value G is compared with a float64 evaluation
    of the same TOLD, and the x6 error may not exceed twice the f32 MFMA error (+1e-6 absolute)."""
    cfg = make_cfg("humanoid", num_samples=512, num_elites=64)
    H = 5
    g = torch.Generator().manual_seed(5)
    outs = {}
    for path in ("chain32", "chain_x6"):
        agent = _agent(cfg, 13, path=path)
        pl = agent.planner
        pl.pack(agent.model)
        T, A, L = pl.T, cfg.action_dim, cfg.latent_dim
        g.manual_seed(5)
        z0 = torch.randn(1, L, generator=g)
        actions = torch.rand(1, H, T, A, generator=g) * 2 - 1
        eps = torch.randn(1, T, A, generator=g)
        v, _, _ = pl.estimate_value(z0, actions, eps, H)
        outs[path] = v[0].double().cpu().numpy()
    told = tdmpc_ref.RefTOLD(synthetic_state_dict(cfg, 13), cfg)
    told.sd = {k: t.double() for k, t in told.sd.items()}
    G64 = tdmpc_ref.estimate_value(told, cfg, z0.double().repeat(T, 1), actions[0].double(), H, eps[0].double())[0]
    G64 = G64[:, 0].numpy()
    e32 = np.abs(outs["chain32"] - G64).max()
    ex6 = np.abs(outs["chain_x6"] - G64).max()
    print(f"max |G - G_fp64|: f32 MFMA {e32:.3e}, x6 {ex6:.3e}")
    assert ex6 <= 2 * e32 + 1e-6, (e32, ex6)


@pytest.mark.parametrize("graph", [False, True])
def test_persist_timeout_raises(monkeypatch, graph):
    """The persistent one-env plan assumes its whole 256-workgroup grid is resident. With a debug knob one workgroup
    never arrives at the first hand-off, so every other one times out (bounded spin): the kernel ORs
    TDMPC_STATUS_P1_TIMEOUT into the caller's status word and plan() raises instead of returning the NaN action.
    The status is sticky until raised; the next healthy call plans normally."""
    cfg = make_cfg("humanoid", num_samples=512, num_elites=64, iterations=6, horizon=5)
    agent = TDMPC(cfg, path="persist", graph=graph)
    agent.model.load_state_dict(synthetic_state_dict(cfg, 9))
    agent.std = 0.05
    obs = np.random.RandomState(0).standard_normal(cfg.obs_shape).astype(np.float32)
    monkeypatch.setenv("TDMPC_P1_DEBUG_SKIP", "1")
    with pytest.raises(RuntimeError, match="timed out"):
        agent.plan(obs, step=10**6, t0=True)
    assert int(agent.planner.status.item()) == 0   # cleared when raised
    monkeypatch.delenv("TDMPC_P1_DEBUG_SKIP")
    agent.planner._graphs.clear()                  # (a captured graph keeps the knob's launch arguments)
    a, m = agent.plan(obs, step=10**6, t0=True)
    assert torch.isfinite(a).all() and np.isfinite(m["current_std"])


@pytest.mark.parametrize("graph", [False, True])
def test_persist_timeout_raises_without_sync(monkeypatch, graph):
    """The non-synchronising path (plan_batch(sync_metrics=False): the bench, EnvShardedPlanner's plan_fn) surfaces
    the sticky device status too: each call queues the word's copy behind an event and the call after next waits for
    it (no stream bubble) and raises; check_status() raises at once. Neither path hands on the NaN actions silently."""
    cfg = make_cfg("humanoid", num_samples=512, num_elites=64, iterations=6, horizon=5)
    agent = TDMPC(cfg, path="persist", graph=graph)
    agent.model.load_state_dict(synthetic_state_dict(cfg, 9))
    agent.std = 0.05
    obs = np.random.RandomState(0).standard_normal((1, *cfg.obs_shape)).astype(np.float32)
    monkeypatch.setenv("TDMPC_P1_DEBUG_SKIP", "1")
    a, m = agent.plan_batch(obs, step=10**6, t0=True, sync_metrics=False)   # failed on the device; no sync yet
    agent.plan_batch(obs, step=10**6, t0=True, sync_metrics=False)
    with pytest.raises(RuntimeError, match="timed out"):
        agent.plan_batch(obs, step=10**6, t0=True, sync_metrics=False)      # call 0's status, two calls later
    assert int(agent.planner.status.item()) == 0
    assert not torch.isfinite(a).all()
    agent.plan_batch(obs, step=10**6, t0=True, sync_metrics=False)
    with pytest.raises(RuntimeError, match="timed out"):
        agent.planner.check_status()                                        # the synchronising check
    monkeypatch.delenv("TDMPC_P1_DEBUG_SKIP")
    agent.planner._graphs.clear()
    for _ in range(3):
        a, m = agent.plan_batch(obs, step=10**6, t0=True, sync_metrics=False)
    agent.planner.check_status()
    assert torch.isfinite(a).all() and torch.isfinite(m).all()


def test_plan_returns_its_own_action():
    """plan() returns a tensor of its own (the reference returns a fresh `a`, tdmpc.py:160-163): the next call, which
    overwrites the planner's action buffer, leaves an earlier returned action untouched. The copy is enqueued right
    after the captured plan and before the metrics sync, so its value is the plan's action, bitwise."""
    cfg = make_cfg("humanoid", num_samples=512, num_elites=64, iterations=6, horizon=5)
    agent = TDMPC(cfg)
    agent.model.load_state_dict(synthetic_state_dict(cfg, 4))
    agent.std = 0.05
    rs = np.random.RandomState(2)
    a0, m0 = agent.plan(rs.standard_normal(cfg.obs_shape).astype(np.float32), step=10**6, t0=True)
    kept = a0.clone()
    assert torch.equal(a0, agent.planner.action[0])
    assert a0.data_ptr() != agent.planner.action.data_ptr()
    a1, m1 = agent.plan(rs.standard_normal(cfg.obs_shape).astype(np.float32), step=10**6, t0=False)
    torch.cuda.synchronize()
    assert torch.equal(a0, kept) and not torch.equal(a0, a1)
    assert torch.equal(a1, agent.planner.action[0])
    assert a0.shape == (cfg.action_dim,) and a0.is_contiguous()
    assert np.isfinite([m0["current_std"], m0["external_reward_mean"], m1["current_std"]]).all()


class _RefTOLDQ64(tdmpc_ref.RefTOLD):
    """The oracle TOLD with helper.q in float64 (the stress test's accuracy yardstick; every other head as is)."""

    def __init__(self, sd, cfg):
        super().__init__(sd, cfg)
        self.sd64 = {k: v.detach().to("cpu", torch.float64) for k, v in sd.items() if k.startswith("_Q")}

    def _q(self, x, pre):
        import torch.nn.functional as F
        m, s = self.cfg.mlp_dim, self.sd64
        x = F.linear(x.double(), s[pre + ".0.weight"], s[pre + ".0.bias"])
        x = torch.tanh(F.layer_norm(x, (m,), s[pre + ".1.weight"], s[pre + ".1.bias"], 1e-5))
        x = F.linear(x, s[pre + ".3.weight"], s[pre + ".3.bias"])
        x = F.elu(F.layer_norm(x, (m,), s[pre + ".4.weight"], s[pre + ".4.bias"], 1e-5))
        return F.linear(x, s[pre + ".6.weight"], s[pre + ".6.bias"]).float()


@pytest.mark.parametrize("stress", ["ln_shift", "ln_scale"])
def test_wide_heads_layernorm_stress_vs_oracle(stress):
    """The wide heads kernel's LayerNorm-1 comes from the pack's statistics block (var = |R [x; 1]|^2 / M) and a
    first layer with the mean and gain folded in (diag(g1) (W1 - 1 wbar^T)), not from the 512 layer-1
    outputs. Stressed here at the bench shape (32 humanoid envs, the wide step + wide heads kernels), every env:
    ln_shift puts the first Q layers' outputs far from zero mean (bias + 30 / - 20: |mean| ~ 10-30 sigma, where an
    E[y^2] - mean^2 variance would cancel), ln_scale shrinks their spread (weights x 1e-2: sigma ~ 1e-2, the LayerNorm
    eps 1e-5 matters) and randomises both LayerNorms' affine parameters.
    A stressed LayerNorm amplifies every fp32 rounding of its input by |y| / sigma, the reference's own included, so
    the yardstick is the oracle with helper.q in float64: iteration 0's 768 values (identical candidates on all
    sides) must be no further from it than 2x the fp32 oracle's own distance from it + the fp32 tolerance's 1e-5
    (the rollout before helper.q rounds differently too: x6 products vs the reference's fp32 GEMMs). Then every iteration
    is compared with the fp32 oracle while the elite sets agree, at the fp32 tolerance (parity_util: 1e-5 + 1e-4
    |ref|) widened by 4x that measured reference error (two fp32 evaluations each that far from exact)."""
    cfg = make_cfg("humanoid", num_samples=512, num_elites=64, iterations=6, horizon=5)
    B = 32
    sd = synthetic_state_dict(cfg, 17)
    g = torch.Generator().manual_seed(5)
    for q, sh in (("_Q1", 30.0), ("_Q2", -20.0)):
        if stress == "ln_shift":
            sd[f"{q}.0.bias"] = sd[f"{q}.0.bias"] + sh
        else:
            sd[f"{q}.0.weight"] = sd[f"{q}.0.weight"] * 1e-2
            sd[f"{q}.0.bias"] = sd[f"{q}.0.bias"] * 1e-2
        for ln in ("1", "4"):
            sd[f"{q}.{ln}.weight"] = 1.0 + 0.5 * torch.randn(sd[f"{q}.{ln}.weight"].shape, generator=g)
            sd[f"{q}.{ln}.bias"] = 0.3 * torch.randn(sd[f"{q}.{ln}.bias"].shape, generator=g)
    traces = {}
    for path in ("auto", "chain_x6"):   # auto: the wide step + wide heads kernels; chain_x6: the two-pass LayerNorms
        agent = TDMPC(cfg, max_batch=B, path=path)
        agent.model.load_state_dict(sd)
        agent.std = 0.05
        rs = np.random.RandomState(7)
        obs = rs.standard_normal((B, cfg.obs_shape[0])).astype(np.float32)
        torch.manual_seed(8)
        np.random.seed(8)
        noises = [tdmpc_ref.draw_noise(cfg, 10**6, False) for _ in range(B)]
        traces[path] = {}
        agent._plan_envs(obs, False, 10**6, [True] * B, trace=traces[path], noise=noises)
        del agent
    tr = traces["auto"]
    told = tdmpc_ref.RefTOLD(sd, cfg)
    told64 = _RefTOLDQ64(sd, cfg)
    full = 0
    errs = {"wide": [], "chain_x6": [], "ref_f32": []}
    for e in range(B):
        vals = {}
        for name, t in (("f32", told), ("f64", told64)):
            rtr = {}
            tdmpc_ref.plan(t, cfg, tdmpc_ref.PlanState(0.05), obs[e], noises[e], eval_mode=False, step=10**6, t0=True,
                           trace=rtr)
            vals[name] = torch.stack(rtr["value"]).squeeze(-1).numpy().astype(np.float64)
        gpu = tr["value"][e].cpu().numpy().astype(np.float64)
        ref_err = np.abs(vals["f32"][0] - vals["f64"][0]).max()
        gpu_err = np.abs(gpu[0] - vals["f64"][0]).max()
        chain_err = np.abs(traces["chain_x6"]["value"][e][0].cpu().numpy().astype(np.float64) - vals["f64"][0]).max()
        errs["wide"].append(float(gpu_err))
        errs["chain_x6"].append(float(chain_err))
        errs["ref_f32"].append(float(ref_err))
        assert gpu_err <= 2 * ref_err + ATOL, f"env {e}: |gpu - exact| {gpu_err:.3e} vs fp32 reference {ref_err:.3e}"
        same = True
        for i in range(vals["f32"].shape[0]):
            ok = _close(gpu[i], vals["f32"][i], atol=ATOL + 4 * ref_err)
            assert ok.all(), f"env {e} iteration {i}: max |dG| {np.abs(gpu[i] - vals['f32'][i]).max():.3e}"
            eg, er = set(np.argsort(-gpu[i], kind="stable")[:64]), set(np.argsort(-vals["f32"][i], kind="stable")[:64])
            if eg != er:
                assert _near_tie(vals["f32"][i], eg, er, 64), f"env {e} iteration {i}: elite sets differ off the cut"
                same = False
                break
        record(same, f"wide_heads_{stress}/env{e}")
        full += int(same)
    assert full >= B - 2, f"{full} of {B} envs compared to the end"
    # the statistics block against the two-pass LayerNorm on the same weights and candidates (iteration 0: every
    # row's value, max over its 768 rows, per env): kept as a record, and bounded in aggregate
    w, c = np.array(errs["wide"]), np.array(errs["chain_x6"])
    out = dict(stress=stress, per_env=errs, wide_max=float(w.max()), chain_x6_max=float(c.max()),
               wide_median=float(np.median(w)), chain_x6_median=float(np.median(c)),
               ref_f32_max=float(max(errs["ref_f32"])), median_ratio=float(np.median(w / np.maximum(c, 1e-12))))
    import json
    import os
    os.makedirs("gpurun_out", exist_ok=True)
    with open(f"gpurun_out/ln_stress_{stress}.json", "w") as f:
        json.dump(out, f, indent=1)
    print(f"ln stress {stress}: wide max {w.max():.3e} median {np.median(w):.3e} | chain_x6 max {c.max():.3e} "
          f"median {np.median(c):.3e} | fp32 reference max {max(errs['ref_f32']):.3e}")
    assert w.max() <= 1.5 * c.max(), f"statistics-block LayerNorm max error {w.max():.3e} > 1.5x two-pass {c.max():.3e}"
    assert np.median(w) <= 1.5 * np.median(c), f"median error {np.median(w):.3e} > 1.5x two-pass {np.median(c):.3e}"
