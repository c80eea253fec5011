"""src/train.py's loop on the drop-in agent (reference: /root/reference/src/train.py:80-110): plan() (HIP graph,
reference-order RNG) -> buffer.add -> update() (the learner's captured HIP graph) -> plan() again. A replayed graph
writes the parameters in place without bumping their tensor versions, so the learner tells the planner to repack;
this test holds the next plan to the oracle evaluated on the agent's CURRENT weights."""
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from learner_io import learner_cfg
from oracle import tdmpc_ref
from tdmpc_amd.told import synthetic_state_dict


def _oracle_first_values(agent, cfg, obs, step):
    """First-iteration candidate values of a cold plan() traced on the GPU, and the oracle's on the same noise and
    the agent's current state_dict (the recipe of __graft_entry__.smoke)."""
    trace = {}
    std = float(agent.std)
    agent._plan_envs(obs[None], False, step, [True], trace=trace)
    pl = agent.planner
    H, I = agent.horizon(step), cfg.iterations
    lay = pl.noise_layout(H, I)
    buf = pl.noise_view(H, I, 1)[0].cpu()
    P, N, A, T = pl.P, pl.N, pl.A, pl.T
    nb = tdmpc_ref.NoiseBundle(eps_pi=buf[:H * P * A].view(H, P, A))
    for i in range(I):
        o = lay["cem_off"] + i * lay["iter"]
        nb.eps_cem.append(buf[o:o + H * N * A].view(H, N, A))
        nb.eps_term.append(buf[o + H * N * A:o + H * N * A + T * A].view(T, A))
    nb.u = float(pl.u[0].cpu())
    nb.eps_act = buf[lay["act_off"]:lay["act_off"] + A]
    sd = {k: v.detach().cpu() for k, v in agent.model.state_dict().items()}
    told = tdmpc_ref.RefTOLD(sd, cfg)
    ref_trace = {}
    tdmpc_ref.plan(told, cfg, tdmpc_ref.PlanState(std), obs, nb, eval_mode=False, step=step, t0=True,
                   trace=ref_trace)
    return trace["value"][0, 0].cpu(), ref_trace["value"][0].squeeze(1)


@pytest.mark.gpu
def test_train_loop_plans_with_updated_weights():
    from tdmpc_amd.replay import ReplayBuffer
    from tdmpc_amd.tdmpc import TDMPC
    cfg = learner_cfg()
    rc = SimpleNamespace(**{**vars(cfg), "device": "cuda", "train_steps": 2000, "max_buffer_size": 10**6,
                            "episode_length": 200, "env_horizon": cfg.horizon})
    rs = np.random.RandomState(3)
    agent = TDMPC(cfg)
    agent.model.load_state_dict(synthetic_state_dict(cfg, 41))
    agent.model_target.load_state_dict(synthetic_state_dict(cfg, 42))
    agent.learner(graph=True, warmup=2)
    buf = ReplayBuffer(rc, latent_plan=True)
    for _ in range(3):
        buf.add(SimpleNamespace(obs=torch.from_numpy(rs.standard_normal((201, 5)).astype(np.float32)),
                                action=torch.from_numpy(rs.uniform(-1, 1, (200, 1)).astype(np.float32)),
                                reward=torch.from_numpy(rs.standard_normal(200).astype(np.float32))))
    w0 = [p.detach().clone() for p in agent.model.parameters()]
    obs = rs.standard_normal(cfg.obs_shape).astype(np.float32)
    torch.manual_seed(0)
    np.random.seed(0)
    step = 10**6
    for k in range(6):
        a, m = agent.plan(obs, step=step, t0=(k == 0))
        assert torch.isfinite(a).all()   # (not clamped: the reference adds std * randn to the mean, tdmpc.py:161)
        agent.update(buf, k + 1)
    assert agent.learner()._graphs, "the learner never replayed its captured graph"
    assert any(not torch.equal(p, q) for p, q in zip(agent.model.parameters(), w0)), "no update reached the model"
    v_gpu, v_ref = _oracle_first_values(agent, cfg, obs, step)
    err = (v_gpu - v_ref).abs().max().item()
    assert err < 1e-4 * (1 + v_ref.abs().max().item()), f"plan after graph-replayed updates: max|dG| {err}"


@pytest.mark.gpu
def test_update_pi_then_plan_repacks():
    """TDMPC.update_pi (tdmpc.py:165-182) on the learner engine writes the policy weights in place (no tensor version
    bump); the next plan() must plan with them: its first-iteration values equal the oracle's on the agent's
    current weights (the planner kept the stale packed policy)."""
    from tdmpc_amd.tdmpc import TDMPC
    cfg = learner_cfg()
    agent = TDMPC(cfg)
    agent.model.load_state_dict(synthetic_state_dict(cfg, 43))
    agent.model_target.load_state_dict(synthetic_state_dict(cfg, 44))
    rs = np.random.RandomState(5)
    obs = rs.standard_normal(cfg.obs_shape).astype(np.float32)
    torch.manual_seed(1)
    np.random.seed(1)
    step = 10**6
    agent.plan(obs, step=step, t0=True)            # packs the initial weights
    pi0 = [p.detach().clone() for p in agent.model._pi.parameters()]
    g = torch.Generator(device="cuda").manual_seed(7)
    zs = [torch.randn(cfg.batch_size, cfg.latent_dim, device="cuda", generator=g) for _ in range(cfg.horizon + 1)]
    for _ in range(3):
        agent.update_pi(zs)
    assert any(not torch.equal(p, q) for p, q in zip(agent.model._pi.parameters(), pi0)), "update_pi changed nothing"
    v_gpu, v_ref = _oracle_first_values(agent, cfg, obs, step)
    err = (v_gpu - v_ref).abs().max().item()
    assert err < 1e-4 * (1 + v_ref.abs().max().item()), f"plan after update_pi: max|dG| {err}"


@pytest.mark.gpu
def test_live_repack_equals_full_pack():
    """The learner's captured update repacks the planner's weights from its flat parameter buffer (one fused
    tdmpc_pack_weights launch inside the graph, no state_dict walk): after graph-replayed updates the packed
    buffer is bitwise what a full pack of the agent's current state_dict writes."""
    from tdmpc_amd.replay import ReplayBuffer
    from tdmpc_amd.tdmpc import TDMPC, pack_told
    cfg = learner_cfg()
    rc = SimpleNamespace(**{**vars(cfg), "device": "cuda", "train_steps": 2000, "max_buffer_size": 10**6,
                            "episode_length": 200, "env_horizon": cfg.horizon})
    rs = np.random.RandomState(9)
    agent = TDMPC(cfg)
    agent.model.load_state_dict(synthetic_state_dict(cfg, 51))
    agent.model_target.load_state_dict(synthetic_state_dict(cfg, 52))
    lrn = agent.learner(graph=True, warmup=2)
    if lrn.engine is None:
        pytest.skip("learner engine not used for this config")
    buf = ReplayBuffer(rc, latent_plan=True)
    for _ in range(3):
        buf.add(SimpleNamespace(obs=torch.from_numpy(rs.standard_normal((201, 5)).astype(np.float32)),
                                action=torch.from_numpy(rs.uniform(-1, 1, (200, 1)).astype(np.float32)),
                                reward=torch.from_numpy(rs.standard_normal(200).astype(np.float32))))
    obs = rs.standard_normal(cfg.obs_shape).astype(np.float32)
    step = 10**6
    for k in range(6):
        agent.plan(obs, step=step, t0=(k == 0))
        agent.update(buf, k + 1)
    assert lrn._graphs and lrn._live_pack, "the captured update did not repack the planner itself"
    pl = agent.planner
    packed0 = pl.packed.clone()
    agent.update(buf, 7)                      # one more graph replay: its live repack changes the packed weights
    torch.cuda.synchronize()
    live = pl.packed.clone()
    assert not torch.equal(live, packed0)
    pl._packed_key = None                     # a full pack of the same (current) weights from the state_dict
    pack_told(pl, agent.model)
    torch.cuda.synchronize()
    assert torch.equal(pl.packed.view(torch.int32), live.view(torch.int32))
