"""GPU parity at BASELINE.json's full sizes for every GPU config, plus the drop-in's per-call state.

* `test_plan_fullsize_configs`: whole `plan()` calls (N=512, H=5, 6 iterations, K=64) for cheetah-run,
  humanoid-run with latent 512, quadruped-run pixels and dog-run, at one env per call (the drop-in) and at
  8 envs per call (configs[3]'s per-GPU share of 64 dog envs) and at the bench's 32 envs per call (the wide step
  and wide heads kernels, each config its own instance; latent 512: the wide step kernel with the folded first
  layer, helper.q on the chain kernel), cold start, warm start and
  a mixed t0 batch,
  every env against the oracle (the CPU restatement of tdmpc.py:94-163, pinned to the reference) on the same
  noise. Tolerances as tests/test_gpu_plan.py (parity_util): values 1e-5 + 1e-4 |ref|, action / mean / std /
  metrics 2e-5 while the elite sets agree; near-tie escapes are counted (tests/test_zz_parity_budget.py).
* `test_mixed_t0_batch_equals_homogeneous`: per-env warm/cold starts in one batch (tdmpc.py:124-125 per env)
  equal, bitwise, the same envs planned in all-warm and all-cold batches.
* `test_graph_serves_std_schedule`: one captured HIP graph serves every self.std of std_schedule and every
  t0 pattern (both read from device memory), bitwise equal to eager calls.
* `test_estimate_value_nonfinite`: the NaN / inf guard (`G.nan_to_num_(0)`, tdmpc.py:92: NaN -> 0,
  +-inf -> +-FLT_MAX) on every kernel path, including activations beyond bf16's range on the x6 products.
"""
import numpy as np
import pytest
import torch

from oracle import tdmpc_ref
from parity_util import close, compare_iterations, record
from tdmpc_amd.config import make_cfg
from tdmpc_amd.tdmpc import TDMPC
from tdmpc_amd.told import synthetic_state_dict

pytestmark = pytest.mark.gpu

FULL = dict(num_samples=512, num_elites=64, iterations=6, horizon=5)
CONFIGS = {
    "cheetah-run": ("cheetah", dict(FULL)),
    "humanoid-run-l512": ("humanoid", dict(FULL, latent_dim=512)),
    "quadruped-run-pixels": ("quadruped", dict(FULL, modality="pixels")),
    "dog-run": ("dog", dict(FULL)),
}
PATHS = ["layered", "chain16", "chain32", "split", "chain_x6", "split_x6", "chain", "persist", "wide"]


def _agent(cfg, wseed, B=1, path="auto", **kw):
    agent = TDMPC(cfg, max_batch=B, path=path, **kw)
    agent.model.load_state_dict(synthetic_state_dict(cfg, wseed))
    agent.std = 0.05
    return agent


def _obs(cfg, rs, B):
    if cfg.modality == "pixels":
        return rs.randint(0, 256, size=(B,) + tuple(cfg.obs_shape)).astype(np.uint8)
    return rs.standard_normal((B,) + tuple(cfg.obs_shape)).astype(np.float32)


@pytest.mark.parametrize("B", [1, 8, 32])
@pytest.mark.parametrize("name", list(CONFIGS))
def test_plan_fullsize_configs(name, B):
    task, ov = CONFIGS[name]
    cfg = make_cfg(task, **ov)
    agent = _agent(cfg, 21, B=B)
    told = tdmpc_ref.RefTOLD(synthetic_state_dict(cfg, 21), cfg)
    states = [tdmpc_ref.PlanState(0.05) for _ in range(B)]
    diverged = [False] * B        # an env whose elite set swapped on a near tie is not compared while warm
    rs = np.random.RandomState(5)
    torch.manual_seed(8)
    np.random.seed(8)
    calls = [[True] * B, [False] * B]
    if B > 1:
        calls.append([e % 2 == 0 for e in range(B)])   # mixed: even envs restart, odd envs warm-start
    for ci, t0s in enumerate(calls):
        obs = _obs(cfg, rs, B)
        noises = [tdmpc_ref.draw_noise(cfg, 10**6, False) for _ in range(B)]
        tr = {}
        a, m = agent._plan_envs(obs, False, 10**6, t0s, trace=tr, noise=noises)
        a = a.cpu().numpy()
        for e in range(B):
            rtr = {}
            ra, rm = tdmpc_ref.plan(told, cfg, states[e], obs[e], noises[e], eval_mode=False, step=10**6,
                                    t0=t0s[e], trace=rtr)
            if t0s[e]:
                diverged[e] = False
            if diverged[e]:
                continue
            ref_vals = torch.stack(rtr["value"]).squeeze(-1).numpy()
            same = compare_iterations(tr["value"][e].cpu().numpy(), ref_vals, cfg.num_elites)
            record(same, f"{name}/B{B}/call{ci}/env{e}")
            if not same:
                diverged[e] = True
                continue
            np.testing.assert_allclose(a[e], ra.numpy(), atol=2e-5, rtol=0, err_msg=f"call {ci} env {e}")
            np.testing.assert_allclose(tr["mean"][e, -1].cpu().numpy(), rtr["mean"][-1].numpy(), atol=2e-5, rtol=0)
            np.testing.assert_allclose(tr["std"][e, -1].cpu().numpy(), rtr["std"][-1].numpy(), atol=2e-5, rtol=0)
            np.testing.assert_allclose([m[e]["external_reward_mean"], m[e]["current_std"]],
                                       [rm["external_reward_mean"], rm["current_std"]], atol=2e-5, rtol=1e-4)
            pm = agent.planner.prev_mean_view(5, B)[e].cpu().numpy()
            np.testing.assert_allclose(pm, states[e].prev_mean.numpy(), atol=2e-5, rtol=0)
    if B == 32:   # the kernels that ran: the wide ones where the bench runs them (latent 512: the wide step kernel
        # with the streamed x and the folded first layer; helper.q stays on the chain kernel -- its statistics block
        # does not fit at 534 columns)
        step_k, q_k = _kernel_of(agent, cfg, 4), _kernel_of(agent, cfg, 6)
        l512 = name == "humanoid-run-l512"
        assert step_k.startswith("wide_step_kernel<17, 32" if l512 else "wide_step_kernel"), step_k
        assert q_k.startswith("chain_kernel" if l512 else "wide_heads_kernel"), q_k


def test_latent512_folded_rollout_accuracy():
    """Latent 512 at the bench shape (32 envs): the sampled rows roll out on the wide step kernel through the folded
    first layer [W1a | W1z W3] [a; h2] + (b1 + W1z b3) -- z' is not formed between steps, only at the last
    (DESIGN.md §4). Iteration 0's 768 values of 4 envs against a float64 evaluation of the same TOLD on the same
    candidates from the same z0: the folded rollout's error may not exceed twice the fp32 reference's own
    (+2e-6: the GPU also starts from its own fp32 encoder output), i.e. skipping the reference's rounding of z'
    costs no accuracy."""
    name = "humanoid-run-l512"
    task, ov = CONFIGS[name]
    cfg = make_cfg(task, **ov)
    B, H = 32, cfg.horizon
    sd = synthetic_state_dict(cfg, 21)
    agent = _agent(cfg, 21, B=B)
    assert _kernel_of(agent, cfg, 4).startswith("wide_step_kernel<17, 32")
    told = tdmpc_ref.RefTOLD(sd, cfg)
    told64 = tdmpc_ref.RefTOLD(sd, cfg)
    told64.sd = {k: t.double() for k, t in told64.sd.items()}
    rs = np.random.RandomState(3)
    obs = _obs(cfg, rs, B)
    torch.manual_seed(4)
    np.random.seed(4)
    noises = [tdmpc_ref.draw_noise(cfg, 10**6, False) for _ in range(B)]
    tr = {}
    agent._plan_envs(obs, False, 10**6, [True] * B, trace=tr, noise=noises)
    for e in range(4):
        rtr = {}
        tdmpc_ref.plan(told, cfg, tdmpc_ref.PlanState(0.05), obs[e], noises[e], eval_mode=False, step=10**6, t0=True,
                       trace=rtr)
        acts = rtr["actions"][0].double()
        z0 = rtr["z0"].double().unsqueeze(0).repeat(acts.shape[1], 1)
        G64 = tdmpc_ref.estimate_value(told64, cfg, z0, acts, H, noises[e].eps_term[0].double())[0][:, 0].numpy()
        e32 = np.abs(rtr["value"][0][:, 0].double().numpy() - G64).max()
        eg = np.abs(tr["value"][e][0].double().cpu().numpy() - G64).max()
        print(f"env {e}: max |G - G_fp64|: fp32 reference {e32:.3e}, folded wide rollout {eg:.3e}")
        assert eg <= 2 * e32 + 2e-6, (e, e32, eg)


def _kernel_of(agent, cfg, prof_cfg):
    """Name of the kernel the library's profiler (tdmpc_profile_begin cfg: 4 the step launches, 6 helper.q) timed
    over one eager plan of the agent's batch."""
    import ctypes as C
    from tdmpc_amd import _lib
    L = _lib.lib()
    B = agent.planner.max_batch if hasattr(agent.planner, "max_batch") else 32
    obs = _obs(cfg, np.random.RandomState(1), B)
    graph, agent.graph = agent.graph, False
    try:
        _lib.check(L.tdmpc_profile_begin(prof_cfg, -1, 0, 0, 256), "profile_begin")
        agent.plan_batch(obs, step=10**6, t0=False, sync_metrics=False)
        n, ms, fl = C.c_int32(), C.c_double(), C.c_double()
        _lib.check(L.tdmpc_profile_end(C.byref(n), C.byref(ms), C.byref(fl)), "profile_end")
    finally:
        agent.graph = graph
    assert n.value > 0, prof_cfg
    return L.tdmpc_profile_kernel().decode()


@pytest.mark.parametrize("path", ["auto", "chain_x6", "layered"])
def test_mixed_t0_batch_equals_homogeneous(path):
    """A batch mixing warm and cold starts equals, env by env and bitwise, the same batch planned all-warm or
    all-cold from the same previous means (same batch shape, so the same kernels run)."""
    cfg = make_cfg("dog", **FULL)
    B = 4
    agent = _agent(cfg, 23, B=B, path=path)
    pl = agent.planner
    rs = np.random.RandomState(9)
    obs0, obs1 = _obs(cfg, rs, B), _obs(cfg, rs, B)
    torch.manual_seed(2)
    n0 = [tdmpc_ref.draw_noise(cfg, 10**6, False) for _ in range(B)]
    n1 = [tdmpc_ref.draw_noise(cfg, 10**6, False) for _ in range(B)]
    agent._plan_envs(obs0, False, 10**6, [True] * B, noise=n0)
    prev = pl.prev_mean_flat.clone()
    outs = {}
    for key, t0s in (("mixed", [True, False, False, True]), ("cold", [True] * B), ("warm", [False] * B)):
        pl.prev_mean_flat.copy_(prev)
        a, m = agent._plan_envs(obs1, False, 10**6, t0s, sync_metrics=False, noise=n1)
        outs[key] = (a.clone(), m.clone(), pl.prev_mean_flat.clone())
    HA = 5 * cfg.action_dim
    for e, t0 in enumerate([True, False, False, True]):
        ref = outs["cold" if t0 else "warm"]
        assert torch.equal(outs["mixed"][0][e], ref[0][e]), e
        assert torch.equal(outs["mixed"][1][e], ref[1][e]), e
        assert torch.equal(outs["mixed"][2][e * HA:(e + 1) * HA], ref[2][e * HA:(e + 1) * HA]), e
    assert not torch.equal(outs["cold"][0], outs["warm"][0])   # the warm start did change something


def test_graph_serves_std_schedule():
    """graph=True: std_schedule moves self.std on every update (tdmpc.py:196-197) and t0 changes per env; both
    live in device memory, so ONE captured graph serves all calls, and each call equals an eager call."""
    cfg = make_cfg("humanoid", **FULL)
    B = 4
    obs = np.random.RandomState(4).standard_normal((B, cfg.obs_shape[0])).astype(np.float32)
    schedule = [(0.5, [True] * B), (0.4, [True, False, False, True]), (0.3, [False] * B), (0.05, [False, True] * 2)]
    outs = []
    for graph in (True, False):
        agent = _agent(cfg, 2, B=B, rng="fused", graph=graph)
        torch.manual_seed(11)
        res = []
        for std, t0s in schedule:
            agent.std = std
            a, m = agent.plan_batch(obs, step=10**6, t0=t0s, sync_metrics=False)
            res.append((a.clone(), m.clone()))
            assert bool((m[:, 1] >= np.float32(std) * (1 - 1e-6)).all()), "the CEM std floor (self.std) was not applied"
        outs.append(res)
        if graph:
            assert len(agent.planner._graphs) == 1, list(agent.planner._graphs)
    for (a1, m1), (a2, m2) in zip(*outs):
        assert torch.equal(a1, a2) and torch.equal(m1, m2)


FMAX = float(np.finfo(np.float32).max)


def _nf_case(case, sd, z0):
    """Weights / start latents that drive estimate_value outside the finite range."""
    if case == "beyond_bf16":
        # a latent above bf16's largest value (3.3895e38; rounds to inf in bf16) whose products stay finite:
        # the x6 split must keep it finite (truncated top half + exact residual)
        # (column weights ~1e-29: their bf16 mid / lo parts stay normal numbers, so the x6 products are exact)
        z0[:, 3] = 3.4e38
        for k in ("_dynamics.0.weight", "_reward.0.weight"):
            sd[k][:, 3] *= 1e-28
    elif case == "inf_latent":
        z0[:, 3] = float("inf")
    elif case == "nan_latent":
        z0[:, 3] = float("nan")
    elif case == "reward_pos_overflow":
        sd["_reward.4.bias"][:] = 3e38            # G overflows to +inf -> +FLT_MAX
    elif case == "reward_neg_overflow":
        sd["_reward.4.bias"][:] = -3e38           # -> -FLT_MAX
    elif case == "inf_minus_inf":
        sd["_reward.4.bias"][:] = 3e38
        sd["_Q1.6.bias"][:] = float("-inf")
        sd["_Q2.6.bias"][:] = float("-inf")       # +inf + -inf = NaN -> 0
    elif case == "large_finite":
        sd["_reward.4.weight"].mul_(3e37)         # |G| ~ 1e37, finite
    elif case == "inf_hidden":
        # an infinite HIDDEN activation: reward unit 5's layer-1 bias is +inf, so h1[5] = ELU(+inf) = +inf
        # on every row; with W2[:, 5] > 0 every layer-2 unit is +inf and with w3 > 0 the reward is +inf: fp32 gives
        # G = +inf -> +FLT_MAX (tdmpc.py:92). The x6 products must keep w * inf = +inf (no 0 * inf from a weight's
        # zero mid / lo part, no inf - inf from a negative mid part)
        sd["_reward.0.bias"][5] = float("inf")
        sd["_reward.2.weight"][:, 5] = sd["_reward.2.weight"][:, 5].abs() + 1e-3
        sd["_reward.4.weight"][:] = sd["_reward.4.weight"].abs() + 1e-3
    elif case == "inf_hidden_rows":
        # the same through overflow, on SOME rows only: reward unit 5 sees 3e38 * (a_0 + a_1), which overflows to +inf
        # where a_0 + a_1 > ~1.13 (then G = +FLT_MAX) and stays finite (or ELU -> -1) elsewhere; W2[:, 5] ~ 1e-31 > 0
        # keeps the finite rows' rewards ~1e8
        L = sd["_reward.0.weight"].shape[1] - sd["_pi.4.weight"].shape[0]   # cat[z, a]: a starts at column L
        sd["_reward.0.weight"][5, L] = 3e38
        sd["_reward.0.weight"][5, L + 1] = 3e38
        sd["_reward.2.weight"][:, 5] = (sd["_reward.2.weight"][:, 5].abs() + 1e-3) * 1e-30
        sd["_reward.4.weight"][:] = sd["_reward.4.weight"].abs() + 1e-3


NF_CASES = ["beyond_bf16", "inf_latent", "nan_latent", "reward_pos_overflow", "reward_neg_overflow", "inf_minus_inf",
            "large_finite", "inf_hidden", "inf_hidden_rows"]


@pytest.mark.parametrize("case", NF_CASES)
@pytest.mark.parametrize("path", PATHS)
def test_estimate_value_nonfinite(case, path):
    cfg = make_cfg("humanoid", num_samples=512, num_elites=64)
    H = 5
    sd = synthetic_state_dict(cfg, 7)
    g = torch.Generator().manual_seed(3)
    z0 = torch.randn(1, cfg.latent_dim, generator=g)
    _nf_case(case, sd, z0)
    agent = TDMPC(cfg, path=path)
    agent.model.load_state_dict(sd)
    pl = agent.planner
    pl.pack(agent.model)
    T, A = pl.T, cfg.action_dim
    actions = torch.rand(1, H, T, A, generator=g) * 2 - 1
    eps = torch.randn(1, T, A, generator=g)
    v, _, _ = pl.estimate_value(z0, actions, eps, H)
    gv = v[0].cpu().numpy()
    told = tdmpc_ref.RefTOLD(sd, cfg)
    rv = tdmpc_ref.estimate_value(told, cfg, z0.repeat(T, 1), actions[0], H, eps[0])[0][:, 0].numpy()
    assert np.isfinite(gv).all(), "nan_to_num left a non-finite value"
    special = (np.abs(rv) == FMAX) | (rv == 0)
    np.testing.assert_array_equal(gv[special], rv[special])
    # large_finite / beyond_bf16: G sums five rewards of ~1e37 / ~1e5 that partly cancel, so its rounding error
    # follows the terms' scale, not |G|: absolute tolerance 1e-5 of the largest |G| there
    atol = 1e-5 * float(np.abs(rv).max()) if case in ("large_finite", "beyond_bf16") else 1e-5
    assert close(gv[~special], rv[~special], atol=atol).all(), np.abs(gv - rv)[~special].max()
    if case in ("reward_pos_overflow", "reward_neg_overflow", "inf_minus_inf", "nan_latent", "inf_latent", "inf_hidden"):
        assert special.all()   # the case does hit the guard's branches
    if case == "inf_hidden":
        assert (rv == FMAX).all()   # +inf -> +FLT_MAX on every row (not NaN -> 0)
    if case == "inf_hidden_rows":
        assert (rv == FMAX).any() and not special.all()   # a mix of overflowed and finite rows
    if case in ("beyond_bf16", "large_finite"):
        assert not special.any()


@pytest.mark.parametrize("case", ["inf_hidden", "inf_hidden_rows"])
@pytest.mark.parametrize("path", ["persist", "auto", "chain_x6"])
def test_plan_nonfinite_hidden(case, path):
    """A whole plan() (one env: the persistent kernel on path persist / auto) with an infinite hidden activation:
    the first CEM iteration's values equal the oracle's -- +FLT_MAX on the overflowed rows, the rest within the
    tolerance. (Later iterations pick elites among +FLT_MAX ties, whose order torch.topk leaves open.)"""
    cfg = make_cfg("humanoid", **FULL)
    sd = synthetic_state_dict(cfg, 7)
    _nf_case(case, sd, torch.zeros(1, cfg.latent_dim))
    agent = TDMPC(cfg, path=path)
    agent.model.load_state_dict(sd)
    agent.std = 0.05
    told = tdmpc_ref.RefTOLD(sd, cfg)
    obs = np.random.RandomState(1).standard_normal(cfg.obs_shape).astype(np.float32)
    torch.manual_seed(2)
    np.random.seed(2)
    nb = tdmpc_ref.draw_noise(cfg, 10**6, False)
    tr, rtr = {}, {}
    agent._plan_envs(obs[None], False, 10**6, [True], trace=tr, noise=[nb])
    tdmpc_ref.plan(told, cfg, tdmpc_ref.PlanState(0.05), obs, nb, eval_mode=False, step=10**6, t0=True, trace=rtr)
    gv = tr["value"][0, 0].cpu().numpy()
    rv = rtr["value"][0][:, 0].numpy()
    assert np.isfinite(gv).all()
    special = (np.abs(rv) == FMAX) | (rv == 0)
    np.testing.assert_array_equal(gv[special], rv[special])
    assert close(gv[~special], rv[~special]).all(), np.abs(gv - rv)[~special].max()
    assert (rv == FMAX).any()


def test_default_plan_graph_equals_eager():
    """TDMPC(cfg) replays plan() from a HIP graph by default (reference-order draws captured with it): the drop-in
    call gives, bitwise, what the eager launches give on the same torch / numpy seeds, over t0, warm starts,
    eval mode and a std_schedule change."""
    cfg = make_cfg("humanoid", **FULL)
    obs = np.random.RandomState(6).standard_normal((4,) + tuple(cfg.obs_shape)).astype(np.float32)
    calls = [(0, True, False, 0.5), (1, False, False, 0.4), (2, False, True, 0.4), (3, True, False, 0.05),
             (4, False, False, 0.05)]
    outs = []
    for graph in (True, False):
        agent = TDMPC(cfg, graph=graph)
        agent.model.load_state_dict(synthetic_state_dict(cfg, 4))
        torch.manual_seed(3)
        np.random.seed(3)
        res = []
        for i, t0, ev, std in calls:
            agent.std = std
            a, m = agent.plan(obs[i % 4], eval_mode=ev, step=10**6, t0=t0)
            res.append((a.cpu(), m))
        outs.append(res)
        assert graph == (len(agent.planner._graphs) == 2)   # (eval_mode False, True)
    for (a1, m1), (a2, m2) in zip(*outs):
        assert torch.equal(a1, a2) and m1 == m2


@pytest.mark.parametrize("case", NF_CASES)
def test_plan_wide_nonfinite(case):
    """The non-finite cases of test_estimate_value_nonfinite through the whole plan at the bench shape (32 humanoid
    envs: the wide step and wide heads kernels, the statistics-block LayerNorm included), where estimate_value's
    entry point does not reach the wide heads. A start-latent case sets the encoder's last bias (z0 = h(obs) then
    carries the value in column 3 for every env). Iteration 0's 768 values of every env (the same candidates on
    both sides) against the oracle's: exactly where the oracle's are nan_to_num's specials (0, +-FLT_MAX),
    elsewhere within 1e-5 (of the largest |G| for the large cases)."""
    cfg = make_cfg("humanoid", **FULL)
    B = 32
    sd = synthetic_state_dict(cfg, 7)
    z0 = torch.zeros(1, cfg.latent_dim)
    _nf_case(case, sd, z0)
    if case in ("beyond_bf16", "inf_latent", "nan_latent"):
        sd["_encoder.2.bias"][3] = z0[0, 3]
    agent = TDMPC(cfg, max_batch=B)
    agent.model.load_state_dict(sd)
    agent.std = 0.05
    told = tdmpc_ref.RefTOLD(sd, cfg)
    rs = np.random.RandomState(4)
    obs = rs.standard_normal((B, cfg.obs_shape[0])).astype(np.float32)
    torch.manual_seed(8)
    np.random.seed(8)
    noises = [tdmpc_ref.draw_noise(cfg, 10**6, False) for _ in range(B)]
    tr = {}
    agent._plan_envs(obs, False, 10**6, [True] * B, trace=tr, noise=noises)
    for e in range(B):
        rtr = {}
        tdmpc_ref.plan(told, cfg, tdmpc_ref.PlanState(0.05), obs[e], noises[e], eval_mode=False, step=10**6, t0=True,
                       trace=rtr)
        rv = rtr["value"][0].squeeze(-1).numpy()
        gv = tr["value"][e][0].cpu().numpy()
        assert np.isfinite(gv).all(), f"env {e}: nan_to_num left a non-finite value"
        special = (np.abs(rv) == FMAX) | (rv == 0)
        np.testing.assert_array_equal(gv[special], rv[special], err_msg=f"env {e}")
        atol = 1e-5 * float(np.abs(rv).max()) if case in ("large_finite", "beyond_bf16") else 1e-5
        assert close(gv[~special], rv[~special], atol=atol).all(), (e, np.abs(gv - rv)[~special].max())
