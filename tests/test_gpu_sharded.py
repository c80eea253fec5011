"""The product env-sharding path with more than one rank (SURVEY.md §8e, configs[3]: 64 vectorised dog-run envs):
two processes, each the real HIP `TDMPC` under `EnvShardedPlanner`'s default plan_fn (plan_batch of its 32-env
shard, HIP graph, reference-order device draws), one all-gather of [envs, A+2] per call. Both ranks share the one
GPU of the test box, so the collective runs on the gloo transport (RCCL refuses two ranks on one device); the
planning path is the one `bench.py --gpus N` runs per GPU. Every env's gathered action and metrics must equal,
bitwise, a single-process plan_batch over all 64 envs: envs are independent and N, T are multiples of the 128-row
block, so an env's arithmetic does not depend on its slot or on the batch size (every row of both batch sizes runs on
the same kernel at >= 32 envs per call: the wide step kernel for the sampled rows, the chain kernel for iteration 0's
policy rows -- the split is by a row's role, tdmpc_kernels.hip step_next)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

import shard_worker as W

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_world(tmp_path, world, *mode, backend="gloo"):
    port = _free_port()
    env = dict(os.environ, WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
               TDMPC_SHARD_BACKEND=backend)
    env.pop("TDMPC_P1_DEBUG_SKIP", None)
    here = os.path.dirname(os.path.abspath(__file__))
    procs = [subprocess.Popen([sys.executable, os.path.join(here, "shard_worker.py"), str(tmp_path), *mode],
                              env=dict(env, RANK=str(r), LOCAL_RANK=str(r)), stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT, text=True) for r in range(world)]
    for p in procs:
        try:
            out, _ = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        assert p.returncode == 0, out[-3000:]


def test_sharded_status_raises_on_every_rank(tmp_path):
    """ABI 6 through the sharded path (sync_metrics=False under the hood): rank 1's one-env persistent plan fails
    on the device (debug knob), its status word rides in the gathered block, and BOTH ranks raise from
    EnvShardedPlanner.plan at that call instead of handing on rank 1's NaN actions; the next call is healthy."""
    world = 2
    _run_world(tmp_path, world, "status")
    for r in range(world):
        raised, finite, st = open(os.path.join(tmp_path, f"status{r}.txt")).read().split("\n")[:3]
        assert "rank(s) [1]" in raised and "status 1" in raised, (r, raised)
        assert finite == "True" and st == "0", (r, finite, st)


def _check_against_single_process(tmp_path, world):
    got = [np.load(os.path.join(tmp_path, f"rank{r}.npz")) for r in range(world)]
    # single process, all 64 envs, same weights and generator states
    c = W.cfg()
    agent = W.TDMPC(c, max_batch=W.N_ENVS)
    agent.model.load_state_dict(W.synthetic_state_dict(c, W.WSEED))
    agent.std = 0.05
    H, I = agent.horizon(10**6), c.iterations
    for k, obs in enumerate(W.observations(c)):
        W.position_rngs(agent, 0, k, H, I)
        a, m = agent.plan_batch(obs, step=10**6, t0=(k == 0), sync_metrics=False)
        a, m = a.cpu().numpy(), m.cpu().numpy()
        assert np.isfinite(a).all()
        for r in range(world):   # every rank holds the whole gathered batch
            np.testing.assert_array_equal(got[r][f"a{k}"], a, err_msg=f"call {k} rank {r} actions")
            np.testing.assert_array_equal(got[r][f"m{k}"], m, err_msg=f"call {k} rank {r} metrics")


def test_sharded_dog64_world2_equals_single_process(tmp_path):
    world = 2
    _run_world(tmp_path, world)
    _check_against_single_process(tmp_path, world)


def test_sharded_dog64_rccl_world1_equals_single_process(tmp_path):
    """The RCCL ("nccl") branch of EnvShardedPlanner on hardware: one rank owning the box's GPU, the device-tensor
    all_gather_into_tensor over RCCL (parallel.py's nccl path, the one `bench.py --gpus N` takes under torchrun), the
    gathered batch bitwise equal to the single-process plan_batch. (Two ranks on one device are refused by RCCL, so
    the multi-rank exchange itself is covered by the gloo test above and tests/test_parallel_cpu.py.)"""
    _run_world(tmp_path, 1, backend="nccl")
    _check_against_single_process(tmp_path, 1)
    assert bool(np.load(os.path.join(tmp_path, "rank0.npz"))["gather_equal"])


def test_world1_deferred_status_raises_two_calls_late():
    """The deferred status path of EnvShardedPlanner (world 1 on the GPU; RCCL ranks take the same path after their
    gather): call 0's one-env persistent plan fails on the device (TDMPC_P1_DEBUG_SKIP), its actions come back NaN
    without a host sync, call 1 (healthy) returns finite actions, and call 2 raises from EnvShardedPlanner's own
    check -- before the agent's HipPlanner check, which it clears -- naming rank 0 and the status; the sticky word is
    cleared, so call 3 plans normally."""
    from tdmpc_amd import TDMPC, EnvShardedPlanner
    from tdmpc_amd.config import make_cfg
    from tdmpc_amd.told import synthetic_state_dict
    c = make_cfg("humanoid", num_samples=512, num_elites=64, iterations=6, horizon=5)
    agent = TDMPC(c, max_batch=1, path="persist")
    agent.model.load_state_dict(synthetic_state_dict(c, 13))
    agent.std = 0.05
    planner = EnvShardedPlanner(1, c.action_dim, agent=agent)
    assert planner.world == 1
    obs = torch.from_numpy(np.random.RandomState(3).standard_normal((1, c.obs_shape[0])).astype(np.float32))
    os.environ["TDMPC_P1_DEBUG_SKIP"] = "1"
    try:
        a0, _ = planner.plan(obs, 10**6, t0=True)
    finally:
        del os.environ["TDMPC_P1_DEBUG_SKIP"]
    agent.planner._graphs.clear()   # (the captured graph keeps the knob's launch arguments)
    assert not bool(torch.isfinite(a0).all())
    a1, _ = planner.plan(obs, 10**6, t0=True)
    assert bool(torch.isfinite(a1).all())
    with pytest.raises(RuntimeError, match=r"rank\(s\) \[0\] \(status 1\)"):
        planner.plan(obs, 10**6, t0=True)
    assert int(agent.planner.status.item()) == 0
    a3, _ = planner.plan(obs, 10**6, t0=True)
    torch.cuda.synchronize()
    assert bool(torch.isfinite(a3).all())
    planner.check_status()   # (nothing pending or set)
