"""Multi-process coverage of the env-sharded path on CPU (gloo, world_size 2 and 4).

Each rank plans its shard of a vectorised batch with the oracle's restatement of the reference plan() (CPU)
and all-gathers the results; the gathered batch must equal a single-process run over all envs with the same
per-env noise (bitwise: every env's computation is identical). Weight broadcast is checked too.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tdmpc_amd.config import make_cfg
from tdmpc_amd.parallel import EnvShardedPlanner, shard_bounds
from tdmpc_amd.told import TOLD, synthetic_state_dict

N_ENVS = 4


def _cfg():
    return make_cfg("cartpole", num_samples=32, num_elites=8, iterations=2, horizon=3, device="cpu")


def _env_noise(cfg, e):
    from oracle import tdmpc_ref
    torch.manual_seed(100 + e)
    np.random.seed(200 + e)
    return tdmpc_ref.draw_noise(cfg, 10**6, False)


def _oracle_plan_fn(cfg, sd, lo):
    from oracle import tdmpc_ref
    told = tdmpc_ref.RefTOLD(sd, cfg)

    def plan(obs, step, t0):
        acts, mets = [], []
        for i in range(obs.shape[0]):
            st = tdmpc_ref.PlanState(0.05)
            a, m = tdmpc_ref.plan(told, cfg, st, obs[i].numpy(), _env_noise(cfg, lo + i), step=step, t0=t0)
            acts.append(a)
            mets.append(torch.tensor([m["external_reward_mean"], m["current_std"]], dtype=torch.float32))
        return torch.stack(acts), torch.stack(mets)
    return plan


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, obs, out_q):
    try:
        _worker_body(rank, world, port, obs, out_q)
    except Exception as e:  # report instead of leaving the parent waiting
        out_q.put((rank, None, None, repr(e)))
        raise


def _worker_body(rank, world, port, obs, out_q):
    torch.set_num_threads(1)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        cfg = _cfg()
        sd = synthetic_state_dict(cfg, 3)
        lo, _ = shard_bounds(N_ENVS, rank, world)
        pl = EnvShardedPlanner(N_ENVS, cfg.action_dim, plan_fn=_oracle_plan_fn(cfg, sd, lo), device="cpu")
        a, m = pl.plan(obs, 10**6, True)
        # weight broadcast: rank 1 starts from different weights and must end equal to rank 0's
        model = TOLD(cfg, init="none")
        model.load_state_dict(synthetic_state_dict(cfg, 3 if rank == 0 else 4))
        pl.broadcast_weights(model, src=0)
        same = all(torch.equal(v, synthetic_state_dict(cfg, 3)[k]) for k, v in model.state_dict().items())
        # numpy, not tensors: torch's queue shares tensor storage through file descriptors that vanish when
        # this worker exits before the parent has received them
        out_q.put((rank, a.numpy().copy(), m.numpy().copy(), same))
    finally:
        dist.destroy_process_group()


def test_shard_bounds():
    assert [shard_bounds(8, r, 4) for r in range(4)] == [(0, 2), (2, 4), (4, 6), (6, 8)]
    assert [shard_bounds(5, r, 2) for r in range(2)] == [(0, 3), (3, 5)]


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_plan_gloo(world):
    """world 4 rehearses more ranks than the 2 the GPU tests run (one env per rank here)."""
    cfg = _cfg()
    rs = np.random.RandomState(0)
    obs = torch.from_numpy(rs.standard_normal((N_ENVS,) + tuple(cfg.obs_shape)).astype(np.float32))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, obs, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for r in res:
        assert r[1] is not None, f"rank {r[0]} failed: {r[3]}"
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single-process reference over all envs
    sd = synthetic_state_dict(cfg, 3)
    a_ref, m_ref = _oracle_plan_fn(cfg, sd, 0)(obs, 10**6, True)
    for rank, a, m, same in res:
        assert same, f"rank {rank} weights not synchronised"
        assert torch.equal(torch.from_numpy(a), a_ref), rank
        assert torch.equal(torch.from_numpy(m), m_ref), rank


def _bench_worker(rank, world, port, out_q):
    try:
        import time as _t
        import bench
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        calls = []

        def step(i):   # rank 1 is the slow one
            calls.append(i)
            _t.sleep(0.002 * (1 + rank))

        el = bench.time_steps(step, 2, 5, dist)
        el_max, value = bench.job_rate(el, 3 * 5, dist, torch.device("cpu"))
        out_q.put((rank, calls, el, el_max, value))
        dist.destroy_process_group()
    except Exception as e:
        out_q.put((rank, repr(e), None, None, None))


def test_bench_timing_contract_gloo_world2():
    """bench.py's multi-rank contract (the driver's N > 1 runs): W untimed + exactly K timed steps per rank between
    barriers, the slowest rank's time (MAX over ranks) on every rank, value = all ranks' units / that time."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_bench_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    for _ in range(world):
        r = q.get(timeout=120)
        res[r[0]] = r
    for p in ps:
        p.join(timeout=60)
    for r in range(world):
        assert isinstance(res[r][1], list), res[r][1]
        assert res[r][1] == list(range(7))            # 2 warm-up + 5 timed steps, in order
    el_max = max(res[r][2] for r in range(world))
    for r in range(world):
        assert res[r][3] == pytest.approx(el_max)      # every rank reports the slowest rank's time
        assert res[r][4] == pytest.approx(world * 3 * 5 / el_max)
    assert res[1][2] >= 5 * 0.004                      # rank 1's own timed region holds its slower steps
