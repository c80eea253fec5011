"""CPU checks of the drop-in boundary (no GPU): the import lines INTEGRATION.md documents, and the default
`EnvShardedPlanner` path over a real `tdmpc_amd.TDMPC` (seed-step branch, per-env t0 slicing, gloo world 2)."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def test_integration_import_lines():
    """`from tdmpc_amd import TDMPC` (src/train.py:80) and the rest of the swapped names."""
    from tdmpc_amd import TDMPC, TOLD, ReplayBuffer, TdICEM, EnvShardedPlanner, load_checkpoint  # noqa: F401
    import tdmpc_amd
    for name in tdmpc_amd.__all__:
        assert getattr(tdmpc_amd, name) is not None, name
    from tdmpc_amd.replay import ReplayBuffer as RB
    from tdmpc_amd.icem import TdICEM as TI
    assert RB is ReplayBuffer and TI is TdICEM


def _cpu_agent(B):
    from tdmpc_amd import TDMPC, make_cfg
    cfg = make_cfg("cartpole")
    cfg.device = "cpu"   # seed steps need no model: the HIP planner is only called after cfg.seed_steps
    return cfg, TDMPC(cfg, max_batch=B)


def test_seed_step_plan_batch_metrics_tensor():
    """plan_batch in the seed-step branch (tdmpc.py:109-110) with sync_metrics=False returns a [B, 2] tensor like
    the planned branch, so EnvShardedPlanner can copy it."""
    cfg, agent = _cpu_agent(4)
    a, m = agent.plan_batch(np.zeros((4, cfg.obs_shape[0]), np.float32), step=0, t0=True, sync_metrics=False)
    assert a.shape == (4, cfg.action_dim) and bool((a.abs() <= 1).all())
    assert torch.is_tensor(m) and m.shape == (4, 2) and not m.any()
    a, m = agent.plan_batch(np.zeros((4, cfg.obs_shape[0]), np.float32), step=0, t0=True)
    assert isinstance(m, list) and len(m) == 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    try:
        torch.set_num_threads(1)
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        from tdmpc_amd import EnvShardedPlanner
        cfg, agent = _cpu_agent(2)
        seen = []
        real = agent.plan_batch

        def spy(obs, step=None, t0=True, sync_metrics=True, eval_mode=False):
            seen.append(list(t0) if not isinstance(t0, bool) else t0)
            return real(obs, step=step, t0=t0, sync_metrics=sync_metrics, eval_mode=eval_mode)
        agent.plan_batch = spy
        pl = EnvShardedPlanner(4, cfg.action_dim, agent=agent, device="cpu")   # the default plan_fn
        obs = torch.zeros(4, cfg.obs_shape[0])
        a, m = pl.plan(obs, 0, t0=[True, False, False, True])   # seed step (step 0 < seed_steps)
        q.put((rank, seen, tuple(a.shape), tuple(m.shape), None))
        dist.destroy_process_group()
    except Exception as e:  # report instead of leaving the parent waiting
        q.put((rank, None, None, None, repr(e)))
        raise


def test_sharded_default_plan_fn_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for rank, seen, ashape, mshape, err in res:
        assert err is None, f"rank {rank}: {err}"
        # each rank saw its own envs' flags: rank 0 envs 0-1, rank 1 envs 2-3
        assert seen == [[[True, False], [False, True]][rank]], seen
        assert ashape == (4, 1) and mshape == (4, 2)
