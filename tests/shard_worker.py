"""One rank of tests/test_gpu_sharded.py (started as a child process, not collected by pytest): plans its shard of a
vectorised dog-run batch with the real HIP `TDMPC` under `EnvShardedPlanner`'s default plan_fn and writes every env's
gathered (action, metrics) of each call to an .npz. The generators are positioned exactly where a single-process
`plan_batch` over all envs would take this rank's envs' draws (torch's Philox offset, numpy's uniforms), so the
gathered batch can be compared with that run bitwise."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from tdmpc_amd import TDMPC, EnvShardedPlanner  # noqa: E402
from tdmpc_amd.config import make_cfg  # noqa: E402
from tdmpc_amd.told import synthetic_state_dict  # noqa: E402

N_ENVS, CALLS, SEED, WSEED = 64, 2, 21, 13


def cfg():
    return make_cfg("dog", num_samples=512, num_elites=64, iterations=6, horizon=5)


def observations(c):
    rs = np.random.RandomState(SEED)
    return [rs.standard_normal((N_ENVS, c.obs_shape[0])).astype(np.float32) for _ in range(CALLS)]


def position_rngs(agent, first_env, call, H, I):
    """Torch's generator and numpy's global state as a single-process plan_batch over N_ENVS envs would have them
    when it reaches env `first_env` of call `call` (every env draws the same amount: reference_advance)."""
    torch.manual_seed(SEED)
    gen = torch.cuda.default_generators[0]
    per_env = agent.planner.reference_advance(1, H, I, False)
    gen.set_offset(gen.get_offset() + (call * N_ENVS + first_env) * per_env)
    np.random.seed(SEED)
    np.random.random_sample(call * N_ENVS + first_env)


def status_main(out):
    """One env per rank (the persistent one-env plan's regime); rank 1's plan1 never completes a hand-off
    (TDMPC_P1_DEBUG_SKIP), so its actions are NaN and its status word is set. Every rank must raise from
    EnvShardedPlanner.plan at the same call -- the failing rank's status travels in the gathered block -- and the
    call after the raise plans normally on every rank."""
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    c = make_cfg("humanoid", num_samples=512, num_elites=64, iterations=6, horizon=5)   # (a plan1 shape)
    agent = TDMPC(c, max_batch=1, path="persist" if rank == 1 else "chain")
    agent.model.load_state_dict(synthetic_state_dict(c, WSEED))
    agent.std = 0.05
    planner = EnvShardedPlanner(world, c.action_dim, agent=agent)
    obs = torch.from_numpy(np.random.RandomState(SEED).standard_normal((world, c.obs_shape[0])).astype(np.float32))
    if rank == 1:
        os.environ["TDMPC_P1_DEBUG_SKIP"] = "1"
    raised = None
    try:
        planner.plan(obs, 10**6, t0=True)
    except RuntimeError as e:
        raised = str(e)
    if rank == 1:
        del os.environ["TDMPC_P1_DEBUG_SKIP"]
        agent.planner._graphs.clear()   # (the captured graph keeps the knob's launch arguments)
    a, m = planner.plan(obs, 10**6, t0=True)
    with open(os.path.join(out, f"status{rank}.txt"), "w") as f:
        f.write(f"{raised}\n{bool(torch.isfinite(a).all())}\n{int(agent.planner.status.item())}\n")


def main(out):
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    backend = os.environ.get("TDMPC_SHARD_BACKEND", "gloo")   # "nccl" (RCCL): one rank per device only
    if backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    if len(sys.argv) > 2 and sys.argv[2] == "status":
        try:
            status_main(out)
        finally:
            dist.destroy_process_group()
        return
    try:
        c = cfg()
        b = N_ENVS // world
        agent = TDMPC(c, max_batch=b)
        agent.model.load_state_dict(synthetic_state_dict(c, WSEED if rank == 0 else WSEED + 1))
        agent.std = 0.05
        planner = EnvShardedPlanner(N_ENVS, c.action_dim, agent=agent)   # the default plan_fn: agent.plan_batch
        planner.broadcast_weights(agent.model, src=0)                   # rank 1 starts from other weights
        H, I = agent.horizon(10**6), c.iterations
        res = {}
        for k, obs in enumerate(observations(c)):
            position_rngs(agent, planner.lo, k, H, I)
            a, m = planner.plan(torch.from_numpy(obs), 10**6, t0=(k == 0))
            res[f"a{k}"], res[f"m{k}"] = a.cpu().numpy(), m.cpu().numpy()
        if world == 1:
            # (plan() skips the exchange at world 1: run the planner's gather itself, so the RCCL device-tensor
            # all_gather_into_tensor executes on the hardware; its output must be the local block, byte for byte)
            planner._all.fill_(float("nan"))
            planner._all_gather()
            torch.cuda.synchronize()
            res["gather_equal"] = np.array(bool(torch.equal(planner._all, planner._local)))
        np.savez(os.path.join(out, f"rank{rank}.npz"), **res)
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
