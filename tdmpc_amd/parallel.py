"""Vectorised-env planning sharded over the GPUs of one node.

Environments are independent units, so a global batch of E = world * B envs is split into contiguous shards:
rank r owns envs [r*B, (r+1)*B), plans them with its own TDMPC (a full weight replica) and one collective --
an all-gather of the per-env results [B, A+2] = (action, reward mean, std) -- gives every rank the whole
vectorised batch. There is no collective inside planning: the only exchange is ~(A+2)*4 bytes per env per
step, latency-bound over xGMI (RCCL picks its one-shot algorithm at this size). Weight replicas are kept in sync
by broadcasting the TOLD parameters from one rank (after loading a checkpoint or a learner update).

The reference has no distributed code (its only parallelism is Ray Tune trial scheduling,
src/train_multi_experiments.py:144-170); this module is the MI355X-native equivalent for the vectorised
configuration BASELINE.json names ("dog-run, 64 vectorised envs sharded 8-per-GPU across 8xMI355X").
"""
from __future__ import annotations

from typing import Callable, Optional

import torch
import torch.distributed as dist


def shard_bounds(n_envs: int, rank: int, world: int):
    """Contiguous, balanced shard [lo, hi) of `n_envs` envs for `rank` (first n_envs % world ranks get one more)."""
    base, extra = divmod(n_envs, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


class EnvShardedPlanner:
    """Plans this rank's shard of a global env batch and all-gathers every env's result.

    plan_fn(obs_shard, step, t0) -> (actions [b, A], metrics [b, 2]) runs on this rank's device; by default it is
    `agent.plan_batch(..., sync_metrics=False)` of a `tdmpc_amd.TDMPC`. Shards must be equal-sized (the
    all-gather is a single fixed-size collective); `n_envs % world == 0` is required."""

    def __init__(self, n_envs: int, action_dim: int, agent=None, plan_fn: Optional[Callable] = None,
                 group=None, device=None):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        if n_envs % self.world:
            raise ValueError(f"{n_envs} envs do not split evenly over {self.world} ranks")
        self.n_envs, self.A = n_envs, action_dim
        self.lo, self.hi = shard_bounds(n_envs, self.rank, self.world)
        self.agent = agent
        if plan_fn is None:
            if agent is None:
                raise ValueError("need an agent or a plan_fn")
            plan_fn = lambda obs, step, t0: agent.plan_batch(obs, step=step, t0=t0, sync_metrics=False)  # noqa
        self.plan_fn = plan_fn
        self.device = torch.device(device) if device is not None else (
            agent.device if agent is not None else torch.device("cpu"))
        b = self.hi - self.lo
        # per env: action | reward mean, std | the planning rank's device status word (as float; 0 = healthy)
        self._local = torch.zeros(b, action_dim + 3, device=self.device)
        self._all = torch.zeros(self.world * b, action_dim + 3, device=self.device)
        # RCCL path: the gathered status column goes down behind an event and is checked two calls later (the copy
        # is queued ahead of the next call, so the wait leaves no bubble); gloo moves host copies anyway and checks
        # at once. Every rank sees the same gathered block, so every rank raises at the same call.
        pin = self.device.type == "cuda"
        self._st_pin = torch.zeros(2, self.world * b, dtype=torch.float32, pin_memory=pin)
        self._st_ev = [None, None]
        self._st_pending = [False, False]
        self._st_k = 0

    def local_obs(self, global_obs):
        return global_obs[self.lo:self.hi]

    @torch.no_grad()
    def plan(self, global_obs, step, t0=True):
        """Plan this rank's envs of `global_obs` ([n_envs, ...]) and return every env's (actions, metrics).
        `t0` is a bool for the whole batch or a sequence of n_envs per-env flags (global env order).
        On RCCL (and at world 1 on the GPU) a rank's device failure is raised on every rank two calls late (its
        status word rides the gathered block); until then the affected envs' returned actions are NaN."""
        if not isinstance(t0, (bool, int)) and not (torch.is_tensor(t0) and t0.dim() == 0):
            t0 = list(t0)
            if len(t0) != self.n_envs:
                raise ValueError(f"per-env t0 has {len(t0)} entries for {self.n_envs} envs")
            t0 = t0[self.lo:self.hi]   # this rank's envs' flags
        self._deferred_status()
        a, m = self.plan_fn(self.local_obs(global_obs), step, t0)
        self._local[:, :self.A].copy_(a)
        self._local[:, self.A:self.A + 2].copy_(m)
        pl = getattr(self.agent, "planner", None)
        if pl is not None and hasattr(pl, "status"):
            self._local[:, self.A + 2].copy_(pl.status.float().expand(self._local.shape[0]))
        if self.world > 1:
            host = self._all_gather()
            res = self._all
        else:
            host, res = None, self._local
        if host is not None:
            self._raise_if_failed(host[:, self.A + 2])
        else:
            self._post_status(res[:, self.A + 2])
        return res[:, :self.A], res[:, self.A:self.A + 2]

    def check_status(self):
        """Synchronising check of every rank's status as last gathered (raises like the deferred check)."""
        self._st_pending = [False, False]
        self._raise_if_failed(self._all[:, self.A + 2].cpu() if self.world > 1 else self._local[:, self.A + 2].cpu())

    def _post_status(self, col):
        if not self._st_pin.is_pinned():
            self._raise_if_failed(col.cpu())
            return
        s = self._st_k % 2
        if self._st_ev[s] is None:
            self._st_ev[s] = torch.cuda.Event()
        self._st_pin[s].copy_(col, non_blocking=True)
        self._st_ev[s].record()
        self._st_pending[s] = True
        self._st_k += 1

    def _deferred_status(self):
        s = self._st_k % 2
        if self._st_pending[s]:
            self._st_ev[s].synchronize()
            self._st_pending[s] = False
            self._raise_if_failed(self._st_pin[s])

    def _raise_if_failed(self, col):
        """Raise on any nonzero gathered status (the device status word of the rank that planned that env: its
        actions are NaN, tdmpc_hip.h ABI 6); the failing rank's sticky word is cleared, so the next call plans."""
        bad = torch.nonzero(col != 0).flatten().tolist()
        if not bad:
            return
        self._st_pending = [False, False]
        b = self.hi - self.lo
        ranks = sorted({e // b for e in bad})
        st = int(col[bad[0]])
        pl = getattr(self.agent, "planner", None)
        if pl is not None and hasattr(pl, "status"):
            pl.status.zero_()
            pl._st_pending = [False, False]
        raise RuntimeError(f"tdmpc_plan failed on the device of rank(s) {ranks} (status {st}): those envs' actions "
                           "are NaN. Status 1 = the persistent one-env plan timed out at a hand-off; set "
                           "TDMPC_PERSIST=0 to plan on the launch chain instead.")

    def _all_gather(self):
        """RCCL ("nccl") gathers the device tensors directly over xGMI. The gloo transport (ranks sharing one GPU, or
        a host without peer access: the world-2 tests) moves host copies; the gathered values are the same bytes."""
        if self._local.is_cuda and dist.get_backend(self.group) == "gloo":
            host_all = torch.empty(self._all.shape, dtype=self._all.dtype)
            dist.all_gather_into_tensor(host_all, self._local.cpu(), group=self.group)
            self._all.copy_(host_all)
            return host_all
        dist.all_gather_into_tensor(self._all, self._local, group=self.group)
        return self._all if not self._all.is_cuda else None

    @torch.no_grad()
    def broadcast_weights(self, model: torch.nn.Module, src: int = 0):
        """Make every rank's TOLD replica equal to rank `src`'s (after a checkpoint load or an update)."""
        if self.world == 1:
            return
        gloo = dist.get_backend(self.group) == "gloo"
        for p in model.state_dict().values():
            if gloo and p.is_cuda:
                h = p.cpu()
                dist.broadcast(h, src=src, group=self.group)
                p.copy_(h)
            else:
                dist.broadcast(p, src=src, group=self.group)
