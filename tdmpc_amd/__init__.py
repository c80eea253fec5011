"""tdmpc_amd: MI355X-native TD-MPC planning (TDMPC.plan + TOLD latent rollout) behind the reference's agent API.

The drop-in names:

    from tdmpc_amd import TDMPC            # src/algorithm/tdmpc.py:53 (agent: plan / update / save / load)
    from tdmpc_amd import TOLD             # src/algorithm/tdmpc.py:9 (same module tree and state_dict keys)
    from tdmpc_amd import ReplayBuffer     # src/algorithm/helper.py:434 (device prioritized replay)
    from tdmpc_amd import TdICEM           # src/algorithm/tdmpc_icem_similarity_mlp.py:116 (iCEM planner)
    from tdmpc_amd import EnvShardedPlanner  # vectorised envs over the GPUs of one node

Imports are resolved lazily, so `import tdmpc_amd` does not load torch or the HIP library.
"""
from __future__ import annotations

import importlib

_EXPORTS = {
    "TDMPC": "tdmpc",
    "HipPlanner": "tdmpc",
    "load_checkpoint": "tdmpc",
    "TOLD": "told",
    "ReplayBuffer": "replay",
    "TdICEM": "icem",
    "EnvShardedPlanner": "parallel",
    "shard_bounds": "parallel",
    "make_cfg": "config",
    "linear_schedule": "config",
}

__all__ = sorted(_EXPORTS)


def __getattr__(name):
    mod = _EXPORTS.get(name)
    if mod is None:
        raise AttributeError(f"module 'tdmpc_amd' has no attribute {name!r}")
    val = getattr(importlib.import_module(f".{mod}", __name__), name)
    globals()[name] = val
    return val


def __dir__():
    return sorted(set(globals()) | set(_EXPORTS))
