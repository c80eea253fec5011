"""Kernel trace helper: humanoid learner updates from the captured HIP graph (development tool)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from types import SimpleNamespace
import numpy as np, torch
from tdmpc_amd.config import bench_cfg
from tdmpc_amd.replay import ReplayBuffer
from tdmpc_amd.tdmpc import TDMPC
from tdmpc_amd.told import synthetic_state_dict

lcfg = bench_cfg("humanoid-run", batch_size=512)
L = 500
rc = SimpleNamespace(**{**vars(lcfg), "train_steps": 50_000, "max_buffer_size": 10**6, "episode_length": L,
                        "env_horizon": lcfg.horizon})
rs = np.random.RandomState(0)
O, A = lcfg.obs_shape[0], lcfg.action_dim
ep = SimpleNamespace(obs=torch.from_numpy(rs.standard_normal((L + 1, O)).astype(np.float32)),
                     action=torch.from_numpy(rs.uniform(-1, 1, (L, A)).astype(np.float32)),
                     reward=torch.from_numpy(rs.standard_normal(L).astype(np.float32)))
agent = TDMPC(lcfg)
agent.model.load_state_dict(synthetic_state_dict(lcfg, 0))
agent.model_target.load_state_dict(synthetic_state_dict(lcfg, 1))
agent.learner(graph=True, warmup=3)
buf = ReplayBuffer(rc, latent_plan=True)
for _ in range(50_000 // L - 1):
    buf.add(ep)
for i in range(5):
    agent.update(buf, i + 1, sync_metrics=False)
torch.cuda.synchronize()
torch.cuda.nvtx.range_push("timed") if hasattr(torch.cuda, "nvtx") else None
for i in range(10):
    agent.update(buf, 6 + i, sync_metrics=False)
torch.cuda.synchronize()
print("ok")
