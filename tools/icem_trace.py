"""Kernel trace helper: a few iCEM plans (device RNG, auto path) for rocprofv3 (development tool)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from tdmpc_amd.config import bench_cfg
from tdmpc_amd.icem import TdICEM
from tdmpc_amd.told import synthetic_state_dict

cfg = bench_cfg("humanoid-run")
agent = TdICEM(cfg, rng=sys.argv[1] if len(sys.argv) > 1 else "device")
agent.model.load_state_dict(synthetic_state_dict(cfg, 0, enc_norm=True))
agent.std = 0.05
obs = np.random.RandomState(0).standard_normal(cfg.obs_shape).astype(np.float32)
for i in range(6):
    agent.plan(obs, step=10**6, t0=(i == 0))
torch.cuda.synchronize()
print("ok")
