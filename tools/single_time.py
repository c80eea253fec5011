"""Literal single-env plan() timing (development tool): TDMPC(cfg) defaults as bench.py's single_env leg (reference-
order draws, HIP graph), numpy obs, metrics synced; prints ms per call. python tools/single_time.py [config] [calls]"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from tdmpc_amd.config import bench_cfg
import importlib
TDMPC = importlib.import_module(os.environ.get("SINGLE_MOD", "tdmpc_amd.tdmpc")).TDMPC   # (A/B of host-side variants)
from tdmpc_amd.told import synthetic_state_dict

cfg = bench_cfg(sys.argv[1] if len(sys.argv) > 1 else "humanoid-run")
K = int(sys.argv[2]) if len(sys.argv) > 2 else 200
obs = np.random.RandomState(0).standard_normal(cfg.obs_shape).astype(np.float32)
agent = TDMPC(cfg)
agent.model.load_state_dict(synthetic_state_dict(cfg, 0))
agent.std = 0.05
for i in range(5):
    agent.plan(obs, step=10**6, t0=(i == 0))
torch.cuda.synchronize()
t = time.perf_counter()
for i in range(K):
    a = agent.plan(obs, step=10**6, t0=False)
torch.cuda.synchronize()
dt = (time.perf_counter() - t) / K
print(f"plan() single env: {dt * 1e3:.4f} ms/call ({1 / dt:.1f} plan-steps/s) finite={bool(torch.isfinite(a[0]).all())}")
