"""Host-side cost of the literal drop-in plan() (development tool): cProfile over repeated calls."""
import cProfile, os, pstats, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from tdmpc_amd.config import bench_cfg
from tdmpc_amd.tdmpc import TDMPC
from tdmpc_amd.told import synthetic_state_dict

cfg = bench_cfg("humanoid-run")
agent = TDMPC(cfg)
agent.model.load_state_dict(synthetic_state_dict(cfg, 0))
agent.std = 0.05
obs = np.random.RandomState(0).standard_normal(cfg.obs_shape).astype(np.float32)
for i in range(5):
    agent.plan(obs, step=10**6, t0=(i == 0))
torch.cuda.synchronize()
K = 200
t = time.perf_counter()
for i in range(K):
    agent.plan(obs, step=10**6, t0=False)
torch.cuda.synchronize()
print(f"plan(): {(time.perf_counter() - t) / K * 1e3:.3f} ms/call")
pr = cProfile.Profile()
pr.enable()
for i in range(K):
    agent.plan(obs, step=10**6, t0=False)
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(18)
