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

# GPU time of one call's device work alone: the cached graph replayed back to back (draws included when they are
# captured, i.e. TDMPC_REF_DRAWS=torch) vs the wall time of a whole plan() call
pl = agent.planner
g = next(iter(pl._graphs.values()))
torch.cuda.synchronize()
t = time.perf_counter()
for i in range(K):
    g.replay()
    torch.cuda.current_stream().synchronize()
print(f"graph replay + sync alone: {(time.perf_counter() - t) / K * 1e3:.3f} ms/call")
t = time.perf_counter()
for i in range(K):
    pl.draw_reference_device(1, 5, 6, False)
    g.replay()
    torch.cuda.current_stream().synchronize()
print(f"one-launch draws + graph replay + sync: {(time.perf_counter() - t) / K * 1e3:.3f} ms/call")
