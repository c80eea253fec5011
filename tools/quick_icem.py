"""Quick timing of TdICEM.plan on one env: wall per call, device busy per call (development tool)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from tdmpc_amd.config import bench_cfg
from tdmpc_amd.icem import TdICEM
from tdmpc_amd.told import synthetic_state_dict

cfg = bench_cfg("humanoid-run")
for path in ("auto", "chain", "layered"):
  for rng in ("reference", "device"):
    agent = TdICEM(cfg, path=path, rng=rng)
    agent.model.load_state_dict(synthetic_state_dict(cfg, 0, enc_norm=True))
    agent.std = 0.05
    obs = np.random.RandomState(0).standard_normal(cfg.obs_shape).astype(np.float32)
    for i in range(3):
        agent.plan(obs, step=10**6, t0=(i == 0))
    torch.cuda.synchronize()
    K = 20
    t = time.perf_counter()
    for i in range(K):
        agent.plan(obs, step=10**6, t0=False)
    torch.cuda.synchronize()
    print(f"iCEM B=1 path={path} rng={rng}: {(time.perf_counter() - t) / K * 1e3:.3f} ms/call")
    # host-only cost of the noise draws
    H = agent.plan_horizon
    cts = agent.counts(agent.mixture_coef, True)
    off = agent._layout(H, cts, True)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for i in range(K):
        if rng == "device":
            agent._draw_device(1, H, cts, off, True)
        else:
            agent._draw(0, H, cts, off, True, False)
    torch.cuda.synchronize()
    print(f"noise draws: {(time.perf_counter() - t) / K * 1e3:.3f} ms/call")
