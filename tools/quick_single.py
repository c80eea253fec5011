"""Single-env TDMPC.plan timing by mode: eager vs HIP graph, reference-order vs fused RNG (development tool)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from tdmpc_amd.config import bench_cfg
from tdmpc_amd.tdmpc import TDMPC
from tdmpc_amd.told import synthetic_state_dict

cfg = bench_cfg(sys.argv[1] if len(sys.argv) > 1 else "humanoid-run")
obs = np.random.RandomState(0).standard_normal(cfg.obs_shape).astype(np.float32)
for graph in (False, True):
    for rng, draws in (("reference", "device"), ("reference", "torch"), ("fused", "device")):
        os.environ["TDMPC_REF_DRAWS"] = draws   # reference-order draws: one kernel, or torch's own launches
        agent = TDMPC(cfg, rng=rng, graph=graph)
        agent.model.load_state_dict(synthetic_state_dict(cfg, 0))
        agent.std = 0.05
        for i in range(3):
            agent.plan(obs, step=10**6, t0=(i == 0))
        torch.cuda.synchronize()
        K = 30
        t = time.perf_counter()
        for i in range(K):
            a, m = agent.plan(obs, step=10**6, t0=False)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / K
        tag = "/" + draws if rng == "reference" else ""
        print(f"plan() single env graph={graph} rng={rng}{tag}: {dt * 1e3:.3f} ms/call ({1 / dt:.0f} plan-steps/s)")
