"""Quick single-GPU timing of TDMPC.plan_batch for a config (development tool)."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from tdmpc_amd.config import bench_cfg
from tdmpc_amd.tdmpc import TDMPC
from tdmpc_amd.told import synthetic_state_dict

name = sys.argv[1] if len(sys.argv) > 1 else "humanoid-run"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1
cfg = bench_cfg(name)
agent = TDMPC(cfg, max_batch=B, rng="fused", path=os.environ.get("QT_PATH", "auto"))
agent.model.load_state_dict(synthetic_state_dict(cfg, 0)); agent.std = 0.05
obs = np.random.RandomState(0).standard_normal((B,) + tuple(cfg.obs_shape)).astype(np.float32)
if cfg.modality == "pixels":
    obs = np.random.RandomState(0).randint(0, 256, size=(B,) + tuple(cfg.obs_shape)).astype(np.uint8)
for i in range(3):
    agent.plan_batch(obs, step=10**6, t0=(i == 0))
torch.cuda.synchronize()
K = 20
t = time.perf_counter()
for i in range(K):
    a, m = agent.plan_batch(obs, step=10**6, t0=False, sync_metrics=False)
torch.cuda.synchronize()
dt = (time.perf_counter() - t) / K
print(f"{name} B={B}: {dt*1e3:.3f} ms/call, {B/dt:.1f} plan-steps/s")

# QT_PROF=<profile cfg> (4: the step launches, 6: helper.q): the library's HIP-event timer over K eager calls
pc = os.environ.get("QT_PROF")
if pc:
    import ctypes as C
    from tdmpc_amd import _lib
    L = _lib.lib()
    agent.graph = False
    agent.plan_batch(obs, step=10**6, t0=False, sync_metrics=False)
    torch.cuda.synchronize()
    _lib.check(L.tdmpc_profile_begin(int(pc), -1, 0, 0, 8192), "profile_begin")
    for i in range(K):
        agent.plan_batch(obs, step=10**6, t0=False, sync_metrics=False)
    n, ms, fl = C.c_int32(), C.c_double(), C.c_double()
    _lib.check(L.tdmpc_profile_end(C.byref(n), C.byref(ms), C.byref(fl)), "profile_end")
    if n.value:
        print(f"  profile cfg {pc}: {L.tdmpc_profile_kernel().decode()} {n.value} launches, "
              f"{ms.value / n.value * 1e3:.2f} us/launch, {ms.value / K * 1e3:.1f} us per call, "
              f"{fl.value / ms.value / 1e9 / 419.5:.4f} of the x6 roof")
