"""Phase timeline of the column-split step kernel (diagnostic; needs the -DCS_STAMPS build, TDMPC_LIB_PATH at it).

    python tools/cs_stamps.py [config] [B]
Plans a few times, then one call with stamps on; prints, for workgroups 0 (dynamics) and 4 (reward) of the last
column-split launch, the shader-clock cycles of each phase: prologue, layer 1, publish + hand-off 1, deferred x,
layer 2, layer 3 / partials, hand-off 2, reduction."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from tdmpc_amd import _lib
from tdmpc_amd.config import bench_cfg
from tdmpc_amd.tdmpc import TDMPC
from tdmpc_amd.told import synthetic_state_dict

name = sys.argv[1] if len(sys.argv) > 1 else "dog-run"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 8
cfg = bench_cfg(name)
agent = TDMPC(cfg, max_batch=B, rng="fused", graph=False)
agent.model.load_state_dict(synthetic_state_dict(cfg, 0))
agent.std = 0.05
obs = np.random.RandomState(0).standard_normal((B,) + tuple(cfg.obs_shape)).astype(np.float32)
for i in range(3):
    agent.plan_batch(obs, step=10**6, t0=(i == 0), sync_metrics=False)
torch.cuda.synchronize()
buf = torch.zeros(2048, dtype=torch.int64, device="cuda")
L = _lib.lib()
L.tdmpc_debug_plan1_stamps(C.c_void_p(buf.data_ptr()))
agent.plan_batch(obs, step=10**6, t0=False, sync_metrics=False)
torch.cuda.synchronize()
L.tdmpc_debug_plan1_stamps(None)
st = buf.cpu().numpy().astype(np.int64)
names = ["prologue", "layer 1", "publish + hand-off 1", "deferred x", "layer 2", "layer 3 / partial", "hand-off 2",
         "reduction"]
for wg, base in (("dynamics wg0", 0), ("reward wg4", 16)):
    s = st[base:base + 9]
    if not s[0]:
        print(wg, "no stamps")
        continue
    print(f"{wg}: total {s[8] - s[0]} cycles")
    for i, nm in enumerate(names):
        if s[i + 1]:
            print(f"   {nm:22s} {s[i + 1] - s[i]:8d}")
