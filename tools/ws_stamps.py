"""Per-step timeline of the wide step kernel (diagnostic; needs the -DWS_STAMPS build, TDMPC_LIB_PATH pointing at it).

    python tools/ws_stamps.py [B]
Runs humanoid-run plan_batch(B) a few times, then one call with stamps on, and prints for workgroups 0 (dynamics) and 4
(reward) per wave: total cycles, cycles waiting at the per-step vmcnt + barrier, and the per-phase split."""
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

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
cfg = bench_cfg("humanoid-run")
agent = TDMPC(cfg, max_batch=B, rng="fused", graph=False)
agent.model.load_state_dict(synthetic_state_dict(cfg, 0))
agent.std = 0.05
obs = np.random.RandomState(0).standard_normal((B,) + tuple(cfg.obs_shape)).astype(np.float32)
for i in range(3):
    agent.plan_batch(obs, step=10**6, t0=(i == 0), sync_metrics=False)
torch.cuda.synchronize()
buf = torch.zeros(8192, dtype=torch.int64, device="cuda")
L = _lib.lib()
L.tdmpc_debug_plan1_stamps(C.c_void_p(buf.data_ptr()))
agent.plan_batch(obs, step=10**6, t0=False, sync_metrics=False)   # the last wide launch's stamps remain
torch.cuda.synchronize()
L.tdmpc_debug_plan1_stamps(None)
st = buf.cpu().numpy().view(np.uint64).astype(np.int64)
S1 = 4   # humanoid: 4 first-layer 32-k groups -> 4 steps per super-chunk, then 16 layer-2 steps
for name, base in (("dynamics wg0", 0), ("reward wg4", 4096)):
    for w in range(8):
        s = st[base + w * 512: base + w * 512 + 512].reshape(256, 2)
        n = int((s[:, 0] > 0).sum())
        s = s[:n]
        wait = s[:, 1] - s[:, 0]
        comp = s[1:, 0] - s[:-1, 1]
        tot = s[-1, 1] - s[0, 0]
        ph = {"L1": [], "L2": [], "L3": []}
        for k in range(n - 1):
            if V2:
                c, r = divmod(k, S1 + 16)
                key = "L3" if c >= 4 else ("L1" if r < S1 else "L2")
            else:
                c, r = divmod(k, S1 + 8)
                key = "L3" if c >= 8 else ("L1" if r < S1 else "L2")
            ph[key].append(comp[k] + wait[k + 1])
        print(f"{name} wave {w}: steps {n} total {tot} cyc, wait {wait.sum()} ({wait.sum() / tot:.2f}); per-step "
              "(compute + next wait) median: " + ", ".join(f"{k} {np.median(v):.0f} x{len(v)}" for k, v in ph.items() if v))
        if w == 0:
            print("   first steps wait:", wait[:12].tolist())
            print("   first steps comp:", comp[:12].tolist())
            print("   steps comp:", comp[:24].tolist())
            print("   steps wait:", wait[:24].tolist())
