"""Per-hand-off timeline of the persistent one-env plan (plan1_kernel) from its diagnostic realtime stamps
(development tool): python tools/p1_stamps.py [config]"""
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

cfg = bench_cfg(sys.argv[1] if len(sys.argv) > 1 else "humanoid-run")
agent = TDMPC(cfg, rng="fused", graph=False, path="persist")
agent.model.load_state_dict(synthetic_state_dict(cfg, 0))
agent.std = 0.05
obs = np.random.RandomState(0).standard_normal((1,) + tuple(cfg.obs_shape)).astype(np.float32)
for i in range(3):
    agent.plan_batch(obs, step=10**6, t0=(i == 0))
st = torch.zeros(2048, dtype=torch.int64, device="cuda")
_lib.lib().tdmpc_debug_plan1_stamps(C.c_void_p(st.data_ptr()))
agent.plan_batch(obs, step=10**6, t0=False)
torch.cuda.synchronize()
_lib.lib().tdmpc_debug_plan1_stamps(None)
s = st.cpu().numpy().astype(np.int64)
H, I = agent.horizon(10**6), cfg.iterations
labels = ["init"]
for i in range(I):
    for t in range(H):
        if i == 0:
            labels += [f"i0 t{t} pi.l1", f"i0 t{t} pi.l3", f"i0 t{t} pi.fin"]
        labels += [f"i{i} t{t} st.l1", f"i{i} t{t} st.l3", f"i{i} t{t} st.red"]
    labels += [f"i{i} pi.l1", f"i{i} pi.l3", f"i{i} pi.fin", f"i{i} q.m1", f"i{i} q.a1", f"i{i} q.m2",
               f"i{i} q.own+GRID"]
    if i < I - 1:
        labels += [f"i{i} cem.x0"]
for w, base in (("wg0", 0), ("wg255", 1024)):
    a = s[base:base + 2 * len(labels) + 2].reshape(-1, 2)
    n = len(labels)
    t0 = a[1, 0]
    print(f"--- {w}: {n} hand-offs, first arrival -> last release {(a[n, 1] - a[1, 0]) / 100:.1f} us")
    tot_work = tot_wait = 0.0
    rows = []
    for k in range(1, n + 1):
        work = (a[k, 0] - a[k - 1, 1]) / 100 if k > 1 else 0.0
        wait = (a[k, 1] - a[k, 0]) / 100
        tot_work += work
        tot_wait += wait
        rows.append((labels[k - 1], work, wait))
    for lab, wk, wt in rows[:62]:
        print(f"{lab:18s} work {wk:7.2f} us  wait {wt:7.2f} us")
    print(f"total work {tot_work:.1f} us, wait {tot_wait:.1f} us")
mk, ck = s[900:906], s[920:926]
print("local hand-offs per group:", list(s[950:958]), " step i1 t0 L2 (us): mm", (mk[1]-mk[0])/100, "put+barrier", (mk[2]-mk[1])/100,
      "last layer", (mk[3]-mk[2])/100, "| cycles", ck[1]-ck[0], ck[2]-ck[1], ck[3]-ck[2])
mk = s[900:920]
print("CEM i1 (us): sort+merge", (mk[11]-mk[10])/100, "elite gather", (mk[12]-mk[11])/100, "refit", (mk[13]-mk[12])/100,
      "-> next sync arrival", (s[2 * (1 + 30 + 3 + 5 + 1 + 1) ] - mk[13]) / 100 if False else "")
ga = s[1400:1656].astype(np.float64)
ga = (ga - ga.min()) / 100
print("grid arrival spread i1 (us): per group max", [round(float(ga[g::8].max()), 1) for g in range(8)],
      "per group min", [round(float(ga[g::8].min()), 1) for g in range(8)])
