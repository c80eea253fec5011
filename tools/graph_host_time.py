"""Host-side cost of the learner's graph replay (development tool): how long g.replay() takes to return vs the
update's GPU time. A replay that returns in ~the GPU time is submission-bound.   python tools/graph_host_time.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import bench
from tdmpc_amd.config import bench_cfg

cfg = bench_cfg("humanoid-run")
bench.learner_bench(cfg, torch.device("cuda"), cpu=False, reps=5, pixels=False, modes=("graph",))
# the bench's agent is gone; rebuild the same setup inline through its helpers
import tdmpc_amd.learner as L
orig = torch.cuda.CUDAGraph.replay
host = []


def timed(self):
    t = time.perf_counter()
    orig(self)
    host.append(time.perf_counter() - t)


torch.cuda.CUDAGraph.replay = timed
out = bench.learner_bench(cfg, torch.device("cuda"), cpu=False, reps=40, pixels=False, modes=("graph",))
h = sorted(host[-40:])
print(f"update {out['graph']['ms_per_update']:.3f} ms; replay() host time median {h[len(h) // 2] * 1e6:.1f} us, "
      f"min {h[0] * 1e6:.1f}, max {h[-1] * 1e6:.1f} (n={len(h)})")
