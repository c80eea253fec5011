"""Quick single-GPU timing of the learner update (bench.py's learner leg without the CPU baseline)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import bench
from tdmpc_amd.config import bench_cfg

cfg = bench_cfg(sys.argv[1] if len(sys.argv) > 1 else "humanoid-run")
modes = tuple(os.environ.get("MODES", "graph").split(","))
print(json.dumps(bench.learner_bench(cfg, torch.device("cuda"), cpu=False, reps=int(os.environ.get("REPS", 30)),
                                     pixels=False, modes=modes)))
