"""Quick single-GPU timing of the pixel learner update (bench.py's pixel leg; development tool).
    python tools/quick_pixel_learner.py [engine|autograd|both] [reps]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import bench

which = sys.argv[1] if len(sys.argv) > 1 else "both"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
print(json.dumps(bench.pixel_learner_bench(torch.device("cuda"), reps=reps,
                                           modes=None if which == "both" else (which,))))
