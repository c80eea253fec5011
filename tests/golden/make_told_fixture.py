"""Generate tests/golden/told_layout.json from the REFERENCE TOLD (checkpoint interop).

Run once in the build container (where /root/reference exists):   python tests/golden/make_told_fixture.py
Imports the reference exactly like make_golden.py (rlpyt stub, Module.cuda no-op, namespace cfg). For every
bench task config it records the reference TOLD's state_dict in key order -- name, shape -- and, for a TOLD
built under torch.manual_seed(0) with the reference initialisation (tdmpc.py:20-23, helper.py:35-45), each
tensor's float64 sum and sum of squares. tests/test_checkpoint.py checks `tdmpc_amd.told.TOLD` against it:
same keys in the same order (so `{'model', 'model_target'}` checkpoints written by the reference's
`TDMPC.save` load with strict=True into the drop-in and vice versa) and the same initial weights.
"""
from __future__ import annotations

import json
import os
import sys

import torch

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

from make_golden import import_reference, ref_cfg  # noqa: E402
from tdmpc_amd.config import bench_cfg  # noqa: E402

CONFIGS = ["cartpole-swingup", "cheetah-run", "humanoid-run", "humanoid-run-l512", "dog-run",
           "quadruped-run-pixels"]


def main():
    ref = import_reference()
    out = {}
    for name in CONFIGS:
        cfg = bench_cfg(name)
        torch.manual_seed(0)
        model = ref.TOLD(ref_cfg(cfg))
        sd = model.state_dict()
        out[name] = [[k, list(v.shape), float(v.double().sum()), float((v.double() ** 2).sum())]
                     for k, v in sd.items()]
    path = os.path.join(HERE, "told_layout.json")
    json.dump(out, open(path, "w"), indent=0)
    print(f"wrote {path}: " + ", ".join(f"{k} {len(v)} tensors" for k, v in out.items()))


if __name__ == "__main__":
    main()
