"""Generate tests/golden/learner_cartpole.npz by running the REFERENCE `TDMPC.update` in this container.

Run once in the build container (where /root/reference exists):   python tests/golden/make_learner_golden.py
Imports the reference like make_golden.py (rlpyt stub, Module.cuda no-op, namespace cfg; CPU). The agent starts
from the seeded synthetic weights (model and target), a stand-in replay buffer hands `update` a fixed batch
(tests/learner_io.py) and records the priorities it is given; torch.manual_seed(0) before the first update
fixes the TruncatedNormal draws of `_td_target` / `update_pi`. Two updates (step 1: no EMA, step 2: EMA). The
.npz holds per update the returned metrics, the new priorities, and for model and target every tensor's
float64 sum and sum of squares plus 64 fixed elements.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, HERE)

from make_golden import import_reference, ref_cfg  # noqa: E402
from learner_io import METRICS, batch, learner_cfg, probe, summarize  # noqa: E402
from tdmpc_amd.told import synthetic_state_dict  # noqa: E402


class FakeBuffer:
    def __init__(self, b):
        self.b = b
        self.prios = []

    def sample(self):
        return self.b

    def update_priorities(self, idxs, p):
        self.prios.append(p.detach().clone())


def main():
    ref = import_reference()
    cfg = learner_cfg()
    agent = ref.TDMPC(ref_cfg(cfg))
    agent.model.load_state_dict(synthetic_state_dict(cfg, 21))
    agent.model_target.load_state_dict(synthetic_state_dict(cfg, 22))
    buf = FakeBuffer(batch(cfg))
    torch.manual_seed(0)
    out = {}
    for k, step in enumerate((1, 2)):
        m = agent.update(buf, step)
        out[f"u{k}_metrics"] = np.array([m[n] for n in METRICS], dtype=np.float64)
        out[f"u{k}_prio"] = buf.prios[-1].numpy()
        for tag, mod in (("model", agent.model), ("target", agent.model_target)):
            s, ss, pr = summarize(mod.state_dict())
            out[f"u{k}_{tag}_sum"], out[f"u{k}_{tag}_sumsq"], out[f"u{k}_{tag}_probe"] = s, ss, pr
    path = os.path.join(HERE, "learner_cartpole.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path} ({os.path.getsize(path)} bytes):",
          {n: round(float(v), 6) for n, v in zip(METRICS, out["u1_metrics"])})


if __name__ == "__main__":
    main()
