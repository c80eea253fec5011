"""Development check: per-tensor gradients of one learner-engine update against the oracle's (GPU box)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))
import numpy as np
import torch

from learner_io import batch, learner_cfg
from oracle.learner_ref import RefLearner
from tdmpc_amd.config import make_cfg
from tdmpc_amd.tdmpc import TDMPC
from tdmpc_amd.told import synthetic_state_dict


class Buf:
    def __init__(self, b):
        self.b = tuple(x.cuda() for x in b)
        self.prio = torch.zeros(self.b[0].shape[0], 1, device="cuda")

    def sample(self):
        return self.b

    def update_priorities(self, idxs, p):
        self.prio.copy_(p)


task = sys.argv[1] if len(sys.argv) > 1 else "cartpole"
cfg = learner_cfg() if task == "cartpole" else make_cfg(task, num_samples=64, num_elites=32, iterations=3,
                                                        horizon=5, batch_size=512)
agent = TDMPC(cfg)
agent.model.load_state_dict(synthetic_state_dict(cfg, 21))
agent.model_target.load_state_dict(synthetic_state_dict(cfg, 22))
ref = RefLearner(cfg, synthetic_state_dict(cfg, 21), synthetic_state_dict(cfg, 22))
b = batch(cfg)
H, B, A = cfg.horizon, cfg.batch_size, cfg.action_dim
torch.manual_seed(0)
noise = [torch.empty(B, A).normal_() for _ in range(2 * H + 1)]
torch.manual_seed(0)
m = agent.update(Buf(b), 1, noise=noise)
rm, _ = ref.update(b, 1)
eng = agent.learner().engine
for k, v in ref.p.items():
    if v.grad is None:
        continue
    o, shape = eng.off[k]
    g = eng.G[o:o + v.numel()].view(shape).double().cpu()
    r = v.grad.double()
    err = float((g - r).abs().max() / (r.abs().max() + 1e-30))
    print(f"{k:24s} |g| {float(g.norm()):.4e} ref {float(r.norm()):.4e} rel-max-err {err:.2e}")
print("metrics", m, rm)
