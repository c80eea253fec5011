import torch, numpy as np, sys
sys.path.insert(0, '.')
from types import SimpleNamespace
from tdmpc_amd.learner import RandomShiftsAug
aug = RandomShiftsAug(SimpleNamespace(img_size=84, modality="pixels"))
x = torch.randint(0, 256, (48, 9, 84, 84), device="cuda").float()
torch.manual_seed(3); e1 = aug(x).clone(); e2 = aug(x).clone()
g = torch.cuda.CUDAGraph()
torch.manual_seed(3)
with torch.cuda.graph(g):
    o = aug(x)
torch.manual_seed(3)
g.replay(); r1 = o.clone(); g.replay(); r2 = o.clone()
print("graph==eager", torch.equal(e1, r1), torch.equal(e2, r2))
