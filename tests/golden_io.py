"""Load the golden fixtures written by tests/golden/make_golden.py (data only; no reference code)."""
import glob
import json
import os

import numpy as np
import torch

from tdmpc_amd.config import make_cfg
from oracle.tdmpc_ref import NoiseBundle

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def case_names():
    """The plan() golden cases (make_golden.py); replay_* / learner_* / icem_* belong to their own tests."""
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "*.npz"))
                  if not os.path.basename(p).startswith(("replay_", "learner_", "icem_")))


def load_case(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    d = {k: z[k] for k in z.files}
    ov = json.loads(str(d["ov_json"]))
    cfg = make_cfg(str(d["task"]), **ov)
    return cfg, int(d["wseed"]), d


def call_noise(d, ci):
    if f"c{ci}_seed_action" in d:
        return NoiseBundle(eps_pi=None, seed_action=torch.from_numpy(d[f"c{ci}_seed_action"]))
    nb = NoiseBundle(eps_pi=torch.from_numpy(d[f"c{ci}_eps_pi"]) if f"c{ci}_eps_pi" in d else None)
    nb.eps_cem = [torch.from_numpy(x) for x in d[f"c{ci}_eps_cem"]]
    nb.eps_term = [torch.from_numpy(x) for x in d[f"c{ci}_eps_term"]]
    nb.u = float(d[f"c{ci}_u"])
    if f"c{ci}_eps_act" in d:
        nb.eps_act = torch.from_numpy(d[f"c{ci}_eps_act"])
    return nb
