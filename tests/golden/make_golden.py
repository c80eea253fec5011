"""Generate the golden vectors under tests/golden/ by running the REFERENCE `TDMPC.plan` in this container.

Run once in the build container (where /root/reference exists):   python tests/golden/make_golden.py
The GPU box never runs this file; tests only read the .npz files it writes.

How the reference is imported (SURVEY.md §8c "Import recipe"):
  1. sys.dont_write_bytecode -- leave nothing behind in /root/reference;
  2. a stub module for `rlpyt.ul.models.ul.encoders` (helper.py:12 imports it; used only by
     `dmlab_enc_norm`, which is not on the TDMPC path);
  3. sys.path += /root/reference/src, so `algorithm.tdmpc` / `algorithm.helper` import as in the reference;
  4. `torch.nn.Module.cuda` patched to identity (tdmpc.py:60 calls `.cuda()`; there is no GPU here);
  5. cfg is a SimpleNamespace with the attributes TDMPC reads (omegaconf is not installed).

For each case the reference plan() is called several times in a row (t0 / warm-start / eval mixes) from
fixed torch+numpy seeds. The noise those calls drew is re-drawn from the same seeds with
`oracle.tdmpc_ref.draw_noise`, and everything (inputs, noise, reference outputs, per-iteration traces from
the reference's own estimate_value via a wrapper) is written to an .npz.
"""
from __future__ import annotations

import json
import os
import sys
import types

import numpy as np
import torch

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from tdmpc_amd.config import make_cfg  # noqa: E402
from tdmpc_amd.told import synthetic_state_dict  # noqa: E402
from oracle import tdmpc_ref  # noqa: E402

REF_SRC = "/root/reference/src"


def import_reference():
    stub = types.ModuleType("rlpyt.ul.models.ul.encoders")
    stub.DmlabEncoderModelNorm = object
    for name in ("rlpyt", "rlpyt.ul", "rlpyt.ul.models", "rlpyt.ul.models.ul"):
        sys.modules.setdefault(name, types.ModuleType(name))
    sys.modules["rlpyt.ul.models.ul.encoders"] = stub
    sys.path.insert(0, REF_SRC)
    torch.nn.Module.cuda = lambda self, *a, **k: self
    import algorithm.tdmpc as ref_tdmpc  # noqa
    return ref_tdmpc


# (name, task, overrides, weight seed, call schedule [(step, t0, eval_mode)])
CASES = [
    ("cartpole_n64", "cartpole", dict(num_samples=64, num_elites=32, iterations=3, horizon=5),
     1, [(10**6, True, False), (10**6, False, False), (10**6, False, True), (10**6, True, True)]),
    ("humanoid_n64", "humanoid", dict(num_samples=64, num_elites=16, iterations=3, horizon=5),
     2, [(10**6, True, False), (10**6, False, False), (10**6, False, True)]),
    ("dog_n64", "dog", dict(num_samples=64, num_elites=16, iterations=2, horizon=5),
     3, [(10**6, True, True), (10**6, False, False)]),
    # horizon schedule mid-way (H=3) and a seed-step call (uniform action, no model)
    ("cheetah_sched", "cheetah", dict(num_samples=32, num_elites=8, iterations=2, horizon=5),
     4, [(10000, True, False), (100, True, False), (12000, False, False)]),
    ("cheetah_nopi", "cheetah", dict(num_samples=32, num_elites=8, iterations=2, horizon=4, mixture_coef=0.0),
     5, [(10**6, True, False), (10**6, False, False)]),
    ("quadpix_n32", "quadruped", dict(modality="pixels", num_samples=32, num_elites=8, iterations=2, horizon=3),
     6, [(10**6, True, False)]),
]


def ref_cfg(cfg):
    c = types.SimpleNamespace(**vars(cfg))
    c.device = "cpu"
    return c


def run_case(ref_tdmpc, name, task, ov, wseed, calls):
    cfg = make_cfg(task, **ov)
    sd = synthetic_state_dict(cfg, wseed)
    agent = ref_tdmpc.TDMPC(ref_cfg(cfg))
    msd = agent.model.state_dict()
    assert list(msd.keys()) == list(sd.keys()), "state_dict layout differs from the reference"
    agent.model.load_state_dict(sd)
    agent.std = 0.05  # trained-regime value of std_schedule; tdmpc.py:59/196

    # record what the reference's estimate_value returned each iteration
    rec = {"value": [], "reward_mean": []}
    orig_ev = agent.estimate_value

    def ev(z, actions, horizon):
        v, rm = orig_ev(z, actions, horizon)
        rec["value"].append(v.clone())
        rec["reward_mean"].append(rm)
        return v, rm
    agent.estimate_value = ev

    rs = np.random.RandomState(100 + wseed)
    out = {"task": task, "wseed": wseed, "ov_json": json.dumps(ov), "ncalls": len(calls)}
    torch.manual_seed(1000 + wseed)
    np.random.seed(2000 + wseed)
    rng_torch = torch.get_rng_state()
    rng_np = np.random.get_state()
    obs_list = []
    for ci, (step, t0, ev_mode) in enumerate(calls):
        if cfg.modality == "pixels":
            obs = rs.randint(0, 256, size=cfg.obs_shape).astype(np.uint8)
        else:
            obs = rs.standard_normal(cfg.obs_shape).astype(np.float32)
        obs_list.append(obs)
        rec["value"].clear(); rec["reward_mean"].clear()
        a, m = agent.plan(obs, eval_mode=ev_mode, step=step, t0=t0)
        out[f"c{ci}_obs"] = obs
        out[f"c{ci}_call"] = np.array([step, int(t0), int(ev_mode)], dtype=np.int64)
        out[f"c{ci}_action"] = a.numpy().copy()
        out[f"c{ci}_metrics"] = np.array([m["external_reward_mean"], m["current_std"]], dtype=np.float64)
        if rec["value"]:
            out[f"c{ci}_values"] = torch.stack(rec["value"]).squeeze(-1).numpy()
            out[f"c{ci}_reward_means"] = np.array(rec["reward_mean"], dtype=np.float64)
        if hasattr(agent, "_prev_mean"):
            out[f"c{ci}_prev_mean"] = agent._prev_mean.numpy().copy()

    # Re-draw the same noise with the oracle's draw order and store it.
    torch.set_rng_state(rng_torch)
    np.random.set_state(rng_np)
    for ci, (step, t0, ev_mode) in enumerate(calls):
        nb = tdmpc_ref.draw_noise(cfg, step, ev_mode)
        if nb.seed_action is not None:
            out[f"c{ci}_seed_action"] = nb.seed_action.numpy()
            continue
        if nb.eps_pi is not None:
            out[f"c{ci}_eps_pi"] = nb.eps_pi.numpy()
        out[f"c{ci}_eps_cem"] = torch.stack(nb.eps_cem).numpy()
        out[f"c{ci}_eps_term"] = torch.stack(nb.eps_term).numpy()
        out[f"c{ci}_u"] = np.float64(nb.u)
        if nb.eps_act is not None:
            out[f"c{ci}_eps_act"] = nb.eps_act.numpy()
    # fingerprint of the synthetic weights so tests notice if the generator changes
    out["w_fingerprint"] = np.array([float(v.double().sum()) for v in sd.values()], dtype=np.float64)
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path} ({os.path.getsize(path)} bytes)")


def main():
    ref_tdmpc = import_reference()
    torch.set_num_threads(1)
    for case in CASES:
        run_case(ref_tdmpc, *case)


if __name__ == "__main__":
    main()
