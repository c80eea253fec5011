"""Checkpoint interop with the reference: `tdmpc_amd.told.TOLD` has the reference TOLD's
state_dict layout (keys, order, shapes) and initialisation, so `{'model', 'model_target'}` checkpoints move
between the reference's `TDMPC.save/load` (tdmpc.py:68-81) and the drop-in in both directions.

Pinned by tests/golden/told_layout.json, recorded from the reference TOLD itself (make_told_fixture.py)."""
import json
import os

import numpy as np
import pytest
import torch

from tdmpc_amd.config import bench_cfg
from tdmpc_amd.told import TOLD, synthetic_state_dict

LAYOUT = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "told_layout.json")))


@pytest.mark.parametrize("name", sorted(LAYOUT))
def test_told_layout_and_init_match_reference(name):
    cfg = bench_cfg(name)
    torch.manual_seed(0)
    sd = TOLD(cfg).state_dict()
    ref = LAYOUT[name]
    assert [k for k, *_ in ref] == list(sd.keys())
    for (k, shape, s1, s2), v in zip(ref, sd.values()):
        assert list(v.shape) == shape, k
        v = v.double()
        # same nn.init calls in the same order on the same generator: the sums agree to rounding
        np.testing.assert_allclose(float(v.sum()), s1, rtol=1e-9, atol=1e-9, err_msg=k)
        np.testing.assert_allclose(float((v ** 2).sum()), s2, rtol=1e-9, atol=1e-9, err_msg=k)


@pytest.mark.parametrize("name", ["humanoid-run", "quadruped-run-pixels"])
def test_reference_format_checkpoint_round_trip(name, tmp_path):
    from tdmpc_amd.tdmpc import load_checkpoint
    cfg = bench_cfg(name)
    src = TOLD(cfg, init="none")
    src.load_state_dict(synthetic_state_dict(cfg, 3))
    tgt = TOLD(cfg, init="none")
    tgt.load_state_dict(synthetic_state_dict(cfg, 4))
    fp = tmp_path / "model.pt"
    # exactly what the reference's TDMPC.save writes (tdmpc.py:68-75)
    torch.save({"model": src.state_dict(), "model_target": tgt.state_dict()}, fp)
    m, mt = TOLD(cfg), TOLD(cfg)
    load_checkpoint(fp, m, mt)
    for a, b in zip(m.state_dict().values(), src.state_dict().values()):
        assert torch.equal(a, b)
    for a, b in zip(mt.state_dict().values(), tgt.state_dict().values()):
        assert torch.equal(a, b)
    # a checkpoint with a missing or renamed key is refused (strict load), not silently half-applied
    bad = {"model": {("x" + k): v for k, v in src.state_dict().items()}, "model_target": tgt.state_dict()}
    torch.save(bad, fp)
    with pytest.raises(RuntimeError):
        load_checkpoint(fp, TOLD(cfg), TOLD(cfg))


@pytest.mark.gpu
def test_loaded_checkpoint_drives_the_planner(tmp_path):
    """save -> load into a fresh agent -> the planner repacks and plans bitwise like the source agent."""
    from oracle import tdmpc_ref
    from tdmpc_amd.config import make_cfg
    from tdmpc_amd.tdmpc import TDMPC
    cfg = make_cfg("humanoid", num_samples=128, num_elites=16, iterations=3)
    a1 = TDMPC(cfg)
    a1.model.load_state_dict(synthetic_state_dict(cfg, 8))
    a1.std = 0.05
    fp = tmp_path / "ckpt.pt"
    a1.save(fp)
    a2 = TDMPC(cfg)
    a2.std = 0.05
    obs = np.random.RandomState(0).standard_normal(cfg.obs_shape).astype(np.float32)
    torch.manual_seed(1)
    nb = tdmpc_ref.draw_noise(cfg, 10**6, False)
    r_before, _ = a2._plan_envs(obs[None], False, 10**6, [True], noise=[nb])
    r_before = r_before.clone()
    a2.load(fp)
    x1, _ = a1._plan_envs(obs[None], False, 10**6, [True], noise=[nb])
    x2, _ = a2._plan_envs(obs[None], False, 10**6, [True], noise=[nb])
    assert torch.equal(x1, x2)
    assert not torch.equal(r_before, x2)   # the new weights were repacked, not the old ones reused
