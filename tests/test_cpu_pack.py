"""The fused weight pack's job table (tdmpc_pack_weights, one launch) bounds-checked on the host for every model
family the packer serves: each job writes inside the packed layout and reads inside its source tensor
(tdmpc_debug_pack_check runs no HIP call, so this holds on the CPU-only driver)."""
import ctypes as C

import pytest

from tdmpc_amd import _lib
from tdmpc_amd.config import make_cfg
from tdmpc_amd.told import TOLD


@pytest.mark.parametrize("task,kw", [("humanoid", {}), ("dog", {}), ("cheetah", {}), ("quadruped", {}),
                                     ("humanoid", {"latent_dim": 512}), ("cheetah", {"modality": "pixels"})])
def test_pack_jobs_in_bounds(task, kw):
    cfg = make_cfg(task, **kw)
    sd = TOLD(cfg).state_dict()
    L = _lib.lib()
    dims = _lib.dims_from_cfg(cfg, max_batch=1)
    n = len(sd)
    assert n == L.tdmpc_num_param_tensors(C.byref(dims))
    numel = (C.c_int64 * n)(*[v.numel() for v in sd.values()])
    rc = L.tdmpc_debug_pack_check(C.byref(dims), numel, n)
    assert rc > 0, L.tdmpc_last_error().decode()
