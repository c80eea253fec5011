"""CPU-side checks of the C ABI library and host logic (no GPU needed)."""
import ctypes as C
import re

import numpy as np
import pytest

from tdmpc_amd import _lib
from tdmpc_amd.config import bench_cfg, linear_schedule, make_cfg
from oracle import tdmpc_ref

HEADER = "include/tdmpc_hip.h"


def _declared():
    import glob
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    names = set()
    for hdr in sorted(glob.glob(os.path.join(root, "include", "*.h"))):
        src = open(hdr).read()
        names |= set(re.findall(r"^(?:int|size_t|const char\*)\s+(tdmpc_\w+)\(", src, re.M))
    return sorted(names)


def test_library_exports_every_declared_symbol():
    L = _lib.lib()
    names = _declared()
    assert "tdmpc_plan" in names and "tdmpc_replay_sample" in names and "tdmpc_loss_forward" in names
    assert len(names) >= 14
    for n in names:
        assert hasattr(L, n), n
    assert L.tdmpc_abi_version() == _lib.ABI_VERSION == 8


@pytest.mark.parametrize("name", ["cartpole-swingup", "cheetah-run", "humanoid-run", "humanoid-run-l512",
                                  "dog-run", "quadruped-run-pixels"])
def test_sizes_for_bench_configs(name):
    cfg = bench_cfg(name)
    d = _lib.dims_from_cfg(cfg, max_batch=8)
    s = _lib.Sizes()
    assert _lib.lib().tdmpc_sizes_for(C.byref(d), C.byref(s)) == 0
    assert s.packed_weight_bytes > 4 * 1_000_000
    N, P, A = d.num_samples, d.num_pi, d.action_dim
    H, I = d.max_horizon, d.max_iterations
    assert s.noise_floats_per_env == H * P * A + I * (H * N * A + (N + P) * A) + A
    assert _lib.lib().tdmpc_num_param_tensors(C.byref(d)) == (10 if cfg.modality == "pixels" else 4) + 38


def test_bad_dims_rejected():
    cfg = make_cfg("humanoid")
    d = _lib.dims_from_cfg(cfg)
    d.mlp_dim = 500  # not a multiple of 64
    s = _lib.Sizes()
    assert _lib.lib().tdmpc_sizes_for(C.byref(d), C.byref(s)) == -1
    assert _lib.lib().tdmpc_sizes_for(None, C.byref(s)) == -3


@pytest.mark.parametrize("sched", ["linear(2, 5, 25000, 0)", "linear(0.5, 0.05, 25000, 0)", "0.3", 1.5])
def test_linear_schedule(sched):
    for step in [0, 1, 100, 12500, 24999, 25000, 10**6]:
        assert linear_schedule(sched, step) == tdmpc_ref.linear_schedule(sched, step)


def test_discount_pows_match_python_accumulation():
    from tdmpc_amd.tdmpc import _discount_pows
    d, ref = 1, []
    for _ in range(6):
        ref.append(float(np.float32(d)))
        d *= 0.99
    assert _discount_pows(0.99, 5) == ref


def test_entry_points_reject_null_arguments():
    """Every compute entry point checks its required pointers before touching the device: TDMPC_E_NULL (-3)."""
    L = _lib.lib()
    cfg = make_cfg("humanoid")
    d = _lib.dims_from_cfg(cfg)
    prm = _lib.PlanParams()
    prm.horizon, prm.iterations, prm.batch = 5, 6, 1
    E_NULL = -3
    assert L.tdmpc_plan(C.byref(d), C.byref(prm), None, None, 0, None, None, None, None, None, None, None, None,
                        None, None, None, 0, None) == E_NULL
    assert L.tdmpc_estimate_value(C.byref(d), C.byref(prm), None, None, None, None, 768, None, None, None, None, 0,
                                  None) == E_NULL
    assert L.tdmpc_pi_rollout(C.byref(d), C.byref(prm), None, None, None, None, None, 0, None) == E_NULL
    assert L.tdmpc_cem_iter(C.byref(d), C.byref(prm), None, None, None, None, None, None, None, None, None, None,
                            None, None, 0, None) == E_NULL
    assert L.tdmpc_encode(C.byref(d), None, None, 0, 1, None, None, None) == E_NULL
    assert L.tdmpc_pack_weights(C.byref(d), None, 0, None, 0, None) == E_NULL
    adv = C.c_uint64(0)
    assert L.tdmpc_reference_normals(C.byref(d), None, 1, 10**6, 5, 6, 0, 1, 0, None, 2048, C.byref(adv), None) == E_NULL
    # shape checks before any launch: an env stride shorter than the stream, too many draws
    x = C.c_void_p(16)
    S = L.tdmpc_noise_floats(C.byref(d), 5, 6)
    assert L.tdmpc_reference_normals(C.byref(d), x, 1, S - 1, 5, 6, 0, 1, 0, None, 2048, C.byref(adv), None) == -1
    assert L.tdmpc_reference_normals(C.byref(d), x, 1, 10**9, 16, 60, 0, 1, 0, None, 2048, C.byref(adv), None) == -1
    assert b"draws" in L.tdmpc_last_error()
    # learner engine (include/tdmpc_learner.h)
    assert L.tdmpc_lg_gemm(None, 1, 1, None) == E_NULL
    assert L.tdmpc_lg_lerp(None, None, 16, 0.5, None) == E_NULL
    assert L.tdmpc_lg_act(None, None, 16, 0, None) == E_NULL
    assert L.tdmpc_lg_adam(None, None, None, None, 16, None, 1, None, 1e-3, 0.9, 0.999, 1e-8, 10.0, None,
                           None) == E_NULL


def test_learner_entry_points_reject_bad_shapes():
    """Shape / mode checks run before any launch: TDMPC_E_DIMS (-1), the message in tdmpc_last_error."""
    L = _lib.lib()
    E_DIMS = -1
    x = C.c_void_p(16)   # never dereferenced: the checks fail first
    assert L.tdmpc_lg_act(x, None, 6, 0, None) == E_DIMS            # n not a multiple of 4
    assert L.tdmpc_lg_act(x, None, 16, 2, None) == E_DIMS           # unknown mode
    assert L.tdmpc_lg_act(x, None, 16, 1, None) == -3               # mode 1 needs the activation
    jobs = (_lib.LgJob * 1)()
    assert L.tdmpc_lg_gemm(jobs, 0, 1, None) == E_DIMS              # no jobs
    assert L.tdmpc_lg_gemm(jobs, 1, 7, None) == E_DIMS              # unknown tile
    assert L.tdmpc_lg_gemm(jobs, 1, 1, None) == E_DIMS              # job without an output / shape


def test_packed_buffer_holds_the_x6_copy():
    """The packed weight buffer carries the x6 (three bf16 planes) copy of the chain kernels' panels next to the
    fp32 ones: at humanoid sizes 6 bytes per panel weight on top of the 4 (tdmpc_kernels.hip Layout::x6)."""
    cfg = bench_cfg("humanoid-run")
    d = _lib.dims_from_cfg(cfg, max_batch=1)
    s = _lib.Sizes()
    assert _lib.lib().tdmpc_sizes_for(C.byref(d), C.byref(s)) == 0
    M, L, A = cfg.mlp_dim, cfg.latent_dim, cfg.action_dim
    r32 = lambda x: -(-x // 32) * 32
    r16 = lambda x: -(-x // 16) * 16
    Ap, Lp = -(-A // 8) * 8, -(-L // 8) * 8
    Kx = Ap + Lp
    x6 = 3 * (2 * M * r16(Kx) + 3 * M * M + r32(L) * M + M * r16(Lp) + r32(A) * M + 2 * M * r16(Kx) + 2 * M * M)
    assert s.packed_weight_bytes >= 2 * x6
