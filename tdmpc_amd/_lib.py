"""ctypes binding of libtdmpc_hip.so (the C ABI declared in include/tdmpc_hip.h).

The library is built in-tree (`python -m tdmpc_amd.build` or `__graft_entry__.build()`). There is no CPU
fallback: if the shared object is missing or fails to load, `lib()` raises.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TDMPC_LIB_PATH") or os.path.join(HERE, "libtdmpc_hip.so")   # override: A/B of builds

ABI_VERSION = 8
PATHS = {"auto": 0, "layered": 1, "chain": 2, "chain32": 3, "chain16": 4, "split": 5, "chain_x6": 6, "split_x6": 7, "chain64": 8, "persist": 9, "wide": 10}

EXPORTED = ("tdmpc_abi_version", "tdmpc_sizes_for", "tdmpc_noise_floats", "tdmpc_num_param_tensors",
            "tdmpc_pack_weights", "tdmpc_pack_forget", "tdmpc_encode", "tdmpc_plan", "tdmpc_estimate_value", "tdmpc_pi_rollout",
            "tdmpc_cem_iter", "tdmpc_reference_normals", "tdmpc_last_error", "tdmpc_debug_plan1_stamps",
            "tdmpc_debug_pack_check",
            "tdmpc_profile_begin", "tdmpc_profile_end", "tdmpc_profile_kernel", "tdmpc_icem_sizes_for", "tdmpc_plan_icem",
            # include/tdmpc_replay.h
            "tdmpc_replay_workspace_bytes", "tdmpc_replay_add_priorities", "tdmpc_replay_update_priorities",
            "tdmpc_replay_sample",
            # include/tdmpc_learner.h
            "tdmpc_loss_forward", "tdmpc_loss_backward", "tdmpc_random_shift", "tdmpc_random_shift_scaled",
            "tdmpc_lg_gemm", "tdmpc_lg_rows_fwd", "tdmpc_lg_rows_bwd", "tdmpc_lg_pi_loss", "tdmpc_lg_finalize",
            "tdmpc_lg_adam", "tdmpc_lg_lerp", "tdmpc_lg_act", "tdmpc_lg_conv_fwd", "tdmpc_lg_conv_bwd_data",
            "tdmpc_lg_conv_bwd_weight")


# tdmpc_plan_params.status bits (include/tdmpc_hip.h)
STATUS_P1_TIMEOUT = 1
STATUS_PACK_STALE = 2


def status_text(st: int) -> str:
    """What a nonzero device status word means (each set bit)."""
    parts = []
    if st & STATUS_P1_TIMEOUT:
        parts.append("the persistent one-env plan timed out at a hand-off -- not every workgroup of its grid was "
                     "resident; set TDMPC_PERSIST=0 to plan on the launch chain instead")
    if st & STATUS_PACK_STALE:
        parts.append("the weight pack found another job table in the packed buffer than the one it was issued for "
                     "(a re-allocated or re-keyed buffer packed under capture without tdmpc_pack_forget): the "
                     "weights are NaN until the next uncaptured pack")
    if st & ~(STATUS_P1_TIMEOUT | STATUS_PACK_STALE):
        parts.append(f"unknown bits {st & ~(STATUS_P1_TIMEOUT | STATUS_PACK_STALE):#x}")
    return "; ".join(parts)


class Dims(C.Structure):
    _fields_ = [(n, C.c_int32) for n in (
        "modality", "obs_dim", "img_c", "img_hw", "num_channels", "action_dim", "latent_dim", "mlp_dim",
        "enc_dim", "num_samples", "num_pi", "num_elites", "max_horizon", "max_iterations", "max_batch",
        "enc_norm")]


class PlanParams(C.Structure):
    _fields_ = [("horizon", C.c_int32), ("iterations", C.c_int32), ("batch", C.c_int32),
                ("warm_start", C.c_int32), ("eval_mode", C.c_int32),
                ("min_std", C.c_float), ("temperature", C.c_float), ("momentum", C.c_float),
                ("one_minus_momentum", C.c_float), ("std_floor", C.c_float),
                ("discount_pow", C.c_float * 17), ("path", C.c_int32),
                ("warm_flags", C.c_void_p), ("std_floor_dev", C.c_void_p), ("status", C.c_void_p)]


class IcemParams(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("horizon", "iterations", "batch", "warm_start", "eval_mode", "has_elites",
                                         "elite_horizon", "n_pi0", "path")] + \
               [("n_samples", C.c_int32 * 16), ("n_pi", C.c_int32 * 16), ("n_elite", C.c_int32 * 16),
                ("samp_off", C.c_int64 * 16), ("term_off", C.c_int64 * 16)] + \
               [(n, C.c_int64) for n in ("reuse_off", "pi_off", "act_off", "env_stride")] + \
               [(n, C.c_float) for n in ("min_std", "temperature", "momentum", "one_minus_momentum", "std_floor",
                                         "init_std")] + [("discount_pow", C.c_float * 17), ("status", C.c_void_p)]


class ReplayDims(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("modality", "obs_dim", "img_hw", "frame_stack", "action_dim",
                                         "episode_length", "capacity", "horizon", "batch_size")]


class ReplayStore(C.Structure):
    _fields_ = [("obs", C.c_void_p), ("last_obs", C.c_void_p), ("action", C.c_void_p), ("reward", C.c_void_p),
                ("priorities", C.c_void_p)]


class LossArgs(C.Structure):   # tdmpc_loss_args (include/tdmpc_learner.h)
    _fields_ = [(n, C.c_void_p) for n in ("zp", "nz", "q1", "q2", "rp", "rw", "td", "w", "rho")] + \
               [("H", C.c_int32), ("B", C.c_int32), ("L", C.c_int32), ("consistency_coef", C.c_float),
                ("reward_coef", C.c_float), ("value_coef", C.c_float)]


class LgSeg(C.Structure):       # tdmpc_lg_seg (include/tdmpc_learner.h)
    _fields_ = [("a", C.c_void_p), ("b", C.c_void_p)] + \
               [(n, C.c_int32) for n in ("lda", "ldb", "k", "amode", "bmode", "ones_col")]


class LgJob(C.Structure):       # tdmpc_lg_job
    _fields_ = [("seg", LgSeg * 3)] + [(n, C.c_int32) for n in ("nseg", "m", "n", "epi")] + \
               [(n, C.c_void_p) for n in ("c", "c2", "bias", "aux", "res")] + \
               [(n, C.c_int32) for n in ("ldc", "ldc2", "ldaux", "ldres")] + \
               [("std_", C.c_float), ("splits", C.c_int32), ("slice", C.c_int64)]


class LgRowHead(C.Structure):   # tdmpc_lg_rowhead
    _fields_ = [(n, C.c_void_p) for n in ("x", "y", "xhat", "rstd", "yact", "g", "beta", "w3", "b3", "out", "dq",
                                          "part")] + \
               [(n, C.c_int32) for n in ("ldx", "ldy", "ln", "act", "tail")]


class LgRows(C.Structure):      # tdmpc_lg_rows
    _fields_ = [("hd", LgRowHead * 3)] + [(n, C.c_int32) for n in ("nh", "rows", "m", "bsz")] + \
               [("reward", C.c_void_p), ("td", C.c_void_p), ("gamma", C.c_float),
                ("q1", C.c_void_p), ("q2", C.c_void_p), ("rho", C.c_void_p)]


class LgConv(C.Structure):      # tdmpc_lg_conv
    _fields_ = [("x", C.c_void_p), ("w", C.c_void_p * 2), ("b", C.c_void_p * 2), ("y", C.c_void_p * 2)] + \
               [(n, C.c_int32) for n in ("nprob", "n", "cin", "hin", "k")] + [("in_div", C.c_float)]


class LgGsrc(C.Structure):      # tdmpc_lg_gsrc
    _fields_ = [("src", C.c_void_p), ("dst", C.c_int64), ("sstride", C.c_int64)] + \
               [(n, C.c_int32) for n in ("rows", "cols", "ld", "nslices")]


class Sizes(C.Structure):
    _fields_ = [("packed_weight_bytes", C.c_size_t), ("workspace_bytes", C.c_size_t),
                ("noise_floats_per_env", C.c_size_t)]


_LIB = None


def lib():
    """Load (once) and return the library. Raises if it is not built: no silent fallback."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is missing: build it with `python -m tdmpc_amd.build` "
                           "(hipcc --offload-arch=gfx950). The planner has no CPU fallback.")
    import torch  # noqa: F401  -- load torch's libamdhip64 first so both share one HIP runtime
    L = C.CDLL(LIB_PATH)
    vp, i32, sz = C.c_void_p, C.c_int32, C.c_size_t
    L.tdmpc_abi_version.restype = C.c_int
    L.tdmpc_debug_plan1_stamps.argtypes = [vp]
    L.tdmpc_sizes_for.argtypes = [C.POINTER(Dims), C.POINTER(Sizes)]
    L.tdmpc_noise_floats.argtypes = [C.POINTER(Dims), i32, i32]
    L.tdmpc_noise_floats.restype = sz
    L.tdmpc_num_param_tensors.argtypes = [C.POINTER(Dims)]
    L.tdmpc_reference_normals.argtypes = [C.POINTER(Dims), vp, i32, C.c_int64, i32, i32, i32, C.c_uint64,
                                          C.c_uint64, vp, i32, C.POINTER(C.c_uint64), vp]
    L.tdmpc_pack_weights.argtypes = [C.POINTER(Dims), C.POINTER(vp), i32, vp, sz, vp]
    L.tdmpc_pack_forget.argtypes = [vp]
    if hasattr(L, "tdmpc_debug_pack_check"):   # (diagnostic; absent from older builds used in A/B runs)
        L.tdmpc_debug_pack_check.argtypes = [C.POINTER(Dims), C.POINTER(C.c_int64), i32]
    L.tdmpc_encode.argtypes = [C.POINTER(Dims), vp, vp, i32, i32, vp, vp, vp]
    L.tdmpc_plan.argtypes = [C.POINTER(Dims), C.POINTER(PlanParams), vp, vp, i32, vp, vp, vp, vp, vp,
                             vp, vp, vp, vp, vp, vp, sz, vp]
    L.tdmpc_estimate_value.argtypes = [C.POINTER(Dims), C.POINTER(PlanParams), vp, vp, vp, vp, i32, vp, vp,
                                       vp, vp, sz, vp]
    L.tdmpc_pi_rollout.argtypes = [C.POINTER(Dims), C.POINTER(PlanParams), vp, vp, vp, vp, vp, sz, vp]
    L.tdmpc_cem_iter.argtypes = [C.POINTER(Dims), C.POINTER(PlanParams), vp, vp, vp, vp, vp, vp, vp, vp, vp, vp,
                                 vp, vp, sz, vp]
    L.tdmpc_last_error.restype = C.c_char_p
    L.tdmpc_profile_kernel.restype = C.c_char_p
    L.tdmpc_profile_begin.argtypes = [i32, i32, i32, i32, i32]
    L.tdmpc_profile_end.argtypes = [C.POINTER(C.c_int32), C.POINTER(C.c_double), C.POINTER(C.c_double)]
    L.tdmpc_icem_sizes_for.argtypes = [C.POINTER(Dims), C.POINTER(Sizes)]
    L.tdmpc_plan_icem.argtypes = [C.POINTER(Dims), C.POINTER(IcemParams), vp, vp, i32, vp, vp, vp, vp, vp, vp,
                                  vp, vp, vp, vp, sz, vp]
    L.tdmpc_replay_workspace_bytes.argtypes = [C.POINTER(ReplayDims)]
    L.tdmpc_replay_workspace_bytes.restype = sz
    L.tdmpc_replay_add_priorities.argtypes = [C.POINTER(ReplayDims), vp, i32, i32, vp, sz, vp]
    L.tdmpc_replay_update_priorities.argtypes = [C.POINTER(ReplayDims), vp, vp, vp, i32, C.c_float, vp, sz, vp]
    L.tdmpc_replay_sample.argtypes = [C.POINTER(ReplayDims), C.POINTER(ReplayStore), i32, i32, C.c_float,
                                      C.c_float, vp, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, sz, vp]
    L.tdmpc_loss_forward.argtypes = [C.POINTER(LossArgs), vp, vp, vp]
    L.tdmpc_loss_backward.argtypes = [C.POINTER(LossArgs), vp, vp, vp, vp, vp, vp, vp, vp]
    L.tdmpc_random_shift.argtypes = [vp, vp, i32, i32, i32, i32, i32, vp, vp]
    L.tdmpc_random_shift_scaled.argtypes = [vp, vp, i32, i32, i32, i32, i32, C.c_float, vp, vp]
    L.tdmpc_lg_gemm.argtypes = [C.POINTER(LgJob), i32, i32, vp]
    L.tdmpc_lg_rows_fwd.argtypes = [C.POINTER(LgRows), vp]
    L.tdmpc_lg_rows_bwd.argtypes = [C.POINTER(LgRows), i32, vp]
    L.tdmpc_lg_pi_loss.argtypes = [vp, vp, vp, i32, i32, vp, vp]
    L.tdmpc_lg_finalize.argtypes = [C.POINTER(LgGsrc), i32, vp, vp, i32, vp, vp]
    L.tdmpc_lg_adam.argtypes = [vp, vp, vp, vp, C.c_int64, vp, i32, vp, C.c_float, C.c_float, C.c_float,
                                C.c_float, C.c_float, vp, vp]
    L.tdmpc_lg_lerp.argtypes = [vp, vp, C.c_int64, C.c_float, vp]
    L.tdmpc_lg_act.argtypes = [vp, vp, C.c_int64, i32, vp]
    L.tdmpc_lg_conv_fwd.argtypes = [C.POINTER(LgConv), vp]
    L.tdmpc_lg_conv_bwd_data.argtypes = [vp, vp, vp, vp, i32, i32, i32, i32, vp]
    L.tdmpc_lg_conv_bwd_weight.argtypes = [vp, vp, C.c_float, vp, i32, i32, i32, i32, i32, vp]
    for name in EXPORTED:
        if not hasattr(L, name) and not (name.startswith("tdmpc_debug_") and os.environ.get("TDMPC_LIB_PATH")):
            raise RuntimeError(f"{LIB_PATH} does not export {name}")
    if L.tdmpc_abi_version() != ABI_VERSION:
        raise RuntimeError("libtdmpc_hip ABI version mismatch")
    _LIB = L
    return L


def check(rc: int, what: str):
    if rc != 0:
        msg = lib().tdmpc_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed with code {rc}: {msg}")


def dims_from_cfg(cfg, max_batch: int = 1, max_horizon=None, max_iterations=None, enc_norm: bool = False) -> Dims:
    d = Dims()
    pixels = cfg.modality == "pixels"
    d.modality = 1 if pixels else 0
    d.obs_dim = 0 if pixels else int(cfg.obs_shape[0])
    d.img_c = int(3 * cfg.frame_stack) if pixels else 0
    d.img_hw = int(cfg.img_size) if pixels else 0
    d.num_channels = int(cfg.num_channels) if pixels else 0
    d.action_dim = int(cfg.action_dim)
    d.latent_dim = int(cfg.latent_dim)
    d.mlp_dim = int(cfg.mlp_dim)
    d.enc_dim = int(cfg.enc_dim)
    d.num_samples = int(cfg.num_samples)
    d.num_pi = int(cfg.mixture_coef * cfg.num_samples)
    d.num_elites = int(cfg.num_elites)
    d.max_horizon = int(max_horizon or cfg.horizon)
    d.max_iterations = int(max_iterations or cfg.iterations)
    d.max_batch = int(max_batch)
    d.enc_norm = int(bool(enc_norm))
    return d


def ptr(t) -> int:
    return 0 if t is None else t.data_ptr()
