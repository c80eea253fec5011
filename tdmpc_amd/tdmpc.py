"""`TDMPC`: drop-in replacement for the reference agent's planning API on MI355X.

Reference: `TDMPC` in /root/reference/src/algorithm/tdmpc.py:53-163. The class keeps the reference's
constructor argument (a cfg namespace), attributes (`cfg`, `device`, `std`, `model`, `model_target`,
`_prev_mean`), `plan(obs, eval_mode=False, step=None, t0=True) -> (action tensor [A], metrics dict)`,
`state_dict / save / load`. Planning runs entirely in the HIP library (libtdmpc_hip.so, include/tdmpc_hip.h):
Python only draws the random numbers (in the reference's order, from torch's and numpy's global generators)
and launches one `tdmpc_plan` call. `update` / `update_pi` / `_td_target` (the learner) run on the GPU in
tdmpc_amd/learner.py, replayed from a HIP graph.

Extensions beyond the reference API:
  * `plan_batch(obs[B], ...)` plans B independent environments in one call (one launch sequence, rows of
    all envs stacked), with per-env state (`_prev_mean` per env).
  * `rng="fused"` draws all of a call's Gaussian noise with one generator call instead of the reference's
    18 separate draws (same distribution, different stream).
  * `graph=True` (the default) replays each call -- the reference-order draws included -- from one HIP graph per
    (horizon, iterations, batch, eval_mode); self.std and the per-env warm starts are read from device memory,
    so the graph serves every call. Equal, bitwise, to `graph=False` (eager launches).
  * `path` picks the kernel family: "auto" (by row count), "layered" (one fused GEMM per Linear) or "chain"
    (one row-block kernel per TOLD head); all agree within the fp32 parity tolerance.
"""
from __future__ import annotations

import ctypes as C
import os
from copy import deepcopy

import numpy as np
import torch

from . import _lib
from .config import linear_schedule
from .told import TOLD


def _discount_pows(discount: float, H: int):
    """float32(discount ** t) for t = 0..H as the reference accumulates it (`discount *= cfg.discount`
    on a Python float starting from the int 1, tdmpc.py:86-90)."""
    out, d = [], 1
    for _ in range(H + 1):
        out.append(float(np.float32(d)))
        d *= discount
    return out


def load_checkpoint(fp, model, model_target, device="cpu"):
    """Load a reference checkpoint -- `{'model': sd, 'model_target': sd}` as written by the reference's
    `TDMPC.save` (tdmpc.py:68-81; logger.py:126-133 saves `agent.state_dict()` the same way) -- into TOLD
    modules with the reference's key names. Loaded with weights_only=True (nothing in the file executes) and
    strict key matching; the planner repacks the new tensors on its next call."""
    d = torch.load(fp, map_location=device, weights_only=True)
    model.load_state_dict(d["model"])
    model_target.load_state_dict(d["model_target"])


def pack_told(pl, model):
    """Pack `model`'s parameters (reference state_dict order) into pl.packed through tdmpc_pack_weights when any
    of them changed since the last call (pl: an object with L, dims, device, packed and the _packed_* cache)."""
    if pl._packed_key is not None and pl._packed_model is model:
        key = tuple((p.data_ptr(), p._version) for p in pl._packed_params)
        if key == pl._packed_key:
            return
    params = list(model.state_dict().values())
    if pl._packed_model is not None and pl._packed_model is not model:
        # another model object: re-key the buffer's job table (a graph captured over the old model's pack -- the
        # learner's update -- then fails loudly if replayed, TDMPC_STATUS_PACK_STALE, instead of packing this one)
        pl.L.tdmpc_pack_forget(C.c_void_p(pl.packed.data_ptr()))
    pl._packed_model, pl._packed_params = model, params
    key = tuple((p.data_ptr(), p._version) for p in params)
    params = [p.detach().to(pl.device, torch.float32).contiguous() for p in params]
    # a source that is not the model's own device fp32 tensor is copied into a staging tensor kept per planner, so the
    # pointer set -- the key of the library's device job-table cache -- stays the same from one repack to the next
    stage = getattr(pl, "_pack_stage", None)
    if stage is None or len(stage) != len(params):
        stage = pl._pack_stage = [None] * len(params)
    for i, (q, p) in enumerate(zip(params, pl._packed_params)):
        if q.data_ptr() != p.data_ptr():
            if stage[i] is None or stage[i].shape != q.shape:
                stage[i] = torch.empty_like(q)
            stage[i].copy_(q)
            params[i] = stage[i]
    n = pl.L.tdmpc_num_param_tensors(C.byref(pl.dims))
    if n != len(params):
        raise ValueError(f"TOLD has {len(params)} tensors, the packer expects {n}")
    arr = (C.c_void_p * n)(*[p.data_ptr() for p in params])
    stream = torch.cuda.current_stream(pl.device).cuda_stream
    _lib.check(pl.L.tdmpc_pack_weights(C.byref(pl.dims), arr, n, C.c_void_p(pl.packed.data_ptr()),
                                        pl.packed.numel() * 4, C.c_void_p(stream)), "tdmpc_pack_weights")
    pl._keep = params  # keep source tensors alive until the stream has consumed them
    pl._packed_key = key
    # the pointer array stays valid for repack_live() while the packed tensors ARE the model's (no dtype / device
    # / layout copy was made)
    live = all(q.data_ptr() == p.data_ptr() for q, p in zip(params, pl._packed_params))
    pl._ptr_arr = (arr, n) if live else None


def repack_live(pl, model) -> bool:
    """Repack after an in-place update of the tensors the last pack_told() read (the learner's flat-buffer views,
    written by its HIP optimizer): one tdmpc_pack_weights launch over the cached pointer array -- no state_dict()
    walk, capturable into the learner's update graph. False (nothing launched) when the planner has not packed
    this model's live tensors yet: the next plan() then packs from the state_dict."""
    if pl._packed_model is not model or getattr(pl, "_ptr_arr", None) is None:
        return False
    arr, n = pl._ptr_arr
    stream = torch.cuda.current_stream(pl.device).cuda_stream
    _lib.check(pl.L.tdmpc_pack_weights(C.byref(pl.dims), arr, n, C.c_void_p(pl.packed.data_ptr()),
                                        pl.packed.numel() * 4, C.c_void_p(stream)), "tdmpc_pack_weights")
    return True


class HipPlanner:
    """Owns the device buffers of one planner instance and calls the C ABI."""

    def __init__(self, cfg, max_batch: int = 1, device=None, path: str = "auto"):
        self.cfg = cfg
        if path not in _lib.PATHS:
            raise ValueError(f"path must be one of {sorted(_lib.PATHS)}")
        self.path = path
        self.device = torch.device(device or "cuda")
        self.L = _lib.lib()
        self.dims = _lib.dims_from_cfg(cfg, max_batch=max_batch)
        sz = _lib.Sizes()
        _lib.check(self.L.tdmpc_sizes_for(C.byref(self.dims), C.byref(sz)), "tdmpc_sizes_for")
        self.sizes = sz
        dev = self.device
        # zeroed once: tdmpc_pack_weights writes every tensor's region (padding included) but not the alignment gaps
        # between them, which padded vector reads may touch
        self.packed = torch.zeros(sz.packed_weight_bytes // 4, dtype=torch.float32, device=dev)
        self.L.tdmpc_pack_forget(C.c_void_p(self.packed.data_ptr()))   # (the address may be a freed buffer's)
        self.workspace = torch.empty(sz.workspace_bytes // 4, dtype=torch.float32, device=dev)
        d = self.dims
        self.N, self.P, self.A = d.num_samples, d.num_pi, d.action_dim
        self.T = self.N + self.P
        self.max_batch = max_batch
        # Env streams are packed with the CALL's per-env size (depends on H and I), so the flat buffers are
        # re-viewed per call (`noise_view`, `prev_mean_view`); sized for the maximum.
        self.noise_flat = torch.zeros(max_batch * sz.noise_floats_per_env, dtype=torch.float32, device=dev)
        self.prev_mean_flat = torch.zeros(max_batch * d.max_horizon * self.A, dtype=torch.float32, device=dev)
        self.action = torch.zeros(max_batch, self.A, dtype=torch.float32, device=dev)
        # one device block [status word | 3 pad words | metrics [max_batch, 2]] so a call's status and metrics come
        # down as ONE copy; status: the sticky device status word (tdmpc_plan_params.status), nonzero after a plan
        # that failed on the device
        self._ms_dev = torch.zeros(4 + 2 * max_batch, dtype=torch.float32, device=dev)
        self.status = self._ms_dev[:1].view(torch.int32)
        self.metrics = self._ms_dev[4:].view(max_batch, 2)
        # per-call state the kernels read from device memory (ABI 5), so one captured graph serves every value
        # of self.std over std_schedule and every per-env t0 pattern
        self.std_dev = torch.zeros(1, dtype=torch.float32, device=dev)
        self.warm_dev = torch.zeros(max_batch, dtype=torch.int32, device=dev)
        self._std_host = None
        self._warm_host = None
        # per-call inputs, staged on the host and sent up as ONE copy: the observations, numpy's elite-choice
        # uniforms (float64) and the torch generator's {seed, offset} that tdmpc_reference_normals reads when the
        # graph replays; obs_buf / u / gen_state are views of one device block mirrored by one pinned host block
        if cfg.modality == "pixels":
            obs_shape, obs_dt, np_dt = (max_batch, *cfg.obs_shape), torch.uint8, np.uint8
        else:
            obs_shape, obs_dt, np_dt = (max_batch, cfg.obs_shape[0]), torch.float32, np.float32
        ob = int(np.prod(obs_shape)) * (1 if obs_dt == torch.uint8 else 4)
        self._u_off = -(-ob // 8) * 8
        total = self._u_off + 8 * (max_batch + 2)
        pin = dev.type == "cuda"
        self._stage_d = torch.zeros(total, dtype=torch.uint8, device=dev)
        self._stage_h = torch.zeros(total, dtype=torch.uint8, pin_memory=pin)
        uo, ge = self._u_off, self._u_off + 8 * max_batch
        self.obs_buf = self._stage_d[:ob].view(obs_dt).view(obs_shape)
        self.u = self._stage_d[uo:ge].view(torch.float64)
        self.gen_state = self._stage_d[ge:].view(torch.int64)
        hs = self._stage_h.numpy()
        self._h_obs = hs[:ob].view(np_dt).reshape(max_batch, -1)
        self._h_u = hs[uo:ge].view(np.float64)
        self._h_gen = hs[ge:].view(np.uint64)
        self._packed_key = None
        self._packed_model = None
        self._packed_params = []
        self._ptr_arr = None
        self._graphs = {}
        # the metrics come down through pinned memory too (a pageable copy blocks the host)
        self._pin_ms = torch.zeros(4 + 2 * max_batch, dtype=torch.float32, pin_memory=pin)
        self._h2d_done = torch.cuda.Event() if pin else None
        # reference-order draws: "device" = one tdmpc_reference_normals launch per call, "torch" = the
        # reference's own normal_ launches (18 per env at humanoid sizes); equal bitwise
        self.ref_draws = os.environ.get("TDMPC_REF_DRAWS", "device")
        if self.ref_draws not in ("device", "torch"):
            raise ValueError(f"TDMPC_REF_DRAWS must be device or torch, not {self.ref_draws!r}")
        self._grid_cap = None
        self._ref_adv = {}
        # deferred status check of the non-synchronising calls (sync_metrics=False): after each call the sticky status
        # word is copied into pinned slot k % 2 behind an event; call k + 2 waits for that event (queued ahead of call
        # k + 1, so the wait leaves no bubble in the stream) and raises on a nonzero word. check_status() drains both.
        self._st_pin = torch.zeros(2, dtype=torch.int32, pin_memory=pin)
        self._st_ev = [None, None]
        self._st_pending = [False, False]
        self._st_k = 0

    # ------------------------------------------------------------------ weights
    def pack(self, model: TOLD):
        """Pack TOLD parameters when any of them changed (in-place updates bump tensor versions)."""
        pack_told(self, model)

    # ------------------------------------------------------------------ noise
    def noise_view(self, H: int, I: int, B: int):
        S = self.noise_layout(H, I)["total"]
        return self.noise_flat[:B * S].view(B, S)

    def prev_mean_view(self, H: int, B: int):
        return self.prev_mean_flat[:B * H * self.A].view(B, H, self.A)

    def noise_layout(self, H: int, I: int):
        P, N, A, T = self.P, self.N, self.A, self.T
        cem_off = H * P * A
        it = H * N * A + T * A
        return dict(pi=(0, (H, P, A)), cem_off=cem_off, iter=it, term_off=H * N * A,
                    act_off=cem_off + I * it, total=cem_off + I * it + A)

    def draw_reference_noise(self, e: int, H: int, I: int, eval_mode: bool):
        """Fill env e's noise stream from torch's global generator in the reference's draw order
        (SURVEY.md §8a A10): H x normal_([P,A]); per iteration randn(H,N,A), normal_([T,A]); then
        numpy's random_sample() (np.random.choice, tdmpc.py:153); then randn(A) unless eval_mode.
        torch and numpy generators are independent, so the numpy draw is returned separately."""
        self.draw_reference_torch(e, H, I, eval_mode)
        return float(np.random.random_sample())

    def draw_reference_torch(self, e: int, H: int, I: int, eval_mode: bool):
        lay = self.noise_layout(H, I)
        buf = self.noise_view(H, I, e + 1)[e]
        P, N, A, T = self.P, self.N, self.A, self.T
        if P > 0:
            for t in range(H):
                buf[t * P * A:(t + 1) * P * A].view(P, A).normal_()
        for i in range(I):
            o = lay["cem_off"] + i * lay["iter"]
            buf[o:o + H * N * A].view(H, N, A).normal_()
            buf[o + H * N * A:o + H * N * A + T * A].view(T, A).normal_()
        if not eval_mode:
            buf[lay["act_off"]:lay["act_off"] + A].normal_()

    def _gen(self):
        gen = torch.cuda.default_generators[self.device.index or 0]
        if self._grid_cap is None:
            prop = torch.cuda.get_device_properties(self.device)
            per_cu = getattr(prop, "max_threads_per_multi_processor", 2048) // 256
            self._grid_cap = prop.multi_processor_count * per_cu   # ATen calc_execution_policy's grid cap
        return gen

    def _reference_normals(self, B, H, I, eval_mode, seed, offset, gen_state):
        buf = self.noise_view(H, I, B)
        adv = C.c_uint64(0)
        rc = self.L.tdmpc_reference_normals(C.byref(self.dims), C.c_void_p(buf.data_ptr()), B, buf.stride(0), H, I,
                                            int(eval_mode), seed, offset, gen_state, self._grid_cap, C.byref(adv),
                                            C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream))
        _lib.check(rc, "tdmpc_reference_normals")
        key = (B, H, I, bool(eval_mode))
        if self._ref_adv.setdefault(key, adv.value) != adv.value:
            raise RuntimeError(f"reference draws: counter advance {adv.value} != staged {self._ref_adv[key]}")
        return adv.value

    def draw_reference_device(self, B: int, H: int, I: int, eval_mode: bool):
        """The same values as B successive `draw_reference_torch` calls (env 0 first), recomputed by one kernel
        (tdmpc_reference_normals) from the global generator's seed and Philox offset, which then advances
        exactly as the B x 18 normal_ launches would have advanced it. Launched now on the current stream with
        the generator state as arguments (not capturable: see launch_reference_draws)."""
        gen = self._gen()
        off = gen.get_offset()
        gen.set_offset(off + self._reference_normals(B, H, I, eval_mode, gen.initial_seed(), off, None))

    def launch_reference_draws(self, B: int, H: int, I: int, eval_mode: bool):
        """Capturable form: the kernel reads {seed, offset} from `gen_state` when it runs; `stage_reference_state`
        fills it (through the staging copy) before every launch or replay."""
        self._gen()
        self._reference_normals(B, H, I, eval_mode, 0, 0, C.c_void_p(self.gen_state.data_ptr()))

    def stage_reference_state(self, B: int, H: int, I: int, eval_mode: bool):
        """Host side of one call's reference-order draws: the generator's seed and offset into the staging block,
        and the generator advanced past the B x 18 draws the kernel will make."""
        gen = self._gen()
        key = (B, H, I, bool(eval_mode))
        adv = self._ref_adv.get(key)
        if adv is None:
            adv = self._ref_adv[key] = self.reference_advance(B, H, I, eval_mode)
        off = gen.get_offset()
        self._h_gen[0] = gen.initial_seed()
        self._h_gen[1] = off
        gen.set_offset(off + adv)

    def reference_advance(self, B: int, H: int, I: int, eval_mode: bool) -> int:
        """Philox counter advance of B envs' reference draws (ATen calc_execution_policy per normal_ call; the
        same sum tdmpc_reference_normals returns)."""
        self._gen()

        def adv(n):
            grid = min(self._grid_cap, -(-n // 256))
            return ((n - 1) // (256 * grid * 4) + 1) * 4
        P, N, A, T = self.P, self.N, self.A, self.T
        per_env = (H * adv(P * A) if P > 0 else 0) + I * (adv(H * N * A) + adv(T * A)) + (0 if eval_mode else adv(A))
        return B * per_env

    def load_noise(self, e: int, H: int, I: int, eps_pi, eps_cem, eps_term, eps_act):
        """Write an explicit noise stream for env e (parity tests feed the oracle's / the reference's draws)."""
        lay = self.noise_layout(H, I)
        buf = self.noise_view(H, I, e + 1)[e]
        P, N, A, T = self.P, self.N, self.A, self.T
        dev = self.device
        if P > 0:
            buf[:H * P * A].copy_(torch.as_tensor(eps_pi).reshape(-1).to(dev))
        for i in range(I):
            o = lay["cem_off"] + i * lay["iter"]
            buf[o:o + H * N * A].copy_(torch.as_tensor(eps_cem[i]).reshape(-1).to(dev))
            buf[o + H * N * A:o + H * N * A + T * A].copy_(torch.as_tensor(eps_term[i]).reshape(-1).to(dev))
        if eps_act is not None:
            buf[lay["act_off"]:lay["act_off"] + A].copy_(torch.as_tensor(eps_act).reshape(-1).to(dev))

    # ------------------------------------------------------------------ plan
    def params(self, H, I, B, warm, eval_mode, std_floor):
        cfg = self.cfg
        p = _lib.PlanParams()
        p.horizon, p.iterations, p.batch = H, I, B
        p.warm_start, p.eval_mode = int(warm), int(eval_mode)
        p.min_std = float(cfg.min_std)
        p.temperature = float(cfg.temperature)
        p.momentum = float(cfg.momentum)
        p.one_minus_momentum = float(1 - cfg.momentum)
        p.std_floor = float(std_floor)
        p.path = _lib.PATHS[self.path]
        for t, v in enumerate(_discount_pows(cfg.discount, H)):
            p.discount_pow[t] = v
        return p

    def set_call_state(self, std_floor: float, warm):
        """Write self.std and the per-env warm flags into the device scalars the kernels read (stream-ordered
        before the launch or graph replay that follows; skipped when unchanged)."""
        s = float(np.float32(std_floor))
        if s != self._std_host:
            self.std_dev.fill_(s)
            self._std_host = s
        w = tuple(int(bool(x)) for x in warm)
        if w != self._warm_host:
            self.warm_dev[:len(w)].copy_(torch.tensor(w, dtype=torch.int32))
            self._warm_host = w

    def device_state_params(self, prm):
        """Point prm at the device-resident std floor and warm flags (set_call_state)."""
        prm.std_floor_dev = self.std_dev.data_ptr()
        prm.warm_flags = self.warm_dev.data_ptr()
        prm.status = self.status.data_ptr()
        return prm

    def raise_status(self, st: int):
        """Raise for a nonzero device status (and clear it): the plan's outputs are NaN, never return them."""
        if st:
            self.status.zero_()
            raise RuntimeError(f"tdmpc_plan failed on the device (status {st}): {_lib.status_text(st)}. "
                               "Its action is NaN.")

    def check_status(self):
        """Synchronising check of the sticky status word (for callers that plan with sync_metrics=False)."""
        self._st_pending = [False, False]
        self.raise_status(int(self.status.item()))

    def post_status(self):
        """After a non-synchronising call: enqueue the status word's copy into the pinned slot of this call."""
        if not self._st_pin.is_pinned():
            return
        s = self._st_k % 2
        if self._st_ev[s] is None:
            self._st_ev[s] = torch.cuda.Event()
        self._st_pin[s:s + 1].copy_(self.status, non_blocking=True)
        self._st_ev[s].record()
        self._st_pending[s] = True
        self._st_k += 1

    def deferred_status(self):
        """Before a call: raise if the status copied two non-synchronising calls ago is nonzero (the word is sticky,
        so that covers every earlier call too). That copy sits ahead of the previous call in the stream, so waiting
        for it does not drain the queue."""
        s = self._st_k % 2
        if not self._st_pending[s]:
            return
        self._st_ev[s].synchronize()
        self._st_pending[s] = False
        st = int(self._st_pin[s])
        if st:
            self._st_pending = [False, False]
            self.raise_status(st)

    def launch(self, prm, obs_is_u8: bool, trace: dict | None = None):
        L = self.L
        stream = torch.cuda.current_stream(self.device).cuda_stream
        B, H, I, K = prm.batch, prm.horizon, prm.iterations, self.dims.num_elites
        outs = {}
        if trace is not None:
            outs = dict(elite=torch.zeros(B, H, K, self.A, device=self.device),
                        score=torch.zeros(B, K, device=self.device),
                        value=torch.zeros(B, I, self.T, device=self.device),
                        mean=torch.zeros(B, I, H, self.A, device=self.device),
                        std=torch.zeros(B, I, H, self.A, device=self.device))
            trace.update(outs)
        g = outs.get
        rc = L.tdmpc_plan(C.byref(self.dims), C.byref(prm), C.c_void_p(self.packed.data_ptr()),
                          C.c_void_p(self.obs_buf.data_ptr()), int(obs_is_u8), C.c_void_p(self.noise_flat.data_ptr()),
                          C.c_void_p(self.u.data_ptr()), C.c_void_p(self.prev_mean_flat.data_ptr()),
                          C.c_void_p(self.action.data_ptr()), C.c_void_p(self.metrics.data_ptr()),
                          C.c_void_p(_lib.ptr(g("elite"))), C.c_void_p(_lib.ptr(g("score"))),
                          C.c_void_p(_lib.ptr(g("value"))), C.c_void_p(_lib.ptr(g("mean"))),
                          C.c_void_p(_lib.ptr(g("std"))), C.c_void_p(self.workspace.data_ptr()),
                          self.workspace.numel() * 4, C.c_void_p(stream))
        _lib.check(rc, "tdmpc_plan")


    def estimate_value(self, z0, actions, eps_term, H: int, std_floor: float = 0.05):
        """TDMPC.estimate_value (tdmpc.py:83-92) through the C ABI for B envs: z0 [B, L], actions
        [B, H, T, A], eps_term [B, T, A] -> (value [B, T], reward at t=H-1 [B, T], z_H [B, T, L])."""
        B = z0.shape[0]
        prm = self.params(H, 1, B, False, True, std_floor)
        dev = self.device
        z0 = z0.to(dev, torch.float32).contiguous()
        actions = actions.to(dev, torch.float32).contiguous()
        eps_term = eps_term.to(dev, torch.float32).contiguous()
        value = torch.empty(B, self.T, device=dev)
        rlast = torch.empty(B, self.T, device=dev)
        zl = torch.empty(B, self.T, self.dims.latent_dim, device=dev)
        stream = torch.cuda.current_stream(dev).cuda_stream
        rc = self.L.tdmpc_estimate_value(C.byref(self.dims), C.byref(prm), C.c_void_p(self.packed.data_ptr()),
                                         C.c_void_p(z0.data_ptr()), C.c_void_p(actions.data_ptr()),
                                         C.c_void_p(eps_term.data_ptr()), self.T, C.c_void_p(value.data_ptr()),
                                         C.c_void_p(rlast.data_ptr()), C.c_void_p(zl.data_ptr()),
                                         C.c_void_p(self.workspace.data_ptr()), self.workspace.numel() * 4,
                                         C.c_void_p(stream))
        _lib.check(rc, "tdmpc_estimate_value")
        return value, rlast, zl

    def pi_rollout(self, z0, eps_pi, H: int):
        """The policy pre-rollout of TDMPC.plan (tdmpc.py:113-118) through the C ABI for B envs: z0 [B, L],
        eps_pi [B, H, P, A] (TruncatedNormal eps of the H pi calls) -> pi_actions [B, H, P, A]."""
        B = z0.shape[0]
        prm = self.params(H, 1, B, False, True, 0.05)
        dev = self.device
        z0 = z0.to(dev, torch.float32).contiguous()
        eps_pi = eps_pi.to(dev, torch.float32).contiguous()
        out = torch.empty(B, H, self.P, self.A, device=dev)
        stream = torch.cuda.current_stream(dev).cuda_stream
        rc = self.L.tdmpc_pi_rollout(C.byref(self.dims), C.byref(prm), C.c_void_p(self.packed.data_ptr()),
                                     C.c_void_p(z0.data_ptr()), C.c_void_p(eps_pi.data_ptr()),
                                     C.c_void_p(out.data_ptr()), C.c_void_p(self.workspace.data_ptr()),
                                     self.workspace.numel() * 4, C.c_void_p(stream))
        _lib.check(rc, "tdmpc_pi_rollout")
        return out

    def cem_iter(self, z0, pi_actions, eps_cem, eps_term, mean, std, H: int, std_floor: float = 0.05):
        """One CEM iteration of TDMPC.plan (tdmpc.py:127-149) through the C ABI for B envs: z0 [B, L],
        pi_actions [B, H, P, A] (or None when P == 0), eps_cem [B, H, N, A], eps_term [B, T, A]; mean/std
        [B, H, A] are updated in place. Returns (elite_actions [B, H, K, A], score [B, K], value [B, T],
        reward_mean [B])."""
        B = z0.shape[0]
        K = self.dims.num_elites
        prm = self.params(H, 1, B, False, True, std_floor)
        dev = self.device
        z0 = z0.to(dev, torch.float32).contiguous()
        pa = None if pi_actions is None else pi_actions.to(dev, torch.float32).contiguous()
        eps_cem = eps_cem.to(dev, torch.float32).contiguous()
        eps_term = eps_term.to(dev, torch.float32).contiguous()
        for t in (mean, std):
            if not t.is_cuda or t.dtype != torch.float32 or not t.is_contiguous() or t.shape != (B, H, self.A):
                raise ValueError("mean/std must be contiguous fp32 [B, H, A] device tensors")
        elite = torch.empty(B, H, K, self.A, device=dev)
        score = torch.empty(B, K, device=dev)
        value = torch.empty(B, self.T, device=dev)
        rmean = torch.empty(B, device=dev)
        stream = torch.cuda.current_stream(dev).cuda_stream
        vp = C.c_void_p
        rc = self.L.tdmpc_cem_iter(C.byref(self.dims), C.byref(prm), vp(self.packed.data_ptr()), vp(z0.data_ptr()),
                                   vp(_lib.ptr(pa)), vp(eps_cem.data_ptr()), vp(eps_term.data_ptr()),
                                   vp(mean.data_ptr()), vp(std.data_ptr()), vp(elite.data_ptr()),
                                   vp(score.data_ptr()), vp(value.data_ptr()), vp(rmean.data_ptr()),
                                   vp(self.workspace.data_ptr()), self.workspace.numel() * 4, vp(stream))
        _lib.check(rc, "tdmpc_cem_iter")
        return elite, score, value, rmean

    def encode(self, obs):
        """TOLD.h for a batch of observations through the C ABI -> z0 [B, L]."""
        B = obs.shape[0]
        dev = self.device
        is_u8 = obs.dtype == torch.uint8
        obs = obs.to(dev).contiguous()
        z0 = torch.empty(B, self.dims.latent_dim, device=dev)
        stream = torch.cuda.current_stream(dev).cuda_stream
        rc = self.L.tdmpc_encode(C.byref(self.dims), C.c_void_p(self.packed.data_ptr()), C.c_void_p(obs.data_ptr()),
                                 int(is_u8), B, C.c_void_p(self.workspace.data_ptr()), C.c_void_p(z0.data_ptr()),
                                 C.c_void_p(stream))
        _lib.check(rc, "tdmpc_encode")
        return z0


class TDMPC:
    """Drop-in for the reference `TDMPC` planning interface (tdmpc.py:53-163)."""

    def __init__(self, cfg, max_batch: int = 1, rng: str = "reference", graph: bool = True, path: str = "auto"):
        self.cfg = cfg
        self.device = torch.device(cfg.device)
        self.std = linear_schedule(cfg.std_schedule, 0)      # tdmpc.py:59
        self.model = TOLD(cfg).to(self.device)               # tdmpc.py:60
        self.model_target = deepcopy(self.model)             # tdmpc.py:61
        self.model.eval()
        self.model_target.eval()
        if rng not in ("reference", "fused"):
            raise ValueError(rng)
        self.rng = rng
        self.graph = graph
        self.planner = HipPlanner(cfg, max_batch=max_batch, device=self.device, path=path)
        from .learner import RandomShiftsAug
        self.aug = RandomShiftsAug(cfg)                       # tdmpc.py:64
        self._learner = None
        self.optim = self.pi_optim = None                     # created with the learner (tdmpc.py:62-63)
        self._has_prev = np.zeros(max_batch, dtype=bool)
        self._prev_H = np.zeros(max_batch, dtype=np.int64)

    # ------------------------------------------------------------------ reference API
    def state_dict(self):
        return {"model": self.model.state_dict(), "model_target": self.model_target.state_dict()}

    def save(self, fp):
        torch.save(self.state_dict(), fp)

    def load(self, fp):
        load_checkpoint(fp, self.model, self.model_target, self.device)

    # ------------------------------------------------------------------ learner (tdmpc.py:165-245)
    def learner(self, graph: bool = True, warmup: int = 3):
        """The GPU learner (tdmpc_amd/learner.py), created on first use with its Adam optimisers."""
        if self._learner is None:
            from .learner import Learner
            self._learner = Learner(self, graph=graph, warmup=warmup)
        return self._learner

    def update(self, replay_buffer, step, sync_metrics: bool = True, noise=None):
        """tdmpc.py:192-245: one TOLD + policy update from `replay_buffer.sample()`. Returns the reference's
        metrics dict (one host sync), or the metrics tensor [7] when sync_metrics=False. With a
        tdmpc_amd.replay.ReplayBuffer the update is replayed from a HIP graph after a few eager warm-ups."""
        from .learner import METRICS
        self.std = linear_schedule(self.cfg.std_schedule, step)   # tdmpc.py:197
        m = self.learner().update(replay_buffer, step, noise=noise)
        if not sync_metrics:
            return m
        if m.is_cuda:   # one non-blocking copy into pinned memory + a stream sync (no cast kernel, no pageable copy)
            if getattr(self, "_pin_upd", None) is None:
                self._pin_upd = torch.zeros(len(METRICS), dtype=torch.float32, pin_memory=True)
            self._pin_upd.copy_(m, non_blocking=True)
            torch.cuda.current_stream(m.device).synchronize()
            vals = self._pin_upd.tolist()
        else:
            vals = m.tolist()
        out = {k: float(v) for k, v in zip(METRICS, vals)}
        if getattr(replay_buffer, "_full", False) and hasattr(replay_buffer, "check_sample"):
            replay_buffer.check_sample()   # numpy's choice(replace=False) error, raised at this existing sync
        return out

    def update_pi(self, zs):
        """tdmpc.py:165-182."""
        loss = float(self.learner().update_pi(zs))
        # the engine writes the policy weights in place (no tensor version bump): repack before the next plan
        self.planner._packed_key = None
        return loss

    def _td_target(self, next_obs, reward):
        """tdmpc.py:184-190."""
        return self.learner().td_target(next_obs, reward)

    @property
    def _prev_mean(self):
        if not self._has_prev[0]:
            raise AttributeError("_prev_mean")
        return self.planner.prev_mean_view(int(self._prev_H[0]), 1)[0]

    @torch.no_grad()
    def plan(self, obs, eval_mode=False, step=None, t0=True):
        """tdmpc.py:94-163. Returns (action tensor [A] on self.device, {'external_reward_mean', 'current_std'})."""
        cfg = self.cfg
        plan_metrics = {"external_reward_mean": 0.0, "current_std": 0.0}
        if step < cfg.seed_steps and not eval_mode:
            return (torch.empty(cfg.action_dim, dtype=torch.float32, device=self.device).uniform_(-1, 1),
                    plan_metrics)
        a, m = self._plan_envs(np.asarray(obs)[None], eval_mode, step, [t0], clone=True)
        plan_metrics.update(m[0])
        return a[0], plan_metrics

    @torch.no_grad()
    def plan_batch(self, obs, eval_mode=False, step=None, t0=True, sync_metrics=True):
        """Plan B independent environments at once (obs: [B, *obs_shape]); `t0` may be a bool or a per-env
        sequence. Equivalent to B sequential reference `plan` calls on B agents sharing weights, with the
        random draws taken env by env in reference order.

        sync_metrics=False returns (actions, metrics tensor [B, 2]) without a host sync. A device failure (the
        persistent one-env plan giving up at a hand-off) then surfaces late: that call's actions are NaN, and the
        raise comes at the next-but-one call (or at check_status()) -- the NaN actions of the failing call and of
        the call after it may already have been returned by then."""
        cfg = self.cfg
        obs = obs if torch.is_tensor(obs) else np.asarray(obs)
        B = obs.shape[0]
        if step < cfg.seed_steps and not eval_mode:
            a = torch.empty(B, cfg.action_dim, dtype=torch.float32, device=self.device)
            for e in range(B):
                a[e].uniform_(-1, 1)
            if not sync_metrics:
                return a, torch.zeros(B, 2, dtype=torch.float32, device=self.device)
            return a, [{"external_reward_mean": 0.0, "current_std": 0.0} for _ in range(B)]
        t0s = [t0] * B if isinstance(t0, (bool, int, np.bool_)) else list(t0)
        return self._plan_envs(obs, eval_mode, step, t0s, sync_metrics)

    # ------------------------------------------------------------------ internals
    def horizon(self, step):
        return int(min(self.cfg.horizon, linear_schedule(self.cfg.horizon_schedule, step)))

    def _plan_envs(self, obs, eval_mode, step, t0s, sync_metrics=True, trace=None, noise=None, clone=False):
        """noise: optional list (one per env) of objects with eps_pi / eps_cem / eps_term / u / eps_act
        (e.g. oracle NoiseBundles) used instead of drawing. clone: return a copy of the actions (enqueued right
        after the plan, before the metrics sync, so its launch is off the host's critical path)."""
        cfg, pl = self.cfg, self.planner
        B = obs.shape[0]
        if B > pl.max_batch:
            raise ValueError(f"batch {B} > max_batch {pl.max_batch}")
        pl.deferred_status()
        H = self.horizon(step)
        I = int(cfg.iterations)
        warm = []
        for e in range(B):
            w = (not t0s[e]) and bool(self._has_prev[e])
            if w and self._prev_H[e] != H:
                # the reference's `mean[:-1] = self._prev_mean[1:]` raises on a horizon change
                raise RuntimeError(f"shape mismatch: prev_mean horizon {self._prev_H[e]} vs {H}")
            warm.append(w)
        pl.pack(self.model)
        host = not torch.is_tensor(obs) or obs.device.type == "cpu"
        if pl._h2d_done is not None:
            pl._h2d_done.synchronize()   # the previous call's staging copy has drained
        if host:
            pl._h_obs[:B] = np.asarray(obs).reshape(B, -1)
        elif cfg.modality == "pixels":
            pl.obs_buf[:B].copy_(obs.to(self.device, torch.uint8).view(B, *cfg.obs_shape))
        else:
            pl.obs_buf[:B].copy_(obs.to(self.device, torch.float32).view(B, -1))
        obs_u8 = cfg.modality == "pixels"
        pl.set_call_state(self.std, warm)
        if noise is not None:
            for e, nb in enumerate(noise):
                pl.load_noise(e, H, I, nb.eps_pi, nb.eps_cem, nb.eps_term, nb.eps_act)
                pl._h_u[e] = float(nb.u)
        elif self.rng == "reference":
            # np.random.choice's uniform, drawn on the host from numpy's global generator (tdmpc.py:153)
            for e in range(B):
                pl._h_u[e] = np.random.random_sample()
        one_launch = noise is None and self.rng == "reference" and pl.ref_draws == "device"
        if one_launch:
            pl.stage_reference_state(B, H, I, eval_mode)
        # one copy up: observations (host ones), uniforms, generator state. A synchronising call (the drop-in
        # plan()) replays it as the captured graph's first node (a memcpy node from the pinned staging block: one
        # launch fewer on the host's critical path); otherwise it goes ahead of the replay, and an event marks the
        # staging block reusable as soon as the copy is done, so the host stages the next call under this plan
        lo = 0 if host else pl._u_off
        copy_in_graph = self.graph and sync_metrics and noise is None and trace is None
        if not copy_in_graph:
            pl._stage_d[lo:].copy_(pl._stage_h[lo:], non_blocking=True)
            if pl._h2d_done is not None:
                pl._h2d_done.record()

        def device_work():
            if copy_in_graph:
                pl._stage_d[lo:].copy_(pl._stage_h[lo:], non_blocking=True)
            if noise is None:
                if one_launch:
                    pl.launch_reference_draws(B, H, I, eval_mode)
                elif self.rng == "reference":
                    for e in range(B):
                        pl.draw_reference_torch(e, H, I, eval_mode)
                else:
                    pl.noise_view(H, I, B).normal_()
                    pl.u[:B].uniform_()
            pl.launch(pl.device_state_params(pl.params(H, I, B, warm[0], eval_mode, self.std)), obs_u8, trace)

        if self.graph and noise is None and trace is None:
            # (self.std and the warm flags live on the device)
            key = (H, I, B, bool(eval_mode), self.rng, one_launch, copy_in_graph, lo)
            g = pl._graphs.get(key)
            if g is None:
                # No eager warm-up: the library has no lazy initialisation left after pack(), and an eager
                # run would advance the planner state (prev_mean) before the captured replay.
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    device_work()
                pl._graphs[key] = g
            g.replay()
            if copy_in_graph and pl._h2d_done is not None:
                pl._h2d_done.record()
        else:
            device_work()
        self._has_prev[:B] = True
        self._prev_H[:B] = H
        actions = pl.action[:B].clone() if clone else pl.action[:B]
        if not sync_metrics:
            pl.post_status()   # raised by the call after next (deferred_status) or by check_status()
            return actions, pl.metrics[:B]
        pl._st_pending = [False, False]   # (the synchronous read below covers every earlier call: the word is sticky)
        if pl._h2d_done is not None:
            pl._pin_ms[:4 + 2 * B].copy_(pl._ms_dev[:4 + 2 * B], non_blocking=True)   # status + metrics: one copy
            torch.cuda.current_stream(self.device).synchronize()
            m = pl._pin_ms[4:4 + 2 * B].view(B, 2).tolist()
            st = int(pl._pin_ms[:1].view(torch.int32)[0])
        else:
            m = pl.metrics[:B].double().cpu().tolist()
            st = int(pl.status[0])
        pl.raise_status(st)
        return actions, [{"external_reward_mean": float(r), "current_std": float(s)} for r, s in m]
