"""`TdICEM`: drop-in for the reference iCEM agent's planning API on MI355X.

Reference: `TdICemSimMlp` in /root/reference/src/algorithm/tdmpc_icem_similarity_mlp.py:74-265 (driven by
src/train_icem_mlp.py). Same `plan(obs, eval_mode=False, step=None, t0=True) -> (action [A], metrics)`, the same
planner state (`plan_horizon`, `mixture_coef`, `std`, `_prev_mean`, `_elite_actions`) and the same model heads
(TOLD with the DSSM's LayerNorm state encoder when cfg.normalize / norm_type 'ln'). The whole plan -- encoder, the
policy pre-rollout, every iteration's rollout of [sampled | reused elites] candidates, terminal policy + Q,
top-k / softmax refit, elite reuse bookkeeping, the final pick -- is one `tdmpc_plan_icem` call on the chain
kernels (include/tdmpc_hip.h); Python draws the random numbers and lays out their per-env stream.

Differences from TDMPC.plan that the kernels follow: N shrinks per iteration (N_i = max(2K, int(N_{i-1} /
factor_decrease_num))), P_i = int(mixture_coef(step) * N_i) (regularization_schedule), std starts at 0.5, a warm
start keeps mean[-1] = prev_mean[-1], int(fraction_elites_reused * K) elites are re-evaluated (time-shifted from
the previous plan in the first iteration with a fresh coloured tail, the previous iteration's afterwards), the last
iteration's sample 0 is the mean, and the sample noise is white / pink (beta 1) / brown (beta 2.5) thirds.

Randomness (`rng="reference"`): torch's and numpy's global generators in the reference's order; the coloured
thirds come from tdmpc_amd.colored_noise on numpy's global RandomState (the reference's `colorednoise` is
absent and unpinned; 2.x seeds each call from OS entropy, so its stream is not reproducible anyway).
`rng="device"` draws everything on the device in ~8 launches (the stream white in one draw, every coloured third
and reuse tail from one batched spectrum draw per sample length with the irfft as a matmul, the pick's uniform):
same distributions, no host work. `plan(..., noise=IcemNoise)` takes explicit draws (parity tests).
"""
from __future__ import annotations

import ctypes as C
from copy import deepcopy

import numpy as np
import torch

from . import _lib
from .colored_noise import BatchedColoredNoise, _scales as _spectrum
from .config import linear_schedule
from .tdmpc import _discount_pows, pack_told
from .told import TOLD


def _thirds(n):
    q, r = divmod(n, 3)
    return [q, q, q] if r == 0 else ([q, q + 1, q] if r == 1 else [q, q + 1, q + 1])


class TdICEM:
    def __init__(self, cfg, max_batch: int = 1, rng: str = "reference", path: str = "auto"):
        if getattr(cfg, "modality", "state") != "state":
            raise NotImplementedError("iCEM drop-in: state observations (the pixel DSSM encoder is rlpyt's)")
        enc_norm = bool(getattr(cfg, "normalize", False))
        if enc_norm and getattr(cfg, "norm_type", "ln") != "ln":
            raise NotImplementedError("iCEM drop-in: the LayerNorm state encoder (norm_type 'ln')")
        if rng not in ("reference", "device"):
            raise ValueError("rng: 'reference' or 'device'")
        self.rng = rng
        if path not in _lib.PATHS:
            raise ValueError(f"path must be one of {sorted(_lib.PATHS)}")
        self.path = path
        self.cfg = cfg
        self.device = torch.device(cfg.device)
        self.std = linear_schedule(cfg.std_schedule, 0)                       # :84
        self.mixture_coef = linear_schedule(cfg.regularization_schedule, 0)   # :85
        self.model = TOLD(cfg, enc_norm=enc_norm).to(self.device)
        self.model_target = deepcopy(self.model)
        self.model.eval()
        self.model_target.eval()
        self.plan_horizon = 1                                                  # :93
        self.max_batch = max_batch
        A, K, N, H = cfg.action_dim, cfg.num_elites, cfg.num_samples, cfg.horizon
        rs = str(cfg.regularization_schedule)
        mix_max = max(linear_schedule(rs, 0), linear_schedule(rs, 10**12))
        self.P_max = max(1, int(mix_max * N))
        d = _lib.dims_from_cfg(cfg, max_batch=max_batch, enc_norm=enc_norm)
        d.num_pi = self.P_max
        self.dims = d
        self.L = _lib.lib()
        sz = _lib.Sizes()
        _lib.check(self.L.tdmpc_icem_sizes_for(C.byref(d), C.byref(sz)), "tdmpc_icem_sizes_for")
        dev = self.device
        self.packed = torch.zeros(sz.packed_weight_bytes // 4, dtype=torch.float32, device=dev)   # (gaps stay 0)
        self.L.tdmpc_pack_forget(C.c_void_p(self.packed.data_ptr()))   # (the address may be a freed buffer's)
        self.workspace = torch.empty(sz.workspace_bytes // 4, dtype=torch.float32, device=dev)
        self.E_max = int(cfg.fraction_elites_reused * K)
        T_max = N + self.E_max + self.P_max
        # per-env stream upper bound: pre-rollout + per iteration (samples + terminal) + reuse tail + action
        self.stream_max = H * self.P_max * A + cfg.iterations * (H * N * A + T_max * A) + H * self.E_max * A + A
        self.noise = torch.zeros(max_batch * self.stream_max, dtype=torch.float32, device=dev)
        self.u = torch.zeros(max_batch, dtype=torch.float64, device=dev)
        self.prev_mean_flat = torch.zeros(max_batch * H * A, dtype=torch.float32, device=dev)
        self.elites = torch.zeros(max_batch, H, K, A, dtype=torch.float32, device=dev)
        self.action = torch.zeros(max_batch, A, dtype=torch.float32, device=dev)
        # [status word | 3 pad words | metrics [max_batch, 2]]: a call's sticky device status (tdmpc_icem_params.status:
        # TDMPC_STATUS_PACK_STALE) comes down with its metrics in one copy
        self._ms_dev = torch.zeros(4 + 2 * max_batch, dtype=torch.float32, device=dev)
        self.status = self._ms_dev[:1].view(torch.int32)
        self.metrics = self._ms_dev[4:].view(max_batch, 2)
        self.obs_buf = torch.zeros(max_batch, cfg.obs_shape[0], dtype=torch.float32, device=dev)
        col_max = cfg.iterations * H * N * A + H * self.E_max * A   # coloured floats of one env and call
        self._stage = torch.empty(col_max, dtype=torch.float32, device=dev)
        self._pinned = torch.empty(col_max, dtype=torch.float32, pin_memory=dev.type == "cuda")
        self._h2d_done = None
        self._dev_plans = {}
        self._packed_key = self._packed_model = None
        self._packed_params = []
        self._has_prev = False
        self._has_elites = False
        self._elite_H = 0

    # ------------------------------------------------------------------ reference state
    @property
    def _prev_mean(self):
        if not self._has_prev:
            raise AttributeError("_prev_mean")
        return self.prev_mean_flat[:self.plan_horizon * self.cfg.action_dim].view(self.plan_horizon, -1)

    @property
    def _elite_actions(self):
        if not self._has_elites:
            raise AttributeError("_elite_actions")
        return self.elites[0, :self._elite_H]

    # ------------------------------------------------------------------ plan
    def counts(self, mixture, has_elites):
        """(N_i, P_i, E_i) per iteration (tdmpc_icem_similarity_mlp.py:201-210)."""
        cfg, out, n = self.cfg, [], self.cfg.num_samples
        for i in range(cfg.iterations):
            if i > 0:
                n = max(2 * cfg.num_elites, int(n / cfg.factor_decrease_num))
            p = int(mixture * n)
            e = self.E_max if (cfg.fraction_elites_reused > 0 and (has_elites or i > 0)) else 0
            out.append((n, p, e))
        return out

    def _layout(self, H, cts, reuse):
        """Per-env noise stream offsets (floats)."""
        A = self.cfg.action_dim
        off = {"pi": 0}
        o = H * cts[0][1] * A
        off["samp"], off["term"] = [], []
        off["reuse"] = 0
        for i, (n, p, e) in enumerate(cts):
            off["samp"].append(o)
            o += H * n * A
            if i == 0 and reuse:
                off["reuse"] = o
                o += H * e * A
            off["term"].append(o)
            o += (n + e + p) * A
        off["act"] = o
        off["total"] = o + A
        return off

    def _colored_specs(self, H, cts, reuse):
        """The coloured-noise draws of one plan call in the reference's order: (beta, n, length, kind, i)."""
        cfg, out = self.cfg, []
        for i, (n, p, ne) in enumerate(cts):
            n0, n1, n2 = _thirds(n)
            out += [(1.0, n1, cfg.horizon, "samp", i), (2.5, n2, cfg.horizon, "samp", i)]
            if i == 0 and reuse and cfg.noise_beta > 0:
                out.append((cfg.noise_beta, ne, H, "reuse", i))
        return out

    def _colored_host(self, specs, H):
        """All of a call's coloured noise on the host -> float32 [sum_k H * n_k * A] ([H][n][A] per draw).
        Numbers identical to consecutive powerlaw_psd_gaussian calls on numpy's global RandomState: one
        standard_normal draw of the whole call (the legacy generator's stream does not depend on how it is
        chunked; normal(scale=s) is s * standard_normal), one irfft per spectrum length (row-independent)."""
        A = self.cfg.action_dim
        sizes = [n * A * ((L // 2) + 1) for _, n, L, _, _ in specs]
        z = np.random.standard_normal(2 * sum(sizes))
        parts, o = [], 0
        for (beta, n, L, _, _), sz in zip(specs, sizes):
            sc, sigma = _spectrum(beta, L)
            sr = z[o:o + sz].reshape(n, A, -1) * sc
            si = z[o + sz:o + 2 * sz].reshape(n, A, -1) * sc
            o += 2 * sz
            if not L % 2:
                si[..., -1] = 0
                sr[..., -1] *= np.sqrt(2)
            si[..., 0] = 0
            sr[..., 0] *= np.sqrt(2)
            parts.append((sr + 1j * si, sigma))
        out = []
        for L in sorted({s[2] for s in specs}):
            idx = [k for k, s in enumerate(specs) if s[2] == L]
            y = np.fft.irfft(np.concatenate([parts[k][0] for k in idx]), n=L, axis=-1)
            r = 0
            for k in idx:
                n = specs[k][1]
                out.append((k, (y[r:r + n] / parts[k][1]).astype(np.float32)[:, :, :H].transpose(2, 0, 1)))
                r += n
        out.sort(key=lambda t: t[0])
        return np.concatenate([a.reshape(-1) for _, a in out]) if out else np.zeros(0, np.float32)

    def _device_plan(self, H, cts, off, reuse, B=1):
        """rng 'device': per sample length, a BatchedColoredNoise over that length's coloured specs of B envs and
        the stream positions [R, H] its rows land on (samp thirds [H][n][A] at their column offset, reuse tail;
        env e's stream at e * off['total'])."""
        key = (H, tuple(cts), reuse, B)
        plan = self._dev_plans.get(key)
        if plan is not None:
            return plan
        A = self.cfg.action_dim
        groups = {}
        for beta, n, L, kind, i in self._colored_specs(H, cts, reuse):
            nt = cts[i][0]
            n0, n1, _ = _thirds(nt)
            if kind == "samp":
                base, rows, c0 = off["samp"][i], nt, (n0 if beta == 1.0 else n0 + n1)
            else:
                base, rows, c0 = off["reuse"], n, 0
            t = np.arange(H)[None, None, :]
            r = np.arange(n)[:, None, None]
            a = np.arange(A)[None, :, None]
            pos = base + t * rows * A + (c0 + r) * A + a                   # [n, A, H]
            g = groups.setdefault(L, ([], []))
            for e in range(B):
                g[0].append((beta, n))
                g[1].append(pos.reshape(n * A, H) + e * off["total"])
        plan = []
        for L, (sp, pos) in sorted(groups.items()):
            plan.append((BatchedColoredNoise(sp, A, L, H, self.device),
                         torch.as_tensor(np.concatenate(pos), dtype=torch.int64, device=self.device)))
        if len(self._dev_plans) > 16:
            self._dev_plans.clear()
        self._dev_plans[key] = plan
        return plan

    def _draw_device(self, B, H, cts, off, reuse):
        """rng 'device' for B envs: the B streams white in one draw, every coloured third / reuse tail overwritten
        from one batched spectrum draw per sample length, the picks' uniforms: ~8 launches per call."""
        self.noise[:B * off["total"]].normal_()
        for gen, pos in self._device_plan(H, cts, off, reuse, B):
            self.noise[pos] = gen.draw()
        self.u[:B].uniform_()

    def _draw(self, e, H, cts, off, reuse, eval_mode):
        """Env e's stream in the reference's draw order on torch's (device) and numpy's global generators.
        The two generators are independent, so the numpy draws (coloured thirds, reused-elite tail, the pick's
        uniform) run first on the host and travel in ONE pinned async copy; the torch draws follow in order."""
        cfg, A = self.cfg, self.cfg.action_dim
        S = off["total"]
        buf = self.noise[e * S:(e + 1) * S]
        dev = self.device
        specs = self._colored_specs(H, cts, reuse)
        host = self._colored_host(specs, H)
        u = float(np.random.random_sample())
        if self._h2d_done is not None:
            self._h2d_done.synchronize()   # the previous call's copy has left the pinned buffer
        stage = self._pinned[:host.size]
        stage.numpy()[:] = host
        dst = self._stage[:host.size]
        dst.copy_(stage, non_blocking=True)
        self._h2d_done = torch.cuda.Event()
        self._h2d_done.record()
        col, o = [], 0
        for b, n, L, _, _ in specs:
            col.append(dst[o:o + H * n * A].view(H, n, A))
            o += H * n * A
        P0 = cts[0][1]
        for t in range(H):
            buf[t * P0 * A:(t + 1) * P0 * A].view(P0, A).normal_()
        k = 0
        for i, (n, p, ne) in enumerate(cts):
            n0, n1, n2 = _thirds(n)
            samp = buf[off["samp"][i]:off["samp"][i] + H * n * A].view(H, n, A)
            samp[:, :n0].copy_(torch.randn(H, n0, A, device=dev))
            samp[:, n0:n0 + n1].copy_(col[k])
            samp[:, n0 + n1:].copy_(col[k + 1])
            k += 2
            if i == 0 and reuse:
                r = buf[off["reuse"]:off["reuse"] + H * ne * A].view(H, ne, A)
                if cfg.noise_beta > 0:
                    r.copy_(col[k])
                    k += 1
                else:
                    r.copy_(torch.randn(H, ne, A, device=dev))
            buf[off["term"][i]:off["term"][i] + (n + ne + p) * A].view(n + ne + p, A).normal_()
        if not eval_mode:
            buf[off["act"]:off["act"] + A].normal_()
        return u

    def _load(self, e, H, cts, off, reuse, nz):
        """Write explicit draws (oracle IcemNoise) into env e's stream."""
        A = self.cfg.action_dim
        S = off["total"]
        buf = self.noise[e * S:(e + 1) * S]
        dev = self.device
        P0 = cts[0][1]
        buf[:H * P0 * A].copy_(nz.eps_pi.reshape(-1).to(dev))
        for i, (n, p, ne) in enumerate(cts):
            buf[off["samp"][i]:off["samp"][i] + H * n * A].copy_(nz.samp[i].reshape(-1).to(dev))
            if i == 0 and reuse:
                buf[off["reuse"]:off["reuse"] + H * ne * A].copy_(nz.reuse.reshape(-1).to(dev))
            buf[off["term"][i]:off["term"][i] + (n + ne + p) * A].copy_(nz.term[i].reshape(-1).to(dev))
        if nz.eps_act is not None:
            buf[off["act"]:off["act"] + A].copy_(nz.eps_act.to(dev))
        return float(nz.u)

    @torch.no_grad()
    def plan(self, obs, eval_mode=False, step=None, t0=True, noise=None, trace=None):
        """tdmpc_icem_similarity_mlp.py:160-265 -> (action tensor [A], metrics dict)."""
        cfg = self.cfg
        metrics = {"external_reward_mean": 0.0, "current_std": 0.0}
        if step < cfg.seed_steps and not eval_mode:
            return torch.empty(cfg.action_dim, dtype=torch.float32, device=self.device).uniform_(-1, 1), metrics
        obs = torch.as_tensor(np.asarray(obs), dtype=torch.float32).view(1, -1)
        a, m = self._plan_envs(obs, eval_mode, step, t0, [noise] if noise is not None else None, trace)
        ms = self._ms_dev[:6].cpu()
        self._raise_status(int(ms[:1].view(torch.int32)))
        m = ms[4:6].double().numpy()
        metrics.update({"external_reward_mean": float(m[0]), "current_std": float(m[1])})
        return a[0].clone(), metrics

    @torch.no_grad()
    def plan_batch(self, obs, eval_mode=False, step=None, t0=True, sync_metrics=True):
        """B independent iCEM plans in one call (vectorised envs, all at the same step / t0): obs [B, obs_dim] ->
        (actions [B, A], metrics). Env e's result equals a single-env plan() on its own noise stream
        (tests/test_icem.py::test_gpu_icem_batched_equals_single). Seed steps are not batched."""
        if step < self.cfg.seed_steps and not eval_mode:
            raise ValueError("plan_batch: seed steps draw uniform actions; call plan() per env")
        obs = torch.as_tensor(obs, dtype=torch.float32)
        a, m = self._plan_envs(obs.view(obs.shape[0], -1), eval_mode, step, t0, None, None)
        if not sync_metrics:
            return a, m
        B = obs.shape[0]
        ms = self._ms_dev[:4 + 2 * B].cpu()
        self._raise_status(int(ms[:1].view(torch.int32)))
        return a, [{"external_reward_mean": float(r), "current_std": float(sd)}
                   for r, sd in ms[4:].view(B, 2).double().numpy()]

    def check_status(self):
        """Synchronising check of the sticky device status word (for plan_batch(sync_metrics=False) callers)."""
        self._raise_status(int(self.status.item()))

    def _raise_status(self, st: int):
        if st:
            self.status.zero_()
            raise RuntimeError(f"tdmpc_plan_icem failed on the device (status {st}): "
                               + _lib.status_text(st) + "; its actions are NaN")

    def _plan_envs(self, obs, eval_mode, step, t0, noise, trace):
        cfg = self.cfg
        B = obs.shape[0]
        if B > self.max_batch:
            raise ValueError(f"batch {B} > max_batch {self.max_batch}")
        horizon = int(min(cfg.horizon, linear_schedule(cfg.horizon_schedule, step)))
        extend = False
        if horizon != self.plan_horizon and t0:
            self.plan_horizon, extend = horizon, True
        H = self.plan_horizon
        self.mixture_coef = linear_schedule(cfg.regularization_schedule, step)
        cts = self.counts(self.mixture_coef, self._has_elites)
        if cts[0][1] <= 0 or any(p <= 0 for _, p, _ in cts):
            raise AssertionError("num_pi_trajs > 0")   # the reference asserts this (:187, :205)
        if cts[0][1] > self.P_max:
            raise ValueError("mixture_coef above the schedule's maximum")
        if cfg.iterations > 1 and cts[1][2] > 0 and not cfg.keep_previous_elites:
            # the reference would then re-use the first iteration's `reused_actions` (a stale loop variable)
            raise NotImplementedError("fraction_elites_reused > 0 needs keep_previous_elites")
        reuse = self._has_elites and cfg.shift_elites_over_time and cts[0][2] > 0
        if reuse and self._elite_H not in (H, H - 1):
            raise RuntimeError("elite horizon mismatch")   # the reference's torch.cat would fail here
        off = self._layout(H, cts, reuse)
        pack_told(self, self.model)
        self.obs_buf[:B].copy_(obs.to(self.device))
        if noise is not None:
            for e, nz in enumerate(noise):
                self.u[e:e + 1].fill_(self._load(e, H, cts, off, reuse, nz))
        elif self.rng == "device":
            self._draw_device(B, H, cts, off, reuse)
        else:
            us = [self._draw(e, H, cts, off, reuse, eval_mode) for e in range(B)]
            self.u[:B].copy_(torch.tensor(us, dtype=torch.float64))
        p = _lib.IcemParams()
        p.horizon, p.iterations, p.batch = H, cfg.iterations, B
        p.warm_start = int((not t0) and self._has_prev)
        p.eval_mode = int(eval_mode)
        p.has_elites = int(reuse)
        p.elite_horizon = self._elite_H if reuse else H
        p.n_pi0 = cts[0][1]
        p.path = _lib.PATHS[self.path]
        for i, (n, pp, e) in enumerate(cts):
            p.n_samples[i], p.n_pi[i], p.n_elite[i] = n, pp, e
            p.samp_off[i], p.term_off[i] = off["samp"][i], off["term"][i]
        p.reuse_off, p.pi_off, p.act_off, p.env_stride = off["reuse"], 0, off["act"], off["total"]
        p.min_std, p.temperature, p.momentum = cfg.min_std, cfg.temperature, cfg.momentum
        p.one_minus_momentum = float(1 - cfg.momentum)
        p.std_floor, p.init_std = float(self.std), 0.5
        for t, v in enumerate(_discount_pows(cfg.discount, H)):
            p.discount_pow[t] = v
        p.status = self.status.data_ptr()
        dev = self.device
        value_out = mean_out = std_out = None
        if trace is not None:
            Tw = cfg.num_samples + cfg.num_elites + self.P_max
            value_out = torch.zeros(B, cfg.iterations, Tw, device=dev)
            mean_out = torch.zeros(B, cfg.iterations, H, cfg.action_dim, device=dev)
            std_out = torch.zeros_like(mean_out)
        stream = torch.cuda.current_stream(dev).cuda_stream
        rc = self.L.tdmpc_plan_icem(
            C.byref(self.dims), C.byref(p), C.c_void_p(self.packed.data_ptr()), C.c_void_p(self.obs_buf.data_ptr()),
            0, C.c_void_p(self.noise.data_ptr()), C.c_void_p(self.u.data_ptr()),
            C.c_void_p(self.prev_mean_flat.data_ptr()), C.c_void_p(self.elites.data_ptr()),
            C.c_void_p(self.action.data_ptr()), C.c_void_p(self.metrics.data_ptr()),
            C.c_void_p(_lib.ptr(value_out)), C.c_void_p(_lib.ptr(mean_out)), C.c_void_p(_lib.ptr(std_out)),
            C.c_void_p(self.workspace.data_ptr()), self.workspace.numel() * 4, C.c_void_p(stream))
        _lib.check(rc, "tdmpc_plan_icem")
        if trace is not None:
            trace.update(value=[value_out[0, i, :n + e + pp] for i, (n, pp, e) in enumerate(cts)],
                         mean=mean_out[0], std=std_out[0], counts=cts,
                         value_all=value_out, mean_all=mean_out, std_all=std_out)   # (every env: [B, I, ...])
        self._has_prev = True
        self._has_elites = True
        self._elite_H = H
        return self.action[:B], self.metrics[:B]
