"""The TD-MPC learner on the GPU: `TDMPC.update / update_pi / _td_target`.

Reference: /root/reference/src/algorithm/tdmpc.py:165-245 (+ helper.py:19-26 mse / l1, 48-52 ema, 71-96
TruncatedNormal, 250-283 RandomShiftsAug). The math is the reference's (the oracle restatement
oracle/learner_ref.py is pinned bit-exact to the reference on the CPU; tests/test_learner.py holds this
against it within the fp32 tolerance stated there), including the reference's quirks: the IS-weighted mean
is the mean over the [B, B] broadcast of total_loss [B, 1] against weights [B] (computed as the equal
mean(total_loss) * mean(weights)); the TD target uses the ONLINE encoder and policy
with the target Q; the policy update re-samples TruncatedNormal noise.

What is MI355X-specific is how it runs. A reference update is ~1,500 small kernel launches issued one by one
from Python with seven host syncs (`.item()` metrics, the host-side replay choice). Here only the latent
dynamics chain z_{t+1} = d(z_t, a_t) stays a loop over the horizon; everything off that chain is batched into
one pass over H*B rows (the TD targets with their encoders, policy and target Q; the Q heads and the reward
head on (z_t, a_t); the losses as rho-weighted sums over the horizon axis) and the policy update is one pass
over (H+1)*B rows -- per row the same math, far fewer and wider launches (the horizon steps' TruncatedNormal
draws come from one [H*B, A] call instead of H calls of [B, A]; with explicit noise they are the same
numbers). Then, after `warmup`
eager updates (which also create Adam's state), one whole update -- the device replay sample
(tdmpc_amd.replay), encoder / dynamics / reward / Q forward over the horizon, the TD targets, backward,
grad-norm clipping, Adam (capturable, foreach), the priority write-back, the policy update -- is captured
into ONE HIP graph per (buffer fill, EMA) shape and replayed: no Python in the loop, no host sync, the RNG
(philox, graph-safe) advancing exactly as the eager calls would. The EMA of the target is one foreach lerp.
"""
from __future__ import annotations

import ctypes as C
import os

import torch
import torch.nn.functional as F

METRICS = ("consistency_loss", "reward_loss", "value_loss", "pi_loss", "total_loss", "weighted_loss", "grad_norm")



def clip_grad_norm_19(params, max_norm):
    """clip_grad_norm_(params, max_norm, error_if_nonfinite=False) as the reference's pinned torch 1.9 runs it
    (/root/reference/environment.yaml:6; tdmpc.py:178, 228): `if clip_coef < 1: grad.mul_(clip_coef)`, so a NaN norm
    scales nothing (torch >= 1.13 clamps and poisons every gradient). Written without a host sync (capturable): the
    coefficient is where(coef < 1, coef, 1), and multiplying by exactly 1 leaves a gradient bitwise unchanged."""
    grads = [p.grad for p in params if p.grad is not None]
    total = torch.linalg.vector_norm(torch.stack(torch._foreach_norm(grads, 2.0)), 2.0)
    coef = max_norm / (total + 1e-6)
    coef = torch.where(coef < 1, coef, torch.ones_like(coef))
    torch._foreach_mul_(grads, coef)
    return total

class RandomShiftsAug(torch.nn.Module):
    """helper.py:250-283: random-shift augmentation of pixel observations (identity for state). The shifts are
    drawn as the reference draws them per call (one torch.randint of [n, 1, 1, 2] on the input's device, so one
    call advances the generator identically; the engine's update makes its calls in another order than the
    reference's, learner_engine.update); the shift itself runs as one HIP gather kernel (tdmpc_random_shift,
    include/tdmpc_learner.h): the reference's pad + grid_sample lands on integer pixel centres, so it is a
    clamped-index copy (tests/test_learner.py holds it to the reference's outputs)."""

    def __init__(self, cfg):
        super().__init__()
        self.pad = int(cfg.img_size / 21) if cfg.modality == "pixels" else None

    def forward(self, x, shift=None, div=0.0):
        """shift: optional explicit [n, 2] (x, y) integer shifts instead of the draw (parity tests). div > 0: the
        frames come back divided by div (NormalizeImg's x / 255 folded into the gather; the learner engine)."""
        if not self.pad:
            return x
        from . import _lib
        shape = x.shape
        if x.dim() == 5:
            x = x.reshape(shape[0] * shape[1], *shape[2:])   # the same shift for a trajectory's frames
        n, c, hh, ww = x.shape
        if hh != ww or not x.is_cuda or x.dtype != torch.float32:
            raise ValueError("RandomShiftsAug: square float32 frames on the GPU")
        if shift is None:
            shift = torch.randint(0, 2 * self.pad + 1, size=(n, 1, 1, 2), device=x.device, dtype=x.dtype)
        else:
            shift = torch.as_tensor(shift, dtype=torch.float32).to(x.device).reshape(n, 1, 1, 2)
        x = x.contiguous()
        out = torch.empty_like(x)
        L = _lib.lib()
        _lib.check(L.tdmpc_random_shift_scaled(C.c_void_p(x.data_ptr()), C.c_void_p(shift.data_ptr()), n, c, hh, ww,
                                               self.pad, float(div), C.c_void_p(out.data_ptr()),
                                               C.c_void_p(torch.cuda.current_stream(x.device).cuda_stream)),
                   "tdmpc_random_shift")
        return out.reshape(shape)


class _FusedLoss(torch.autograd.Function):
    """TDMPC.update's loss composition (tdmpc.py:209-224) and its backward as HIP kernels (include/tdmpc_learner.h):
    forward(zp, nz, q1, q2, rp, rw, td, w, rho) -> (scal [6], rows [5, B]); scal = (mean consistency, mean reward,
    mean value, mean total, weighted, mean w), rows = (consistency, reward, value, clamped priority, total) per
    batch row. Only scal[4] (the weighted loss) carries a gradient."""

    @staticmethod
    def forward(ctx, zp, nz, q1, q2, rp, rw, td, w, rho, coefs):
        from . import _lib
        H, B, L = zp.shape
        ins = [t.detach().contiguous() for t in (zp, nz, q1, q2, rp, rw, td, w, rho)]
        args = _lib.LossArgs(*[t.data_ptr() for t in ins], H, B, L, *coefs)
        rows = torch.empty(5, B, dtype=torch.float32, device=zp.device)
        scal = torch.empty(6, dtype=torch.float32, device=zp.device)
        stream = torch.cuda.current_stream(zp.device).cuda_stream
        _lib.check(_lib.lib().tdmpc_loss_forward(C.byref(args), C.c_void_p(rows.data_ptr()),
                                                  C.c_void_p(scal.data_ptr()), C.c_void_p(stream)),
                   "tdmpc_loss_forward")
        ctx.save_for_backward(*ins, rows, scal)
        ctx.coefs = coefs
        ctx.mark_non_differentiable(rows)
        return scal, rows

    @staticmethod
    def backward(ctx, g_scal, g_rows):
        from . import _lib
        zp, nz, q1, q2, rp, rw, td, w, rho, rows, scal = ctx.saved_tensors
        H, B, L = zp.shape
        args = _lib.LossArgs(*[t.data_ptr() for t in (zp, nz, q1, q2, rp, rw, td, w, rho)], H, B, L, *ctx.coefs)
        g = g_scal.contiguous()
        need = ctx.needs_input_grad
        dzp = torch.empty_like(zp) if need[0] else None
        dq1 = torch.empty_like(q1) if need[2] else None
        dq2 = torch.empty_like(q2) if need[3] else None
        drp = torch.empty_like(rp) if need[4] else None
        stream = torch.cuda.current_stream(zp.device).cuda_stream
        _lib.check(_lib.lib().tdmpc_loss_backward(
            C.byref(args), C.c_void_p(rows.data_ptr()), C.c_void_p(scal.data_ptr()), C.c_void_p(g.data_ptr() + 16),
            C.c_void_p(_lib.ptr(dzp)), C.c_void_p(_lib.ptr(dq1)), C.c_void_p(_lib.ptr(dq2)),
            C.c_void_p(_lib.ptr(drp)), C.c_void_p(stream)), "tdmpc_loss_backward")
        return dzp, None, dq1, dq2, drp, None, None, None, None, None


def _mse(pred, target):
    return F.mse_loss(pred, target, reduction="none")


def _l1(pred, target):
    return F.l1_loss(pred, target, reduction="none")


class Learner:
    """Owns the optimisers and (in graph mode) the captured update graphs of one TDMPC agent."""

    def __init__(self, agent, graph: bool = True, warmup: int = 3):
        self.agent = agent
        self.cfg = agent.cfg
        self.graph = graph
        self.warmup = warmup
        model = agent.model
        self.params = list(model.parameters())
        self.pi_params = list(model._pi.parameters())
        self.target_params = list(agent.model_target.parameters())
        from . import learner_engine
        self.engine = None
        # (TDMPC_LEARNER_ENGINE=0: the autograd path with PyTorch's kernels, the bench's comparison leg)
        if (str(agent.device).startswith("cuda") and learner_engine.supported(self.cfg) and
                os.environ.get("TDMPC_LEARNER_ENGINE", "1") != "0"):
            # explicit forward / backward kernels over flat parameters (tdmpc_amd/learner_engine.py); its two
            # Adam states stand in for the reference's optimisers
            self.engine = learner_engine.Engine(agent)
            agent.optim, agent.pi_optim = self.engine.opt_main, self.engine.opt_pi
        else:
            # tdmpc.py:62-63 (Adam over all TOLD parameters; the policy's own Adam, both at cfg.lr)
            agent.optim = torch.optim.Adam(self.params, lr=self.cfg.lr, capturable=graph, fused=True)
            agent.pi_optim = torch.optim.Adam(self.pi_params, lr=self.cfg.lr, capturable=graph, fused=True)
        self.calls = 0
        self._graphs = {}
        self._live_pack = False   # the last update repacked the planner's weights itself (repack_live)
        H = self.cfg.horizon
        # rho^t, t = 0..H, as float32 like the reference's Python-float scalar multiplies (tdmpc.py:212, 179)
        self._rho = torch.tensor([self.cfg.rho ** t for t in range(H + 1)], dtype=torch.float32,
                                 device=agent.device).view(H + 1, 1, 1)

    # ------------------------------------------------------------------ reference math
    @torch.no_grad()
    def td_target(self, next_obs, reward, eps=None):
        """tdmpc.py:184-190."""
        a, cfg = self.agent, self.cfg
        next_z = a.model.h(next_obs)
        return reward + cfg.discount * torch.min(*a.model_target.Q(next_z, a.model.pi(next_z, cfg.min_std, eps=eps)))

    def update_pi(self, zs, eps=None):
        """tdmpc.py:165-182 -> pi_loss (tensor): the H+1 latents in one pass, sum_t -mean(min Q_t) rho^t."""
        a, cfg = self.agent, self.cfg
        if self.engine is not None:
            return self.engine.update_pi(zs, eps)
        a.pi_optim.zero_grad(set_to_none=True)
        a.model.track_q_grad(False)
        n = len(zs)
        Z = torch.cat(zs)
        act = a.model.pi(Z, cfg.min_std, eps=None if eps is None else torch.cat(list(eps[:n])))
        q = torch.min(*a.model.Q(Z, act)).view(n, -1)
        pi_loss = (-q.mean(dim=1) * self._rho[:n].view(n)).sum()
        pi_loss.backward()
        clip_grad_norm_19(self.pi_params, cfg.grad_clip_norm)
        a.pi_optim.step()
        a.model.track_q_grad(True)
        return pi_loss.detach()

    def step(self, buffer, noise=None):
        """One TDMPC.update without the EMA (tdmpc.py:192-241) -> metrics tensor [7] (METRICS order).
        noise: optional list of 2H+1 [B, A] TruncatedNormal draws (H for the TD targets, H+1 for update_pi)."""
        if self.engine is not None:
            m = self.engine.update(buffer, noise)
            from .tdmpc import repack_live
            # the planner's packed weights straight from the engine's flat buffer (one fused launch, inside the
            # captured graph when this step is captured); without a live pack the next plan() repacks
            self._live_pack = repack_live(self.agent.planner, self.agent.model)
            return m
        a, cfg = self.agent, self.cfg
        m = a.model
        H = cfg.horizon
        obs, next_obses, action, reward, idxs, weights = buffer.sample()
        B = obs.shape[0]
        a.optim.zero_grad(set_to_none=True)
        act, rew = action[:H], reward[:H]                                   # [H, B, A], [H, B, 1]
        with torch.no_grad():   # targets of every horizon step at once (tdmpc.py:206-208, 184-190)
            next_obs = a.aug(next_obses[:H].reshape(H * B, *next_obses.shape[2:]))
            next_z = a.model_target.h(next_obs).view(H, B, -1)
            td_target = self.td_target(next_obs, rew.reshape(H * B, 1),
                                       eps=None if noise is None else torch.cat(list(noise[:H]))).view(H, B, 1)
        # the latent dynamics chain (tdmpc.py:203-205): the only sequential part
        z = m.h(a.aug(obs))
        zs = [z]
        for t in range(H):
            z = m._dynamics(torch.cat([z, act[t]], dim=-1))
            zs.append(z)
        x = torch.cat([torch.stack(zs[:H]), act], dim=-1).view(H * B, -1)  # (z_t, a_t), t < H
        Q1, Q2 = m._Q1(x).view(H, B, 1), m._Q2(x).view(H, B, 1)
        reward_pred = m._reward(x).view(H, B, 1)
        rho = self._rho[:H]
        if obs.is_cuda:
            # the loss composition and its backward as three HIP launches (_FusedLoss) instead of ~60 ATen ones
            scal, rows = _FusedLoss.apply(torch.stack(zs[1:]), next_z, Q1.view(H, B), Q2.view(H, B),
                                          reward_pred.view(H, B), rew.reshape(H, B), td_target.view(H, B),
                                          weights, rho.view(H),
                                          (float(cfg.consistency_coef), float(cfg.reward_coef),
                                           float(cfg.value_coef)))
            means = (scal[0], scal[1], scal[2], scal[3])
            weighted_loss = scal[4]
            prio = rows[3].view(B, 1)   # [B, 1] like the reference's priority_loss
        else:
            consistency_loss = (rho * torch.mean(_mse(torch.stack(zs[1:]), next_z), dim=2, keepdim=True)).sum(0)
            reward_loss = (rho * _mse(reward_pred, rew)).sum(0)
            value_loss = (rho * (_mse(Q1, td_target) + _mse(Q2, td_target))).sum(0)
            priority_loss = (rho * (_l1(Q1, td_target) + _l1(Q2, td_target))).sum(0)
            total_loss = cfg.consistency_coef * consistency_loss.clamp(max=1e4) + \
                cfg.reward_coef * reward_loss.clamp(max=1e4) + \
                cfg.value_coef * value_loss.clamp(max=1e4)
            # the reference's (total_loss [B, 1] * weights [B]).mean() is a mean over the [B, B] broadcast, i.e.
            # mean(total_loss) * mean(weights): computed in that factored form (no B x B tensor, same gradient)
            weighted_loss = total_loss.mean() * weights.mean()
            means = (consistency_loss.mean(), reward_loss.mean(), value_loss.mean(), total_loss.mean())
            prio = priority_loss.clamp(max=1e4).detach()
        zs = [zz.detach() for zz in zs]
        weighted_loss.register_hook(lambda grad: grad * (1 / H))
        weighted_loss.backward()
        grad_norm = clip_grad_norm_19(self.params, cfg.grad_clip_norm)
        a.optim.step()
        buffer.update_priorities(idxs, prio)
        pi_loss = self.update_pi(zs, eps=None if noise is None else noise[H:])
        return torch.stack([means[0], means[1], means[2], pi_loss, means[3], weighted_loss, grad_norm]).detach()

    @torch.no_grad()
    def ema(self):
        """helper.py:48-52: target <- lerp(target, model, tau)."""
        if self.engine is not None:
            return self.engine.ema(self.cfg.tau)
        torch._foreach_lerp_(self.target_params, self.params, self.cfg.tau)

    # ------------------------------------------------------------------ graph driver
    def _capturable(self, buffer):
        return self.graph and getattr(buffer, "graph_safe", False)

    def update(self, buffer, step, noise=None):
        """TDMPC.update semantics -> metrics tensor [7] on the device (no sync)."""
        # the engine's hipBLASLt products (learner_engine.mm) follow torch's process-wide fp32 matmul setting: pin
        # full fp32 around every eager pass and capture, whatever the caller set
        prec = torch.get_float32_matmul_precision()
        tf32 = torch.backends.cuda.matmul.allow_tf32
        torch.set_float32_matmul_precision("highest")
        torch.backends.cuda.matmul.allow_tf32 = False
        try:
            return self._update(buffer, step, noise)
        finally:
            torch.set_float32_matmul_precision(prec)
            torch.backends.cuda.matmul.allow_tf32 = tf32

    def _update(self, buffer, step, noise=None):
        self.agent.model.train()
        if noise is not None or not self._capturable(buffer) or self.calls < self.warmup:
            if self._capturable(buffer) and self.calls == self.warmup - 1:
                # the last warm-up runs on a side stream, as graph capture requires of lazily created state
                s = torch.cuda.Stream()
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    m = self.step(buffer, noise)
                torch.cuda.current_stream().wait_stream(s)
            else:
                m = self.step(buffer, noise)
        else:
            key = (buffer.idx, buffer._full)
            g = self._graphs.get(key)
            if g is None:
                if len(self._graphs) >= 2:   # the buffer grew: drop the stale captures
                    self._graphs.clear()
                if self.engine is not None:
                    # the captured update repacks the planner from the engine's buffer (repack_live): pack once now
                    # so the planner holds the live tensors and the pack's job table exists before the capture
                    self.agent.planner.pack(self.agent.model)
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph):
                    out = self.step(buffer)
                g = self._graphs[key] = (graph, out)
                # capture recorded the kernels without running them: run this call's update
            g[0].replay()
            m = g[1]
        self.calls += 1
        if step % self.cfg.update_freq == 0:
            self.ema()
        self.agent.model.eval()
        # parameters changed in place (a graph replay does not bump tensor versions): repack for planning, unless
        # the update itself repacked from the engine's buffer (repack_live)
        if not self._live_pack:
            self.agent.planner._packed_key = None
        return m
