"""The learner engine: one TDMPC.update (tdmpc.py:192-245) as explicit forward and backward passes of HIP kernels.

Reference: /root/reference/src/algorithm/tdmpc.py:165-245 (update_pi, _td_target, update), helper.py:150-176
(TOLD heads), helper.py:71-96 (TruncatedNormal.sample), helper.py:48-52 (ema), torch.optim.Adam and
clip_grad_norm_ as the reference calls them (tdmpc.py:62-63, 180, 236). The math is the reference's; what is
different is that no autograd graph is built: the backward of every head is written out (include/tdmpc_learner.h
documents each kernel), so an update is ~80 launches instead of ~400 autograd / hipBLASLt kernels (ours before)
or ~1,500 (the reference).

Layout (device, float32):
  * every TOLD parameter is a view into ONE flat buffer P (likewise the target into PT), ordered encoder, dynamics,
    reward, Q1, Q2 | pi, so the main optimiser is one Adam pass over P[:n_main] and the policy optimiser one over
    P[n_main:]; gradients go to the flat G, Adam moments to flat M / V;
  * X0 [(H+1) B][L+A, padded to a multiple of 4]: rows t*B..t*B+B-1 hold (z_t, a_t) -- the encoder writes z_0, dynamics step t writes z_{t+1}
    into block t+1 -- so the Q / reward heads read all H steps as one [H B][L+A] operand and the policy update reads
    the H+1 latents in place (stride L+A);
  * activations saved for the backward: each hidden layer's output (ELU / Tanh output; the derivative is a function
    of it), the LayerNorm's xhat and 1/std per row.
Weight gradients: one grouped split-K GEMM launch per optimiser (every dW with the bias as a column of ones), the
LayerNorm affine and scalar output layers as per-workgroup column sums; lg_finalize sums the slices in a fixed order
(so graph replay == eager, bitwise), lg_adam clips by the global norm and applies Adam.
"""
from __future__ import annotations

import ctypes as C
import os

import torch

from . import _lib

ELU, TANH = 2, 1
EPI_NONE, EPI_ELU, EPI_PI, EPI_ELU_BWD, EPI_PI_BWD, EPI_RELU_BWD = 0, 1, 2, 3, 4, 5
CONV_K = (7, 5, 3, 3)                       # helper.enc's pixel convolutions (stride 2, no padding)
CONV_NAMES = ("_encoder.1", "_encoder.3", "_encoder.5", "_encoder.7")
LIN_NAME = "_encoder.10"                    # Flatten -> Linear(32 * 3 * 3 -> L)
NBLK = 2048         # capacity of the norm partials (one per lg_finalize workgroup of 2048 gradients)
ROWS_NWG = 256      # lg_rows_bwd workgroups (column-sum partials per head)
TILE_EXACT = 0x100  # TDMPC_LG_TILE_EXACT (include/tdmpc_learner.h)


def supported(cfg) -> bool:
    """The plain encoder (state MLP, or the pixel conv stack with 32 channels), hidden width 256 / 512 / 1024 (one
    wave per row in the row kernels)."""
    if getattr(cfg, "enc_norm", False) or int(cfg.mlp_dim) not in (256, 512, 1024):
        return False
    if getattr(cfg, "modality", "state") == "pixels":
        return int(cfg.num_channels) == 32 and len(cfg.obs_shape) == 3 and cfg.obs_shape[1] == cfg.obs_shape[2]
    return getattr(cfg, "modality", "state") == "state"


def _p(t, off: int = 0) -> int:
    return t.data_ptr() + 4 * off


def _seg(a, lda, b, ldb, k, amode=0, bmode=0, ones=-1):
    return (a, b, lda, ldb, k, amode, bmode, ones)


class _Adam:
    """Adam state of one flat parameter range (the engine's counterpart of agent.optim / agent.pi_optim)."""

    def __init__(self, params, lo, hi, lr, device):
        self.lo, self.hi, self.lr = lo, hi, lr
        self.exp_avg = torch.zeros(hi - lo, device=device)
        self.exp_avg_sq = torch.zeros(hi - lo, device=device)
        self.step_t = torch.zeros(1, dtype=torch.int32, device=device)
        self.param_groups = [{"params": params, "lr": lr, "betas": (0.9, 0.999), "eps": 1e-8}]

    def state_dict(self):
        return {"step": self.step_t, "exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq}


class Engine:
    def __init__(self, agent):
        self.agent = agent
        cfg = self.cfg = agent.cfg
        self.dev = torch.device(agent.device)
        self.O, self.E, self.L = int(cfg.obs_shape[0]), int(cfg.enc_dim), int(cfg.latent_dim)
        # pixels: the conv stack's spatial sizes 84 -> 39 -> 18 -> 8 -> 3 and the flattened width
        self.pix = getattr(cfg, "modality", "state") == "pixels"
        if self.pix:
            hw = [int(cfg.obs_shape[1])]
            for k in CONV_K:
                hw.append((hw[-1] - k) // 2 + 1)
            self.hw, self.C0 = hw, int(cfg.obs_shape[0])
            self.flat = 32 * hw[-1] * hw[-1]
        self.A, self.M, self.H = int(cfg.action_dim), int(cfg.mlp_dim), int(cfg.horizon)
        self.LA = self.L + self.A
        # X0 / Xtd rows padded to a multiple of 4 floats: their products take 16-byte loads
        self.LAP = (self.LA + 3) & ~3
        order = ["_encoder", "_dynamics", "_reward", "_Q1", "_Q2", "_pi"]
        self.off = {}
        sd = agent.model.state_dict()
        names = [k for pre in order for k in sd if k.startswith(pre + ".")]
        assert len(names) == len(sd), "unexpected TOLD parameters"
        # every tensor starts on a 16-byte boundary (the scalar heads' 1-float biases would leave the next weights
        # misaligned and their products on 4-byte loads); the gaps hold zeros in P, PT, G and the Adam moments
        off = 0
        for k in names:
            off = (off + 3) & ~3
            self.off[k] = (off, tuple(sd[k].shape))
            off += sd[k].numel()
        total = (off + 3) & ~3
        self.P = torch.zeros(total, device=self.dev)
        self.PT = torch.zeros(total, device=self.dev)
        self.G = torch.zeros(total, device=self.dev)
        self.n_main = self.off["_pi.0.weight"][0]
        self._alias(agent.model, self.P)
        self._alias(agent.model_target, self.PT)
        # every parameter's .grad is a view of the flat gradient (lg_adam leaves the clipped gradient there, as
        # clip_grad_norm_ leaves it in .grad)
        for k, p in agent.model.named_parameters():
            o, shape = self.off[k]
            p.grad = self.G[o:o + p.numel()].view(shape)
        lr = float(cfg.lr)
        params = dict(agent.model.named_parameters())
        self.opt_main = _Adam([params[k] for k in names if not k.startswith("_pi.")], 0, self.n_main, lr, self.dev)
        self.opt_pi = _Adam([params[k] for k in names if k.startswith("_pi.")], self.n_main, total, lr, self.dev)
        self.normp = torch.zeros(2, NBLK, device=self.dev)
        self.rho = torch.tensor([cfg.rho ** t for t in range(self.H + 1)], dtype=torch.float32, device=self.dev)
        self.gw = torch.full((1,), 1.0, dtype=torch.float32, device=self.dev) * (1 / self.H)   # the 1/H hook
        self._bufs = {}
        self.lib = _lib.lib()
        # independent passes run on a second stream (forked from and joined back into the caller's; captured into
        # the learner's HIP graph as parallel branches): the TD target beside the encoder + latent rollout, the
        # heads' weight gradients beside the rollout's backward. Both pairs touch disjoint buffers.
        self.side = torch.cuda.Stream(self.dev)
        # lg_gemm's products: the exact f32 MFMA (default: as fast as x6 on the learner's shapes, which are launch-
        # and latency-bound rather than MFMA-bound) or the x6 form (TDMPC_LG_X6=1; set before the first update: the
        # captured graph keeps the choice)
        self.x6 = os.environ.get("TDMPC_LG_X6", "0") == "1"
        # 64 x 64 tiles from this many 64 x 64 output tiles per launch (measured: profiles/r04/learner_tile_ab.txt)
        self.t64 = 240
        # products over at least this many rows (the heads over H B rows; 0 = never) and >= 256 columns run on the
        # LDS-staged macro tiles, tdmpc_lg_gemm tile `big_tile` (tools/lg_gemm_bench.py --big); narrower ones (the
        # latent / action outputs) keep the K-split register tiles
        self.big_rows = int(os.environ.get("TDMPC_LG_BIG_ROWS", "1024"))
        self.big_tile = int(os.environ.get("TDMPC_LG_BIG_TILE", "3"))
        # every grouped product of prod() -- the heads' Q / reward / policy layers over R = H B rows and their dX,
        # with their ELU (pi's layers, the reward first layer) or ELU' (dX) epilogues fused -- runs as ONE grouped
        # tdmpc_lg_gemm launch on the macro tiles: 1.196-1.200 ms per humanoid update against 1.205-1.209 with
        # those products on hipBLASLt (torch.mm / addmm + a tdmpc_lg_act launch) and 1.317-1.320 on the register
        # tiles, graph replay (profiles/r06/learner_macro_tiles_ab.txt). Every sum in a fixed order (graph == eager
        # bitwise). TDMPC_LG_BLAS=1 sends them to hipBLASLt instead (the library picks its own reduction order;
        # Learner.update pins full-fp32 matmul precision around it); set before the first update: the graph keeps it.
        self.blas = os.environ.get("TDMPC_LG_BLAS", "0") == "1"
        self._aux = {}

    def _alias(self, model, flat):
        """Make every parameter of `model` a view into `flat` (values kept)."""
        with torch.no_grad():
            for k, p in model.named_parameters():
                o, shape = self.off[k]
                n = p.numel()
                flat[o:o + n].copy_(p.detach().reshape(-1))
                p.data = flat[o:o + n].view(shape)

    # ---------------------------------------------------------------------------------------------- helpers
    def w(self, k, target=False):
        o, _ = self.off[k]
        return _p(self.PT if target else self.P, o)

    def wv(self, k, target=False):
        """The parameter `k` as a tensor view of the flat buffer."""
        o, shape = self.off[k]
        n = int(torch.Size(shape).numel())
        return (self.PT if target else self.P)[o:o + n].view(shape)

    def mm(self, x, k, out, bias=None, target=False, transpose=False, cols=None, acc=False):
        """out = x @ W^T (+ bias) -- or x @ W with transpose=True (the backward's dX) -- on hipBLASLt (the heads'
        plain products, see self.blas). cols: W's input columns [c0, c1) only; acc: out += x @ W^T."""
        w = self.wv(k, target)
        if cols is not None:
            w = w[:, cols[0]:cols[1]]
        w = w if transpose else w.t()
        if acc:
            out.addmm_(x, w)
        elif bias is None:
            torch.mm(x, w, out=out)
        else:
            torch.addmm(self.wv(bias, target), x, w, out=out)

    def job(self, parts, k, out, bias=None, target=False, transpose=False, epi=EPI_NONE, aux=None):
        """One lg_gemm job: out = sum over parts (x, c0, c1) of x @ W[:, c0:c1]^T (+ bias, + epilogue) -- or
        x @ W (transpose=True, the backward's dX; parts = [(dY, 0, 0)]). x / out may be row-strided views.
        epi EPI_ELU fuses the ELU, EPI_ELU_BWD multiplies by ELU'(aux) (aux: the ELU output)."""
        w = self.wv(k, target)
        N, K = w.shape
        segs = []
        for x, c0, c1 in parts:
            if transpose:
                segs.append(_seg(_p(x), x.stride(0), _p(w), K, N, bmode=1))
            else:
                segs.append(_seg(_p(x), x.stride(0), _p(w, c0), K, c1 - c0))
        j = dict(segs=segs, m=out.shape[0], n=K if transpose else N, c=_p(out), ldc=out.stride(0), epi=epi)
        if bias is not None:
            j["bias"] = self.w(bias, target)
        if aux is not None:
            j["aux"], j["ldaux"] = _p(aux), aux.stride(0)
        return j

    def mms(self, jobs, blas):
        """Run a group of `job` products: each on hipBLASLt through `mm` plus a tdmpc_lg_act launch for a fused
        epilogue (default), or -- TDMPC_LG_BLAS=0 -- ONE grouped lg_gemm launch. blas: the mm() arguments per job."""
        if not self.blas:
            self.gemm(jobs)
            return
        for j, (parts, k, out, bias, target, transpose) in zip(jobs, blas):
            for i, (x, c0, c1) in enumerate(parts):
                self.mm(x, k, out, bias=bias if i == 0 else None, target=target, transpose=transpose,
                        cols=None if transpose or (c0 == 0 and c1 == self.wv(k, target).shape[1]) else (c0, c1),
                        acc=i > 0)
            if j["epi"] == EPI_ELU:
                self.act(out)
            elif j["epi"] == EPI_ELU_BWD:
                self.act(out, self._aux[j["aux"]])

    def prod(self, specs):
        """specs: (parts, k, out, bias, target, transpose, epi, aux) per product -> one grouped launch."""
        jobs, blas = [], []
        for parts, k, out, bias, target, transpose, epi, aux in specs:
            jobs.append(self.job(parts, k, out, bias, target, transpose, epi, aux))
            blas.append((parts, k, out, bias, target, transpose))
            if aux is not None:
                self._aux[_p(aux)] = aux
        self.mms(jobs, blas)

    def act(self, x, y=None):
        """x <- ELU(x) (y None) or x <- x * ELU'(y) in place (tdmpc_lg_act)."""
        _lib.check(self.lib.tdmpc_lg_act(_p(x), None if y is None else _p(y), x.numel(), 0 if y is None else 1,
                                         self._stream()), "tdmpc_lg_act")

    def _stream(self):
        return C.c_void_p(torch.cuda.current_stream(self.dev).cuda_stream)

    def _pair(self, main_steps, side_steps):
        """Issue two independent launch sequences (generators that yield after each launch): main_steps on the
        caller's stream, side_steps on self.side (forked from it here; the caller joins it back), one launch from
        each in turn. In the captured graph the main branch (the critical path) then leads: 1.20 vs 1.21 ms per
        humanoid update against capturing the side branch whole first (profiles/r05/learner_branches.txt)."""
        main = torch.cuda.current_stream(self.dev)
        self.side.wait_stream(main)
        live = [(main, main_steps), (self.side, side_steps)]
        while live:
            for e in list(live):
                with torch.cuda.stream(e[0]):
                    if next(e[1], StopIteration) is StopIteration:
                        live.remove(e)

    def gemm(self, jobs, tile=None):
        """jobs: dicts (segs, m, n, c, ldc, bias, epi, aux, ldaux, res, ldres, c2, ldc2, std, splits, slice)."""
        arr = (_lib.LgJob * len(jobs))()
        tiles64 = 0
        for i, j in enumerate(jobs):
            J = arr[i]
            segs = j["segs"]
            for s, sg in enumerate(segs):
                a, b, lda, ldb, k, am, bm, ones = sg
                J.seg[s].a, J.seg[s].b = a, b
                J.seg[s].lda, J.seg[s].ldb, J.seg[s].k = lda, ldb, k
                J.seg[s].amode, J.seg[s].bmode, J.seg[s].ones_col = am, bm, ones
            J.nseg, J.m, J.n, J.epi = len(segs), j["m"], j["n"], j.get("epi", EPI_NONE)
            J.c, J.ldc = j["c"], j["ldc"]
            J.c2, J.ldc2 = j.get("c2"), j.get("ldc2", 0)
            J.bias = j.get("bias")
            J.aux, J.ldaux = j.get("aux"), j.get("ldaux", 0)
            J.res, J.ldres = j.get("res"), j.get("ldres", 0)
            J.std_ = j.get("std", 0.0)
            J.splits, J.slice = j.get("splits", 1), j.get("slice", 0)
            tiles64 += -(-j["m"] // 64) * -(-j["n"] // 64) * J.splits
        if tile is None and self.big_rows and max(j["m"] for j in jobs) >= self.big_rows and \
                min(j["n"] for j in jobs) >= 256 and all(j.get("splits", 1) == 1 for j in jobs) and \
                all(sg[5] == 0 and sg[7] < 0 for j in jobs for sg in j["segs"]):
            tile = self.big_tile   # LDS-staged macro tiles (exact f32 MFMA) for the products over H B rows
        if tile is None:
            # 64 x 64 tiles only for wide launches of row-major operands; a transposed weight operand (the
            # backward's dX) runs 15-25 % faster on 32 x 32 tiles (tools/lg_gemm_bench.py)
            tbw = any(sg[6] == 1 for j in jobs for sg in j["segs"])
            tile = 2 if tiles64 >= self.t64 and not tbw else 1
        if tile < 3:
            tile |= 0 if self.x6 else TILE_EXACT
        _lib.check(self.lib.tdmpc_lg_gemm(arr, len(jobs), tile, self._stream()), "tdmpc_lg_gemm")

    def rows(self, heads, n, bwd=False, **kw):
        a = _lib.LgRows()
        for i, h in enumerate(heads):
            H = a.hd[i]
            for f in ("x", "y", "xhat", "rstd", "yact", "g", "beta", "w3", "b3", "out", "dq", "part"):
                setattr(H, f, h.get(f))
            H.ldx, H.ldy = h.get("ldx", self.M), h.get("ldy", self.M)
            H.ln, H.act, H.tail = int(h.get("ln", 0)), h["act"], int(h.get("tail", 0))
        a.nh, a.rows, a.m, a.bsz = len(heads), n, self.M, kw.get("bsz", 1)
        a.reward, a.td, a.gamma = kw.get("reward"), kw.get("td"), kw.get("gamma", 0.0)
        a.q1, a.q2, a.rho = kw.get("q1"), kw.get("q2"), kw.get("rho")
        if bwd:
            _lib.check(self.lib.tdmpc_lg_rows_bwd(C.byref(a), ROWS_NWG, self._stream()), "tdmpc_lg_rows_bwd")
        else:
            _lib.check(self.lib.tdmpc_lg_rows_fwd(C.byref(a), self._stream()), "tdmpc_lg_rows_fwd")

    def conv_stack(self, x, n, ys, targets=(False,)):
        """helper.enc's conv stack (4 x Conv2d + ReLU after NormalizeImg; helper.py:119-133) on n normalised frame
        stacks x [n][C0][S][S] (x / 255: the augmentation divides) for one or two weight sets (targets[q]: set q is the target encoder's) -> ReLU outputs ys[q][layer].
        The first layer runs both sets in one launch (same input); later layers read their own set's output."""
        a = _lib.LgConv()
        st = self._stream()
        for i, k in enumerate(CONV_K):
            for g in ([list(range(len(targets)))] if i == 0 else [[q] for q in range(len(targets))]):
                a.x = _p(x) if i == 0 else _p(ys[g[0]][i - 1])
                a.nprob, a.n, a.cin, a.hin, a.k = len(g), n, self.C0 if i == 0 else 32, self.hw[i], k
                a.in_div = 0.0
                for j, q in enumerate(g):
                    a.w[j] = self.w(CONV_NAMES[i] + ".weight", targets[q])
                    a.b[j] = self.w(CONV_NAMES[i] + ".bias", targets[q])
                    a.y[j] = _p(ys[q][i])
                _lib.check(self.lib.tdmpc_lg_conv_fwd(C.byref(a), st), "tdmpc_lg_conv_fwd")

    def conv_backward(self, b, x, B):
        """The conv stack's backward for the main batch (tdmpc.py:200 z = h(aug(obs))): from b["dy"][3] (the masked
        gradient of the last conv's output) down to the first conv's weights -> {name: (slices ptr, K, nslices)}."""
        st, out = self._stream(), {}
        for i in range(3, -1, -1):
            k, hin = CONV_K[i], self.hw[i]
            cin = self.C0 if i == 0 else 32
            K = cin * k * k
            ips = 1                                      # one image per slice: B x ceil(tiles / 4) workgroups
            nsl = -(-B // ips)
            part = self.slot(b, f"conv{i}", nsl * 32 * (K + 1))
            xin = x if i == 0 else b["ym"][i - 1]
            _lib.check(self.lib.tdmpc_lg_conv_bwd_weight(_p(b["dy"][i]), _p(xin), 0.0, _p(part),
                                                          B, cin, hin, k, ips, st), "tdmpc_lg_conv_bwd_weight")
            out[CONV_NAMES[i]] = (_p(part), K, nsl)
            if i > 0:   # the gradient of the layer below's ReLU output, masked by its ReLU
                _lib.check(self.lib.tdmpc_lg_conv_bwd_data(_p(b["dy"][i]), self.w(CONV_NAMES[i] + ".weight"),
                                                            _p(b["ym"][i - 1]), _p(b["dy"][i - 1]), B, 32, hin, k, st),
                           "tdmpc_lg_conv_bwd_data")
        return out

    def bufs(self, B):
        b = self._bufs.get(B)
        if b is not None:
            return b
        H, L, A, M, E, O, LA, LAP = self.H, self.L, self.A, self.M, self.E, self.O, self.LA, self.LAP
        R, R1 = H * B, (H + 1) * B
        z = lambda *s: torch.zeros(*s, device=self.dev)  # noqa: E731
        b = dict(
            eps=z((2 * H + 1) * B, A),
            # TD target
            Yt1=z(R, E), Yo1=z(R, E), NZ=z(R, L), Xtd=z(R, LAP), T1=z(R, M), T2=z(R, M), MUtd=z(R, A),
            TQ=z(2, R), TD=z(R), PAt=z(2, R, M), PBt=z(2, R, M),
            # main forward
            Ye1=z(B, E), X0=z(R1, LAP), Yd1=z(R, M), Yd2=z(R, M), ZP=z(R, L),
            PA=z(3, R1, M), PB=z(3, R1, M), Y1=z(2, R1, M), Y2=z(3, R1, M), XH1=z(2, R1, M), XH2=z(2, R1, M),
            RS1=z(2, R1), RS2=z(2, R1), Q=z(3, R1),
            lrows=z(5, B), scal=z(6), dZP=z(R1, L), dq=z(3, R),
            # main backward
            dP2=z(3, R1, M), dA=z(2, R1, M), dP1=z(3, R1, M), S=z(R, L), DG=z(max(R - B, 1), L), DZ0=z(B, L),
            dP2d=z(R, M), dP1d=z(R, M), dP1e=z(B, E),
            # pi
            Yp1=z(R1, M), Yp2=z(R1, M), ACT=z(R1, A), MU=z(R1, A), dACT=z(R1, A), dPp2=z(R1, M), dPp1=z(R1, M),
            piloss=z(1), gnorm=z(1),
        )
        if self.pix:   # the conv stacks' ReLU outputs (TD: target and online encoders; main: online) and gradients
            hw, R = self.hw, H * B
            b["yt"] = [z(R, 32, hw[i + 1], hw[i + 1]) for i in range(4)]
            b["yo"] = [z(R, 32, hw[i + 1], hw[i + 1]) for i in range(4)]
            b["ym"] = [z(B, 32, hw[i + 1], hw[i + 1]) for i in range(4)]
            b["dy"] = [z(B, 32, hw[i + 1], hw[i + 1]) for i in range(4)]
        # weight-gradient slots: (name, out, in, dY, X, K) resolved per pass; sized for the largest pass
        self._bufs[B] = b
        b["slots"] = {}
        return b

    def slot(self, b, key, numel):
        s = b["slots"].get(key)
        if s is None:
            s = b["slots"][key] = torch.zeros(numel, device=self.dev)
        return s

    # ------------------------------------------------------------------------------------------- passes
    def _td_steps(self, b, nxo_t, rew, R, eps):
        """tdmpc.py:184-190 for all H steps: online encoder + pi (TruncatedNormal draws `eps`), target Q, and the
        target encoder's next_z (tdmpc.py:206-207) -> b["TD"], b["NZ"]. A generator: yields after each launch
        (see _pair)."""
        O, E, L, A, M, LA, LAP = self.O, self.E, self.L, self.A, self.M, self.LA, self.LAP
        w, wt = self.w, (lambda k: self.w(k, True))
        nxo = _p(nxo_t)
        if self.pix:   # the conv stacks of both encoders, then their Linear
            F = self.flat
            self.conv_stack(nxo_t, R, [b["yt"], b["yo"]], targets=(True, False))
            yield
            self.gemm([dict(segs=[_seg(_p(b["yt"][3]), F, wt(LIN_NAME + ".weight"), F, F)], m=R, n=L, c=_p(b["NZ"]),
                            ldc=L, bias=wt(LIN_NAME + ".bias")),
                       dict(segs=[_seg(_p(b["yo"][3]), F, w(LIN_NAME + ".weight"), F, F)], m=R, n=L, c=_p(b["Xtd"]),
                            ldc=LAP, bias=w(LIN_NAME + ".bias"))])
            yield
        else:
            self.gemm([dict(segs=[_seg(nxo, O, wt("_encoder.0.weight"), O, O)], m=R, n=E, c=_p(b["Yt1"]), ldc=E,
                            bias=wt("_encoder.0.bias"), epi=EPI_ELU),
                       dict(segs=[_seg(nxo, O, w("_encoder.0.weight"), O, O)], m=R, n=E, c=_p(b["Yo1"]), ldc=E,
                            bias=w("_encoder.0.bias"), epi=EPI_ELU)])
            yield
            self.gemm([dict(segs=[_seg(_p(b["Yt1"]), E, wt("_encoder.2.weight"), E, E)], m=R, n=L, c=_p(b["NZ"]),
                            ldc=L, bias=wt("_encoder.2.bias")),
                       dict(segs=[_seg(_p(b["Yo1"]), E, w("_encoder.2.weight"), E, E)], m=R, n=L, c=_p(b["Xtd"]),
                            ldc=LAP, bias=w("_encoder.2.bias"))])
            yield
        self.prod([([(b["Xtd"][:, :L], 0, L)], "_pi.0.weight", b["T1"], "_pi.0.bias", False, False, EPI_ELU, None)])
        yield
        self.prod([([(b["T1"], 0, M)], "_pi.2.weight", b["T2"], "_pi.2.bias", False, False, EPI_ELU, None)])
        yield
        self.gemm([dict(segs=[_seg(_p(b["T2"]), M, w("_pi.4.weight"), M, M)], m=R, n=A, c=_p(b["Xtd"], L),
                        ldc=LAP, bias=w("_pi.4.bias"), epi=EPI_PI, aux=eps, ldaux=A, c2=_p(b["MUtd"]), ldc2=A,
                        std=float(self.cfg.min_std))])
        yield
        PA, PB = b["PAt"], b["PBt"]
        self.prod([([(b["Xtd"][:, :LA], 0, LA)], f"_Q{h + 1}.0.weight", PA[h, :R], f"_Q{h + 1}.0.bias", True, False,
                    EPI_NONE, None) for h in range(2)])
        yield
        self.rows([dict(x=_p(PA[h]), y=_p(PB[h]), ln=1, g=wt(f"_Q{h + 1}.1.weight"), beta=wt(f"_Q{h + 1}.1.bias"),
                        act=TANH) for h in range(2)], R)
        yield
        self.prod([([(PB[h, :R], 0, M)], f"_Q{h + 1}.3.weight", PA[h, :R], f"_Q{h + 1}.3.bias", True, False,
                    EPI_NONE, None) for h in range(2)])
        yield
        self.rows([dict(x=_p(PA[h]), ln=1, g=wt(f"_Q{h + 1}.4.weight"), beta=wt(f"_Q{h + 1}.4.bias"), act=ELU,
                        tail=1, w3=wt(f"_Q{h + 1}.6.weight"), b3=wt(f"_Q{h + 1}.6.bias"), out=_p(b["TQ"][h]))
                   for h in range(2)], R, reward=rew, td=_p(b["TD"]), gamma=float(self.cfg.discount))

    def _fwd_steps(self, b, obs, action, B):
        """The update's forward (tdmpc.py:199-213): encoder, latent rollout, heads over the H B rollout rows. A
        generator: yields after each launch (see _pair)."""
        H, O, E, L, M, LA, LAP = self.H, self.O, self.E, self.L, self.M, self.LA, self.LAP
        R = H * B
        w, X0 = self.w, b["X0"]
        if self.pix:
            F = self.flat
            self.conv_stack(obs, B, [b["ym"]])
            yield
            self.gemm([dict(segs=[_seg(_p(b["ym"][3]), F, w(LIN_NAME + ".weight"), F, F)], m=B, n=L, c=_p(X0), ldc=LAP,
                            bias=w(LIN_NAME + ".bias"))])
            yield
        else:
            self.gemm([dict(segs=[_seg(_p(obs), O, w("_encoder.0.weight"), O, O)], m=B, n=E, c=_p(b["Ye1"]), ldc=E,
                            bias=w("_encoder.0.bias"), epi=EPI_ELU)])
            yield
            self.gemm([dict(segs=[_seg(_p(b["Ye1"]), E, w("_encoder.2.weight"), E, E)], m=B, n=L, c=_p(X0), ldc=LAP,
                            bias=w("_encoder.2.bias"))])
            yield
        X0.view(H + 1, B, LAP)[:H, :, L:LA].copy_(action[:H])
        yield
        for t in range(H):
            self.gemm([dict(segs=[_seg(_p(X0, t * B * LAP), LAP, w("_dynamics.0.weight"), LA, LA)], m=B, n=M,
                            c=_p(b["Yd1"], t * B * M), ldc=M, bias=w("_dynamics.0.bias"), epi=EPI_ELU)])
            yield
            self.gemm([dict(segs=[_seg(_p(b["Yd1"], t * B * M), M, w("_dynamics.2.weight"), M, M)], m=B, n=M,
                            c=_p(b["Yd2"], t * B * M), ldc=M, bias=w("_dynamics.2.bias"), epi=EPI_ELU)])
            yield
            self.gemm([dict(segs=[_seg(_p(b["Yd2"], t * B * M), M, w("_dynamics.4.weight"), M, M)], m=B, n=L,
                            c=_p(X0, (t + 1) * B * LAP), ldc=LAP, bias=w("_dynamics.4.bias"),
                            c2=_p(b["ZP"], t * B * L), ldc2=L)])
            yield
        # reward head layer 1 (ELU) rides in its own slot 2 of PA / Y2 buffers, in the Q heads' first-layer launch
        PA = b["PA"]
        PA, PB, Y1, Y2, XH1, XH2, RS1, RS2 = self.q_forward(
            b, R, [(X0[:R, :LA], 0, LA)], extra=[([(X0[:R, :LA], 0, LA)], "_reward.0.weight", PA[2, :R], "_reward.0.bias",
                                              False, False, EPI_ELU, None)])
        yield
        self.prod([([(Y1[h, :R], 0, M)], f"_Q{h + 1}.3.weight", PB[h, :R], f"_Q{h + 1}.3.bias", False, False,
                    EPI_NONE, None) for h in range(2)] +
                  [([(PA[2, :R], 0, M)], "_reward.2.weight", PB[2, :R], "_reward.2.bias", False, False, EPI_NONE,
                    None)])
        yield
        Q = b["Q"]
        heads = [dict(x=_p(PB[h]), y=_p(Y2[h]), xhat=_p(XH2[h]), rstd=_p(RS2[h]), ln=1, g=w(f"_Q{h + 1}.4.weight"),
                      beta=w(f"_Q{h + 1}.4.bias"), act=ELU, tail=1, w3=w(f"_Q{h + 1}.6.weight"),
                      b3=w(f"_Q{h + 1}.6.bias"), out=_p(Q[h])) for h in range(2)]
        heads.append(dict(x=_p(PB[2]), y=_p(Y2[2]), act=ELU, tail=1, w3=w("_reward.4.weight"),
                          b3=w("_reward.4.bias"), out=_p(Q[2])))
        self.rows(heads, R)

    def _rollout_bwd_steps(self, b, B):
        """Backward through the latent rollout (tdmpc.py:203-205), newest step first: b["S"] (the heads' gradient
        of z_t) and dZP -> DG / DZ0. A generator: yields after each launch (see _pair)."""
        H, L, M, LA = self.H, self.L, self.M, self.LA
        w, S, dZP = self.w, b["S"], b["dZP"]
        DG, dP2d, dP1d, DZ0 = b["DG"], b["dP2d"], b["dP1d"], b["DZ0"]
        for t in range(H - 1, -1, -1):
            g_t = _p(dZP, H * B * L) if t == H - 1 else _p(DG, t * B * L)     # d loss / d z_{t+1}
            self.gemm([dict(segs=[_seg(g_t, L, w("_dynamics.4.weight"), M, L, bmode=1)], m=B, n=M,
                            c=_p(dP2d, t * B * M), ldc=M, epi=EPI_ELU_BWD, aux=_p(b["Yd2"], t * B * M), ldaux=M)])
            yield
            self.gemm([dict(segs=[_seg(_p(dP2d, t * B * M), M, w("_dynamics.2.weight"), M, M, bmode=1)], m=B, n=M,
                            c=_p(dP1d, t * B * M), ldc=M, epi=EPI_ELU_BWD, aux=_p(b["Yd1"], t * B * M), ldaux=M)])
            yield
            out = _p(DG, (t - 1) * B * L) if t > 0 else _p(DZ0)
            self.gemm([dict(segs=[_seg(_p(dP1d, t * B * M), M, w("_dynamics.0.weight"), LA, M, bmode=1)], m=B,
                            n=L, c=out, ldc=L, res=_p(S, t * B * L), ldres=L)])
            yield

    def q_forward(self, b, n, parts, extra=()):
        """helper.q layer 1 + LayerNorm + Tanh for both Q heads over n rows; the input is the concatenation of
        parts [(tensor [n, c1 - c0], c0, c1)] along the feature axis. extra: more prod() specs run in the same
        grouped launch as the two first layers (the reward head's, which reads the same input)."""
        w = self.w
        PA, PB, Y1, Y2, XH1, XH2, RS1, RS2 = (b[k] for k in ("PA", "PB", "Y1", "Y2", "XH1", "XH2", "RS1", "RS2"))
        self.prod([(parts, f"_Q{h + 1}.0.weight", PA[h, :n], f"_Q{h + 1}.0.bias", False, False, EPI_NONE, None)
                   for h in range(2)] + list(extra))
        self.rows([dict(x=_p(PA[h]), y=_p(Y1[h]), xhat=_p(XH1[h]), rstd=_p(RS1[h]), ln=1,
                        g=w(f"_Q{h + 1}.1.weight"), beta=w(f"_Q{h + 1}.1.bias"), act=TANH) for h in range(2)], n)
        return PA, PB, Y1, Y2, XH1, XH2, RS1, RS2

    def update(self, buffer, noise=None):
        """One TDMPC.update without the EMA -> metrics [7] (learner.METRICS order)."""
        cfg, dev = self.cfg, self.dev
        H, O, E, L, A, M, LA = self.H, self.O, self.E, self.L, self.A, self.M, self.LA
        obs, next_obses, action, reward, idxs, weights = buffer.sample()
        B = obs.shape[0]
        R, R1 = H * B, (H + 1) * B
        b = self.bufs(B)
        if self.pix:
            # RandomShiftsAug (helper.py:250-283) on the H next-observation stacks, then on obs: the same shift
            # distribution as the reference's update, NOT its random stream -- the reference draws aug(obs) first
            # (tdmpc.py:200) and then one B-sized draw per horizon step (tdmpc.py:209), so at one seed the shifts
            # differ; the frames may come as uint8 from the replay buffer
            # (NormalizeImg's x / 255 folded into the shift's gather: the conv stack reads normalised frames)
            nx = next_obses[:H].reshape(H * B, *next_obses.shape[2:])
            nxo_t = self.agent.aug(nx if nx.dtype == torch.float32 else nx.float(), div=255.0).contiguous()
            obs = self.agent.aug(obs if obs.dtype == torch.float32 else obs.float(), div=255.0).contiguous()
        else:
            obs = obs.contiguous()
            nxo_t = next_obses[:H].contiguous()
        rew_t = reward[:H].contiguous()
        weights = weights.contiguous()
        if noise is None:
            b["eps"].normal_()
        else:
            b["eps"].copy_(torch.cat([x.reshape(B, A) for x in noise]).to(dev))
        eps = b["eps"]
        rew = _p(rew_t)
        w = self.w

        # ---- forward (encoder, latent rollout, heads) beside the TD targets and target latents (no gradient) ----
        main = torch.cuda.current_stream(dev)
        self._pair(self._fwd_steps(b, obs, action, B), self._td_steps(b, nxo_t, rew, R, _p(eps)))
        X0, Q = b["X0"], b["Q"]
        PA, PB, Y1, Y2, XH1, XH2, RS1, RS2 = (b[k] for k in ("PA", "PB", "Y1", "Y2", "XH1", "XH2", "RS1", "RS2"))

        main.wait_stream(self.side)   # TD / NZ ready
        # ---- losses (fused HIP loss, include/tdmpc_learner.h) ----
        la = _lib.LossArgs(_p(b["ZP"]), _p(b["NZ"]), _p(Q[0]), _p(Q[1]), _p(Q[2]), rew, _p(b["TD"]), _p(weights),
                           _p(self.rho), H, B, L, float(cfg.consistency_coef), float(cfg.reward_coef),
                           float(cfg.value_coef))
        st = self._stream()
        _lib.check(self.lib.tdmpc_loss_forward(C.byref(la), _p(b["lrows"]), _p(b["scal"]), st), "loss_forward")
        dq = b["dq"]
        _lib.check(self.lib.tdmpc_loss_backward(C.byref(la), _p(b["lrows"]), _p(b["scal"]), _p(self.gw),
                                                _p(b["dZP"], B * L), _p(dq[0]), _p(dq[1]), _p(dq[2]), st),
                   "loss_backward")

        # ---- backward through the heads ----
        dP2, dA, dP1 = b["dP2"], b["dA"], b["dP1"]
        PW2, PWr, PW1 = 3 * M + 1, M + 1, 2 * M
        part2 = [self.slot(b, f"pq2_{h}", ROWS_NWG * PW2) for h in range(2)]
        partr = self.slot(b, "pr", ROWS_NWG * PWr)
        part1 = [self.slot(b, f"pq1_{h}", ROWS_NWG * PW1) for h in range(2)]
        heads = [dict(y=_p(dP2[h]), yact=_p(Y2[h]), xhat=_p(XH2[h]), rstd=_p(RS2[h]), ln=1,
                      g=w(f"_Q{h + 1}.4.weight"), act=ELU, tail=1, w3=w(f"_Q{h + 1}.6.weight"), dq=_p(dq[h]),
                      part=_p(part2[h])) for h in range(2)]
        heads.append(dict(y=_p(dP2[2]), yact=_p(Y2[2]), act=ELU, tail=1, w3=w("_reward.4.weight"), dq=_p(dq[2]),
                          part=_p(partr)))
        self.rows(heads, R, bwd=True)
        self.prod([([(dP2[h, :R], 0, 0)], f"_Q{h + 1}.3.weight", dA[h, :R], None, False, True, EPI_NONE, None)
                   for h in range(2)] +
                  [([(dP2[2, :R], 0, 0)], "_reward.2.weight", dP1[2, :R], None, False, True, EPI_ELU_BWD, PA[2, :R])])
        self.rows([dict(x=_p(dA[h]), y=_p(dP1[h]), yact=_p(Y1[h]), xhat=_p(XH1[h]), rstd=_p(RS1[h]), ln=1,
                        g=w(f"_Q{h + 1}.1.weight"), act=TANH, part=_p(part1[h])) for h in range(2)], R, bwd=True)
        # gradient of z_t from the three heads (+ the consistency term on z_t): S = sum_h dP1_h W1_h[:, :L] + dZP
        S, dZP = b["S"], b["dZP"]
        self.gemm([dict(segs=[_seg(_p(dP1[0]), M, w("_Q1.0.weight"), LA, M, bmode=1),
                              _seg(_p(dP1[1]), M, w("_Q2.0.weight"), LA, M, bmode=1),
                              _seg(_p(dP1[2]), M, w("_reward.0.weight"), LA, M, bmode=1)],
                         m=R, n=L, c=_p(S), ldc=L, res=_p(dZP), ldres=L)])
        # ---- the heads' weight gradients (side stream) beside the latent rollout's backward ----
        sp = 4 if R >= 1024 else 1
        dw_h = [("_reward.2", M, M, [_seg(_p(dP2[2]), M, _p(PA[2]), M, R, 1, 1, M)], sp),
                ("_reward.0", M, LA, [_seg(_p(dP1[2]), M, _p(X0), self.LAP, R, 1, 1, LA)], sp)]
        for h in range(2):
            dw_h += [(f"_Q{h + 1}.3", M, M, [_seg(_p(dP2[h]), M, _p(Y1[h]), M, R, 1, 1, M)], sp),
                     (f"_Q{h + 1}.0", M, LA, [_seg(_p(dP1[h]), M, _p(X0), self.LAP, R, 1, 1, LA)], sp)]
        # pi's forward over the detached latents z_0..z_H for update_pi (reads X0 and pi's weights only, which the
        # main optimiser step does not touch) rides on the side stream after them
        slots = {}

        def side_steps():
            slots.update(self._dw(b, "mainh", dw_h))
            yield
            yield from self._pi_fwd_steps(b, X0[:, :L], R1, _p(eps, R * A))

        self._pair(self._rollout_bwd_steps(b, B), side_steps())
        DG, dP2d, dP1d, DZ0 = b["DG"], b["dP2d"], b["dP1d"], b["DZ0"]
        conv = {}
        if self.pix:   # Linear backward with the last conv's ReLU mask, then the conv stack's backward
            F = self.flat
            self.gemm([dict(segs=[_seg(_p(DZ0), L, w(LIN_NAME + ".weight"), F, L, bmode=1)], m=B, n=F,
                            c=_p(b["dy"][3]), ldc=F, epi=EPI_RELU_BWD, aux=_p(b["ym"][3]), ldaux=F)])
            conv = self.conv_backward(b, obs, B)
            dw_enc = [(LIN_NAME, L, F, [_seg(_p(DZ0), L, _p(b["ym"][3]), F, B, 1, 1, F)], 1)]
        else:
            self.gemm([dict(segs=[_seg(_p(DZ0), L, w("_encoder.2.weight"), E, L, bmode=1)], m=B, n=E,
                            c=_p(b["dP1e"]), ldc=E, epi=EPI_ELU_BWD, aux=_p(b["Ye1"]), ldaux=E)])
            dw_enc = [("_encoder.2", L, E, [_seg(_p(DZ0), L, _p(b["Ye1"]), E, B, 1, 1, E)], 1),
                      ("_encoder.0", E, O, [_seg(_p(b["dP1e"]), E, _p(obs), O, B, 1, 1, O)], 1)]

        # ---- the rollout's weight gradients (one grouped launch) ----
        g_dyn3 = ([_seg(_p(DG), L, _p(b["Yd2"]), M, R - B, 1, 1, M)] if H > 1 else []) + \
            [_seg(_p(dZP, H * B * L), L, _p(b["Yd2"], (H - 1) * B * M), M, B, 1, 1, M)]
        dw = dw_enc + [
              ("_dynamics.4", L, M, g_dyn3, sp),
              ("_dynamics.2", M, M, [_seg(_p(dP2d), M, _p(b["Yd1"]), M, R, 1, 1, M)], sp),
              ("_dynamics.0", M, LA, [_seg(_p(dP1d), M, _p(X0), self.LAP, R, 1, 1, LA)], sp)]
        slots.update(self._dw(b, "main", dw))
        main.wait_stream(self.side)   # the heads' slices ready
        dw += dw_h

        # ---- finalize (sum slices, global norm), clip + Adam ----
        src = {}
        for name, o, i, _, s in dw:
            src[name + ".weight"] = (slots[name], o, i, i + 1, s, o * (i + 1))
            src[name + ".bias"] = (slots[name] + 4 * i, o, 1, i + 1, s, o * (i + 1))
        for h in range(2):
            q = f"_Q{h + 1}"
            src[q + ".1.weight"] = (_p(part1[h]), 1, M, M, ROWS_NWG, PW1)
            src[q + ".1.bias"] = (_p(part1[h], M), 1, M, M, ROWS_NWG, PW1)
            src[q + ".4.weight"] = (_p(part2[h]), 1, M, M, ROWS_NWG, PW2)
            src[q + ".4.bias"] = (_p(part2[h], M), 1, M, M, ROWS_NWG, PW2)
            src[q + ".6.weight"] = (_p(part2[h], 2 * M), 1, M, M, ROWS_NWG, PW2)
            src[q + ".6.bias"] = (_p(part2[h], 3 * M), 1, 1, 1, ROWS_NWG, PW2)
        for name, (ptr, K, nsl) in conv.items():   # the conv weight-gradient slices [nsl][32][K + 1]
            src[name + ".weight"] = (ptr, 32, K, K + 1, nsl, 32 * (K + 1))
            src[name + ".bias"] = (ptr + 4 * K, 32, 1, K + 1, nsl, 32 * (K + 1))
        src["_reward.4.weight"] = (_p(partr), 1, M, M, ROWS_NWG, PWr)
        src["_reward.4.bias"] = (_p(partr, M), 1, 1, 1, ROWS_NWG, PWr)
        self._optimise(self.opt_main, src, 0, _p(b["gnorm"]))
        buffer.update_priorities(idxs, b["lrows"][3].view(B, 1))

        # ---- update_pi on the detached latents z_0..z_H (tdmpc.py:165-182) ----
        pi_loss = self._update_pi(b, X0[:, :L], H + 1, B, _p(eps, R * A), pi_fwd_done=True)
        scal = b["scal"]
        return torch.cat([scal[0:3], pi_loss, scal[3:5], b["gnorm"]])

    def _dw(self, b, tag, dw):
        """One grouped launch of every weight gradient of a pass -> {name: slot pointer}."""
        jobs, slots = [], {}
        for name, o, i, segs, s in dw:
            buf = self.slot(b, f"{tag}:{name}", s * o * (i + 1))
            slots[name] = _p(buf)
            jobs.append(dict(segs=segs, m=o, n=i + 1, c=_p(buf), ldc=i + 1, splits=s, slice=o * (i + 1)))
        # 32 x 32 tiles, K (the rows) split 4 ways: 2-3x faster than 64 x 64 tiles for these narrow-N / long-K
        # products on MI355X (tools/lg_gemm_bench.py --dw: 512 x 122 x 2560 12 vs 38 us)
        self.gemm(jobs, tile=1)
        return slots

    def _optimise(self, opt, src, g_lo, norm_out):
        """lg_finalize over the optimiser's tensors (in flat order), then lg_adam over its flat range."""
        names = [k for k in self.off if (k in src)]
        names.sort(key=lambda k: self.off[k][0])
        arr = (_lib.LgGsrc * len(names))()
        for i, k in enumerate(names):
            p, rows, cols, ld, ns, ss = src[k]
            o, shape = self.off[k]
            assert rows * cols == int(torch.Size(shape).numel()), k
            T = arr[i]
            T.src, T.dst, T.sstride, T.rows, T.cols, T.ld, T.nslices = p, o - opt.lo, ss, rows, cols, ld, ns
        assert self.off[names[0]][0] == opt.lo
        which = 0 if opt is self.opt_main else 1
        normp = _p(self.normp[which])
        st = self._stream()
        _lib.check(self.lib.tdmpc_lg_finalize(arr, len(names), _p(self.G, opt.lo), normp, NBLK, _p(opt.step_t), st),
                   "tdmpc_lg_finalize")
        _lib.check(self.lib.tdmpc_lg_adam(_p(self.P, opt.lo), _p(self.G, opt.lo), _p(opt.exp_avg),
                                          _p(opt.exp_avg_sq), opt.hi - opt.lo, normp, NBLK, _p(opt.step_t),
                                          opt.lr, 0.9, 0.999, 1e-8, float(self.cfg.grad_clip_norm), norm_out, st),
                   "tdmpc_lg_adam")

    def _pi_fwd_steps(self, b, zt, n, eps):
        """pi's forward for update_pi over the n rows of zt (TruncatedNormal draws `eps`) -> b["Yp1"], b["Yp2"],
        b["ACT"], b["MU"]. A generator: yields after each launch (see _pair)."""
        L, A, M = self.L, self.A, self.M
        w = self.w
        self.prod([([(zt, 0, L)], "_pi.0.weight", b["Yp1"][:n], "_pi.0.bias", False, False, EPI_ELU, None)])
        yield
        self.prod([([(b["Yp1"][:n], 0, M)], "_pi.2.weight", b["Yp2"][:n], "_pi.2.bias", False, False, EPI_ELU, None)])
        yield
        self.gemm([dict(segs=[_seg(_p(b["Yp2"]), M, w("_pi.4.weight"), M, M)], m=n, n=A, c=_p(b["ACT"]), ldc=A,
                        bias=w("_pi.4.bias"), epi=EPI_PI, aux=eps, ldaux=A, c2=_p(b["MU"]), ldc2=A,
                        std=float(self.cfg.min_std))])
        yield

    def _update_pi(self, b, zt, nt, B, eps, pi_fwd_done=False):
        """TDMPC.update_pi over the nt latent blocks of B rows of zt ([nt B, L], rows may be strided) -> pi_loss
        tensor [1]. pi_fwd_done: _pi_fwd_steps already ran over the same rows and draws."""
        L, A, M, LA = self.L, self.A, self.M, self.LA
        n = nt * B
        w = self.w
        z, ldz = _p(zt), zt.stride(0)
        if not pi_fwd_done:
            for _ in self._pi_fwd_steps(b, zt, n, eps):
                pass
        PA, PB, Y1, Y2, XH1, XH2, RS1, RS2 = self.q_forward(b, n, [(zt, 0, L), (b["ACT"][:n], L, LA)])
        self.prod([([(Y1[h, :n], 0, M)], f"_Q{h + 1}.3.weight", PB[h, :n], f"_Q{h + 1}.3.bias", False, False,
                    EPI_NONE, None) for h in range(2)])
        Q = b["Q"]
        self.rows([dict(x=_p(PB[h]), y=_p(Y2[h]), xhat=_p(XH2[h]), rstd=_p(RS2[h]), ln=1, g=w(f"_Q{h + 1}.4.weight"),
                        beta=w(f"_Q{h + 1}.4.bias"), act=ELU, tail=1, w3=w(f"_Q{h + 1}.6.weight"),
                        b3=w(f"_Q{h + 1}.6.bias"), out=_p(Q[h])) for h in range(2)], n)
        st = self._stream()
        _lib.check(self.lib.tdmpc_lg_pi_loss(_p(Q[0]), _p(Q[1]), _p(self.rho), nt, B, _p(b["piloss"]), st),
                   "tdmpc_lg_pi_loss")
        # backward to the action (Q weights frozen: no weight gradients), then through pi
        dP2, dA, dP1 = b["dP2"], b["dA"], b["dP1"]
        self.rows([dict(y=_p(dP2[h]), yact=_p(Y2[h]), xhat=_p(XH2[h]), rstd=_p(RS2[h]), ln=1,
                        g=w(f"_Q{h + 1}.4.weight"), act=ELU, tail=1, w3=w(f"_Q{h + 1}.6.weight"))
                   for h in range(2)], n, bwd=True, q1=_p(Q[0]), q2=_p(Q[1]), rho=_p(self.rho), bsz=B)
        self.prod([([(dP2[h, :n], 0, 0)], f"_Q{h + 1}.3.weight", dA[h, :n], None, False, True, EPI_NONE, None)
                   for h in range(2)])
        self.rows([dict(x=_p(dA[h]), y=_p(dP1[h]), yact=_p(Y1[h]), xhat=_p(XH1[h]), rstd=_p(RS1[h]), ln=1,
                        g=w(f"_Q{h + 1}.1.weight"), act=TANH) for h in range(2)], n, bwd=True)
        self.gemm([dict(segs=[_seg(_p(dP1[h]), M, w(f"_Q{h + 1}.0.weight") + 4 * L, LA, M, bmode=1)
                              for h in range(2)],
                        m=n, n=A, c=_p(b["dACT"]), ldc=A, epi=EPI_PI_BWD, aux=_p(b["MU"]), ldaux=A)])
        self.gemm([dict(segs=[_seg(_p(b["dACT"]), A, w("_pi.4.weight"), M, A, bmode=1)], m=n, n=M,
                        c=_p(b["dPp2"]), ldc=M, epi=EPI_ELU_BWD, aux=_p(b["Yp2"]), ldaux=M)])
        self.prod([([(b["dPp2"][:n], 0, 0)], "_pi.2.weight", b["dPp1"][:n], None, False, True, EPI_ELU_BWD,
                    b["Yp1"][:n])])
        sp = 4 if n >= 1024 else 1
        dw = [("_pi.4", A, M, [_seg(_p(b["dACT"]), A, _p(b["Yp2"]), M, n, 1, 1, M)], sp),
              ("_pi.2", M, M, [_seg(_p(b["dPp2"]), M, _p(b["Yp1"]), M, n, 1, 1, M)], sp),
              ("_pi.0", M, L, [_seg(_p(b["dPp1"]), M, z, ldz, n, 1, 1, L)], sp)]
        slots = self._dw(b, f"pi{n}", dw)
        src = {}
        for name, o, i, _, s in dw:
            src[name + ".weight"] = (slots[name], o, i, i + 1, s, o * (i + 1))
            src[name + ".bias"] = (slots[name] + 4 * i, o, 1, i + 1, s, o * (i + 1))
        self._optimise(self.opt_pi, src, self.n_main, None)
        return b["piloss"]

    def update_pi(self, zs, eps=None):
        """The public TDMPC.update_pi(zs): zs a list of [B, L] latents (detached) -> pi_loss tensor [1]."""
        B = zs[0].shape[0]
        nt = len(zs)
        b = self.bufs(B)
        if nt > self.H + 1:
            raise ValueError(f"update_pi: at most horizon + 1 = {self.H + 1} latent blocks")
        Z = torch.cat([z.detach().reshape(B, self.L) for z in zs]).contiguous()
        e = b["eps"][self.H * B:(self.H + nt) * B]
        if eps is None:
            e.normal_()
        else:
            e.copy_(torch.cat([x.reshape(B, self.A) for x in list(eps)[:nt]]).to(self.dev))
        b["zpi"] = Z          # kept alive until the kernels have run
        return self._update_pi(b, Z, nt, B, _p(e)).clone()

    def ema(self, tau):
        _lib.check(self.lib.tdmpc_lg_lerp(_p(self.PT), _p(self.P), self.P.numel(), float(tau), self._stream()),
                   "tdmpc_lg_lerp")
