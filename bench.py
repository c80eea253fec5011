"""bench.py -- plan-steps/sec of TDMPC.plan on MI355X (BASELINE.json metric), one process per GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config humanoid-run] [--envs-per-gpu B]
    torchrun --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...

Workload (BASELINE.json configs[2], the north-star target): humanoid-run, N=512 candidates, H=5, 6 CEM
iterations, mixture 0.5 (P=256 pi trajectories, T=768 rows), K=64 elites, latent 100 (cfgs/tasks/humanoid.yaml:6),
fp32. A "step" is one planning call for the B environments a GPU owns: B complete, independent TDMPC.plan
computations (each env its own observation, noise, CEM state and elite choice; bitwise identical to B separate
single-env calls, tests/test_gpu_plan.py::test_batched_equals_single). The default B = 32 envs per GPU is the
smallest vectorised batch that fills the chip: its rollout launches are 1024 chain workgroups (4 per CU, two
co-resident), where B = 8 (BASELINE.json configs[3]'s "8 per GPU") is exactly one per CU and leaves latency
exposed (plan FP32 fraction 0.56 at B = 8, 0.76 at B = 32, 0.78 at B = 64). B = 8 and the
single-env drop-in path (B = 1, one plan() per call, latency-bound) are timed in the same run and reported
under "batch_sweep" and "single_env".

Multi-GPU: environments are independent units, so every rank plans its own B envs on its own
weight replica (weak scaling) and each step ends with one RCCL all-gather over xGMI of the per-env results
([B, A+2]: action, reward mean, std) so that every rank holds the whole vectorised batch.

Rank 0 prints ONE JSON line with, besides the driver's contract fields,
  roofline     : the dominant kernel -- the CEM rollout step (TOLD.next over the B*N candidate rows, 5 launches
                 per iteration): algorithmic FLOPs per launch / average launch time, HIP events around every
                 launch on its stream over an eager replay of the same steps; traffic from
                 profiles/pmc_traffic.json (rocprofv3 PMC FETCH_SIZE x2 + WRITE_SIZE per launch,
                 MI355X_MICROARCH.md §HBM correction) when present;
  cpu_baseline : the oracle's CPU restatement of the reference plan() (pinned bit-exact to the reference's own
                 outputs, tests/test_oracle.py) timed on this host's cores over a bounded sample.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from tdmpc_amd import _lib  # noqa: E402
from tdmpc_amd.config import bench_cfg  # noqa: E402
from tdmpc_amd.parallel import EnvShardedPlanner  # noqa: E402
from tdmpc_amd.tdmpc import TDMPC  # noqa: E402
from tdmpc_amd.told import synthetic_state_dict  # noqa: E402

FP32_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 matrix = vector peak (spec)
# x6 chain kernels: each fp32 product is 6 bf16 MFMA products (three-way split of both operands), so their roof is
# the dense BF16 MFMA peak / 6 in fp32-product FLOP/s (BF16 = 16 x the f32 MFMA rate, MI355X_MICROARCH.md)
X6_PEAK_TFLOPS = round(FP32_PEAK_TFLOPS * 16 / 6, 1)
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E peak (spec)
LDSDMA_CEILING_TBS = 16.4  # measured: the wide kernel's own LDS-DMA ring alone, 256 CUs (tools/mb/dma_ring.hip, profiles/r05/)


def plan_flops(cfg, executed: bool) -> float:
    """Algorithmic FLOPs of one plan-step: 2*[P*H*(pi+d+R) + I*T*(H*(d+R) + pi + 2Q) + enc].
    executed=True counts what this build runs: the pi rows' H-step rollout is identical in every CEM
    iteration (same z0, same pi actions), so it is computed once per plan and only N rows are rolled out
    per iteration; the pi rows' terminal mean tanh(pi(z_H)) likewise, so the terminal pi runs over T rows in
    iteration 0 and over the N sampled rows after it (only the TruncatedNormal sample is redrawn); and at t = 0
    every row of an env starts from its z0, so TOLD.next's first layer runs over the action k group(s) only
    (rup(A, 16) columns) with the latent share computed once per env and head (z0c_kernel)."""
    L, A, M, E = cfg.latent_dim, cfg.action_dim, cfg.mlp_dim, cfg.enc_dim
    N = cfg.num_samples
    P = int(cfg.mixture_coef * N)
    T, H, I = N + P, cfg.horizon, cfg.iterations
    d = (L + A) * M + M * M + M * L
    R = (L + A) * M + M * M + M
    pi = L * M + M * M + M * A
    Q = (L + A) * M + M * M + M
    if cfg.modality == "pixels":
        enc = 0
        s, c, ch = cfg.img_size, 3 * cfg.frame_stack, cfg.num_channels
        for k in (7, 5, 3, 3):
            so = (s - k) // 2 + 1
            enc += ch * so * so * c * k * k
            s, c = so, ch
        enc += ch * s * s * L
    else:
        enc = cfg.obs_shape[0] * E + E * L
    if executed:
        macs = P * H * (pi + d + R) + I * (N * H * (d + R) + T * 2 * Q) + (T + (I - 1) * N) * pi + enc
        k1c = -(-A // 16) * 16
        macs -= (I * N + P) * 2 * M * max(0, L + A - k1c)   # t = 0 first layers: action columns only
        macs += 2 * M * max(0, L + A - k1c)                  # z0c: once per env
    else:
        macs = P * H * (pi + d + R) + I * T * (H * (d + R) + pi + 2 * Q) + enc
    return 2.0 * macs


def synthetic_obs(cfg, B, seed=0):
    rs = np.random.RandomState(seed)
    if cfg.modality == "pixels":
        return rs.randint(0, 256, size=(B,) + tuple(cfg.obs_shape)).astype(np.uint8)
    return rs.standard_normal((B,) + tuple(cfg.obs_shape)).astype(np.float32)


def _core_id(c: int) -> str:
    try:
        with open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list") as f:
            return f.read().strip()
    except OSError:
        return str(c)


def physical_cores() -> int:
    """Physical cores this process may run on: the affinity mask's CPUs, counting SMT siblings once."""
    cpus = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else list(range(os.cpu_count() or 1))
    return max(1, len({_core_id(c) for c in cpus}))


def cpu_quota():
    """CPUs' worth of time the cgroup grants this process (cpu.max / cfs quota), None when unlimited."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return None if q <= 0 else q / per
    except (OSError, ValueError):
        return None


def numa_cores():
    """{node: [one CPU per physical core]} over the CPUs this process may use (node order, SMT siblings once)."""
    allowed = set(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else set(range(os.cpu_count() or 1))
    nodes = {}
    base = "/sys/devices/system/node"
    try:
        names = sorted((d for d in os.listdir(base) if d.startswith("node") and d[4:].isdigit()), key=lambda d: int(d[4:]))
    except OSError:
        names = []
    for d in names:
        cpus = []
        for part in open(f"{base}/{d}/cpulist").read().strip().split(","):
            if part:
                lo, _, hi = part.partition("-")
                cpus += range(int(lo), int(hi or lo) + 1)
        seen, pick = set(), []
        for c in cpus:
            if c in allowed and _core_id(c) not in seen:
                seen.add(_core_id(c))
                pick.append(c)
        if pick:
            nodes[int(d[4:])] = pick
    return nodes or {0: sorted(allowed)}


def cpu_baseline(cfg, budget_s: float, threads: int):
    """Time the oracle (CPU restatement of the reference plan(), bit-exact to the reference's golden vectors)
    on this host with `threads` torch threads: 2 warm-up calls, then calls until `budget_s` seconds of CPU work
    (>= 3 calls), median."""
    from oracle import tdmpc_ref
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    told = tdmpc_ref.RefTOLD(synthetic_state_dict(cfg, 0), cfg)
    st = tdmpc_ref.PlanState(0.05)
    obs = synthetic_obs(cfg, 1)[0]
    step = 10**6
    times = []
    for i in range(2 + 400):
        nb = tdmpc_ref.draw_noise(cfg, step, False)
        t = time.perf_counter()
        tdmpc_ref.plan(told, cfg, st, obs, nb, eval_mode=False, step=step, t0=(i == 0))
        dt = time.perf_counter() - t
        if i >= 2:
            times.append(dt)
        if len(times) >= 3 and sum(times) > budget_s:
            break
    torch.set_num_threads(prev)
    med = float(np.median(times))
    cpu_model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": round(1.0 / med, 3), "unit": "plan-steps/s", "cores": threads, "kind": "port",
            "sample": f"{len(times)} plan() calls ({sum(times):.1f} s) of {cfg.task} N={cfg.num_samples} "
                      f"H={cfg.horizon} I={cfg.iterations} L={cfg.latent_dim} after 2 warm-up, median; "
                      f"torch CPU fp32, {threads} threads, {cpu_model}"}


def cpu_baselines(cfg, budget_s: float):
    """The oracle at 1 thread and on one NUMA node (the reference's CPU path on the host cores of the
    same box). The node leg pins the process to one physical core per thread of NUMA node 0 (no SMT sibling, no
    cross-socket traffic) with as many threads as the cgroup's CPU quota allows. The headline cpu_baseline is the
    fastest leg (the CPU's best showing); all are reported.

    Why not every core: the GPU box's cgroup grants this process ~16 CPUs of time (cpu.max) while its affinity mask
    spans both sockets' 128 cores. Round 2 ran 128 unpinned threads and got 1.18 plan-steps/s against 10.1 at 16:
    torch's intra-op threads were time-sliced by the quota (each parallel region waits for its slowest, throttled
    thread) and spread over two sockets. Threads beyond the quota buy nothing."""
    quota = cpu_quota()
    nodes = numa_cores()
    node0 = nodes[min(nodes)]
    n_node = len(node0) if quota is None else max(1, min(len(node0), int(quota)))
    keep = os.sched_getaffinity(0) if hasattr(os, "sched_setaffinity") else None
    runs = {}
    try:
        for n in sorted({1, n_node}):
            if keep is not None:
                os.sched_setaffinity(0, node0[:n])
            r = cpu_baseline(cfg, budget_s if n > 1 else 2 * budget_s, n)
            r["sample"] += f"; pinned to {n} physical core(s) of NUMA node {min(nodes)}"
            runs[str(n)] = r
    finally:
        if keep is not None:
            os.sched_setaffinity(0, keep)
    best = max(runs.values(), key=lambda r: r["value"])
    out = dict(best)
    out["physical_cores"] = physical_cores()
    out["numa_nodes"] = {str(k): len(v) for k, v in nodes.items()}
    out["cgroup_cpu_quota"] = quota
    out["by_threads"] = {k: {"value": v["value"], "sample": v["sample"]} for k, v in runs.items()}
    return out


def cpu_node_leg(cfg, budget_s: float):
    """The oracle for one config on NUMA node 0's physical cores, as many threads as the cgroup quota grants (the
    faster of cpu_baselines' two legs at every config measured so far)."""
    quota = cpu_quota()
    nodes = numa_cores()
    node0 = nodes[min(nodes)]
    n = len(node0) if quota is None else max(1, min(len(node0), int(quota)))
    keep = os.sched_getaffinity(0) if hasattr(os, "sched_setaffinity") else None
    try:
        if keep is not None:
            os.sched_setaffinity(0, node0[:n])
        r = cpu_baseline(cfg, budget_s, n)
    finally:
        if keep is not None:
            os.sched_setaffinity(0, keep)
    r["sample"] += f"; pinned to {n} physical core(s) of NUMA node {min(nodes)}"
    return r


def config_leg(name, B, args, dev, graph, cpu):
    """One more BASELINE.json config timed in the same run: B envs per plan_batch call on this GPU (graph replay,
    device RNG), the dominant step kernel's roofline and helper.q's rate from HIP events, and the oracle on this
    host's cores as its own cpu_baseline."""
    oc = bench_cfg(name)
    oc.device = str(dev)
    ao = make_agent(oc, B, args.rng, graph, 3)
    oo = torch.from_numpy(synthetic_obs(oc, B, seed=0)).to(dev)
    step = 10**6
    ko = max(20, args.steps // 2)

    def fn(i):
        return ao.plan_batch(oo, step=step, t0=(i % 100 == 0), sync_metrics=False)

    elo = time_steps(fn, 3, ko, None)
    ao.planner.check_status()
    fo = min(plan_flops(oc, False), plan_flops(oc, True))
    value = B * ko / elo
    out = {"value": round(value, 3), "unit": "plan-steps/s", "ms_per_step": round(elo / ko * 1e3, 4),
           "envs_per_gpu": B, "steps": ko,
           "workload": f"{name}: TDMPC.plan N={oc.num_samples} H={oc.horizon} iters={oc.iterations} "
                       f"K={oc.num_elites} L={oc.latent_dim} A={oc.action_dim} modality={oc.modality}, {B} envs per call",
           "frac_of_fp32_peak": round(value * fo / 1e12 / FP32_PEAK_TFLOPS, 4),
           "frac_of_x6_peak": round(value * fo / 1e12 / X6_PEAK_TFLOPS, 4)}
    if not args.no_roofline:
        out["roofline"] = step_roofline(oc, B, ao, fn, 3, dev, f"{name}/B{B}")
        out["roofline"]["q_head"] = q_roofline(oc, B, ao, fn, 3)
    del ao
    if cpu:
        c = cpu_node_leg(oc, args.cpu_budget_config)
        out["cpu_baseline"] = c
        out["speedup_vs_cpu"] = round(value / c["value"], 2)
    return out


def sampleable(rs, total, n, L=500, H=5):
    """n random storage indices outside the masked last H steps of each episode (helper.py:468-470): the
    positions a learner's priority write-back can touch, so every sampled window stays inside its episode."""
    r = rs.randint(0, total // L * (L - H), n)
    return (r // (L - H)) * L + r % (L - H)


def replay_bench(cfg, dev, cpu=True, reps=200):
    """one prioritized-replay sample() (batch 512, H+1 = 6-step windows) from a buffer of the
    task's capacity (train_steps 500000 / action_repeat 2 = 250k transitions, 500-step episodes), random
    priorities, on the device (tdmpc_amd.replay) -- with replacement (buffer not yet full, the common case) and
    without (full). CPU baseline: the oracle's restatement of the reference sample() (torch CPU + numpy choice,
    1 process) on the same buffer contents."""
    from types import SimpleNamespace
    from tdmpc_amd.replay import ReplayBuffer
    L, cap, B, H = 500, 250_000, 512, 5
    obs_dim, A = cfg.obs_shape[0], cfg.action_dim
    rc = SimpleNamespace(device=str(dev), modality="state", obs_shape=(obs_dim,), action_dim=A, episode_length=L,
                         train_steps=cap, max_buffer_size=10**6, batch_size=B, horizon=H, env_horizon=H,
                         per_alpha=0.6, per_beta=0.4, frame_stack=1)
    rs = np.random.RandomState(0)
    ep = SimpleNamespace(obs=torch.from_numpy(rs.standard_normal((L + 1, obs_dim)).astype(np.float32)),
                         action=torch.from_numpy(rs.uniform(-1, 1, (L, A)).astype(np.float32)),
                         reward=torch.from_numpy(rs.standard_normal(L).astype(np.float32)))
    out = {"config": f"capacity {cap}, batch {B}, window H+1={H + 1}, obs {obs_dim}, A {A}, alpha 0.6, beta 0.4"}
    for full in (False, True):
        buf = ReplayBuffer(rc, latent_plan=True)
        for _ in range(cap // L if full else cap // L - 1):
            buf.add(ep)
        total = cap if full else buf.idx
        buf.update_priorities(torch.from_numpy(sampleable(rs, total, 50_000)),
                              torch.from_numpy(rs.exponential(1.0, (50_000, 1)).astype(np.float32)))
        for _ in range(5):
            buf.sample()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(reps):
            buf.sample()
        torch.cuda.synchronize()
        dt_eager = (time.perf_counter() - t) / reps
        # as the learner runs it: captured in its HIP graph (device time, no per-call host launch cost)
        g = torch.cuda.CUDAGraph()
        per = 20
        with torch.cuda.graph(g):
            for _ in range(per):
                buf.sample()
        g.replay()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(reps // per):
            g.replay()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / (reps // per * per)
        key = "without_replacement" if full else "with_replacement"
        if not full:
            # update_priorities at the learner's write-back size and at 50k (helper.py:487-488; duplicates: last wins)
            upd = {}
            for n in (B, 50_000):
                ui = torch.from_numpy(sampleable(rs, total, n)).to(dev)
                uv = torch.from_numpy(rs.exponential(1.0, (n, 1)).astype(np.float32)).to(dev)
                for _ in range(3):
                    buf.update_priorities(ui, uv)
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                for _ in range(reps):
                    buf.update_priorities(ui, uv)
                torch.cuda.synchronize()
                upd[str(n)] = round((time.perf_counter() - t1) / reps * 1e6, 2)
            out["update_priorities_us"] = upd
        # algorithmic HBM bytes: priorities read, p**alpha write + read, probs write, float64 cdf write, window gather
        alg = total * (4 + 8 + 4 + 8) + B * (H + 2) * (obs_dim + A + 1) * 4
        out[key] = {"value": round(1.0 / dt, 1), "unit": "samples/s", "us_per_sample": round(dt * 1e6, 2),
                    "us_per_sample_eager": round(dt_eager * 1e6, 2),
                    "note": "sample() (device uniforms included) replayed from a HIP graph of 20 samples, as the "
                            "learner's captured update runs it; eager = one Python call per sample",
                    "total": total, "hbm_gbs_algorithmic": round(alg / dt / 1e9, 1)}
        if cpu:
            from oracle.replay_ref import RefReplay
            ref = RefReplay(SimpleNamespace(modality="state", obs_shape=(obs_dim,), action_dim=A, episode_length=L,
                                            capacity=cap, batch_size=B, horizon=H, per_alpha=0.6, per_beta=0.4))
            ref._obs = buf._obs.cpu()
            ref._last_obs = buf._last_obs.cpu()
            ref._action, ref._reward = buf._action.cpu(), buf._reward.cpu()
            ref._priorities, ref._full, ref.idx = buf._priorities.cpu(), full, buf.idx
            n, t0 = 0, time.perf_counter()
            while n < 5 or time.perf_counter() - t0 < 3.0:
                ref.sample(np.random.random_sample(4 * B))
                n += 1
            cdt = (time.perf_counter() - t0) / n
            out[key]["cpu_baseline"] = {"value": round(1.0 / cdt, 2), "unit": "samples/s", "kind": "port",
                                        "cores": torch.get_num_threads(),
                                        "sample": f"{n} oracle sample() calls (torch CPU + numpy choice)"}
            out[key]["speedup_vs_cpu"] = round(cdt / dt, 1)
    return out


def learner_bench(cfg, dev, cpu=True, reps=30, pixels=True, modes=("graph", "eager", "hipblaslt")):
    """TDMPC.update (batch 512, horizon 5, the task's TOLD) fed by the device replay buffer
    (50k transitions): HIP-graph replay of the whole update vs the same update issued eagerly (the reference's
    execution model on a GPU), and the oracle restatement of the reference update on the host CPU."""
    from types import SimpleNamespace
    from tdmpc_amd.replay import ReplayBuffer
    lcfg = bench_cfg(args_config_for_learner(cfg), batch_size=512)
    lcfg.device = str(dev)
    L = 500
    rc = SimpleNamespace(**{**vars(lcfg), "train_steps": 50_000, "max_buffer_size": 10**6, "episode_length": L,
                            "env_horizon": lcfg.horizon})
    rs = np.random.RandomState(0)
    O, A = lcfg.obs_shape[0], lcfg.action_dim
    ep = SimpleNamespace(obs=torch.from_numpy(rs.standard_normal((L + 1, O)).astype(np.float32)),
                         action=torch.from_numpy(rs.uniform(-1, 1, (L, A)).astype(np.float32)),
                         reward=torch.from_numpy(rs.standard_normal(L).astype(np.float32)))
    out = {"config": f"{lcfg.task}: batch {lcfg.batch_size}, horizon {lcfg.horizon}, latent {lcfg.latent_dim}, "
                     f"mlp {lcfg.mlp_dim}, replay 50k transitions"}
    for mode, warm in (("graph", 3), ("eager", 10**9), ("hipblaslt", 3)):
        if mode not in modes:
            continue
        agent = TDMPC(lcfg)
        agent.model.load_state_dict(synthetic_state_dict(lcfg, 0))
        agent.model_target.load_state_dict(synthetic_state_dict(lcfg, 1))
        lrn = agent.learner(graph=True, warmup=warm)
        if mode == "hipblaslt" and lrn.engine is not None:
            lrn.engine.blas = True    # the heads' products on hipBLASLt (the default: tdmpc_lg_gemm's macro tiles)
        buf = ReplayBuffer(rc, latent_plan=True)
        for _ in range(50_000 // L - 1):
            buf.add(ep)
        for i in range(5):
            agent.update(buf, i + 1, sync_metrics=False)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for i in range(reps):
            agent.update(buf, 6 + i, sync_metrics=False)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / reps
        out[mode] = {"value": round(1.0 / dt, 1), "unit": "updates/s", "ms_per_update": round(dt * 1e3, 3)}
        if mode == "hipblaslt":
            out[mode]["note"] = ("the same graph-replayed update with the heads' products on hipBLASLt (torch.mm + "
                                 "an activation launch, TDMPC_LG_BLAS=1) instead of tdmpc_lg_gemm's macro tiles")
    if "eager" in out and "graph" in out:
        out["graph_speedup_vs_eager"] = round(out["eager"]["ms_per_update"] / out["graph"]["ms_per_update"], 2)
    if pixels:
        out["pixels"] = pixel_learner_bench(dev)
    if cpu:
        from oracle.learner_ref import RefLearner
        ref = RefLearner(lcfg, synthetic_state_dict(lcfg, 0), synthetic_state_dict(lcfg, 1))
        b = tuple(x.cpu() for x in buf.sample())
        n, t0 = 0, time.perf_counter()
        while n < 2 or time.perf_counter() - t0 < 5.0:
            ref.update(b, n + 1)
            n += 1
        cdt = (time.perf_counter() - t0) / n
        out["cpu_baseline"] = {"value": round(1.0 / cdt, 2), "unit": "updates/s", "kind": "port",
                               "cores": torch.get_num_threads(),
                               "sample": f"{n} oracle update() calls (reference math on torch CPU)"}
        out["speedup_vs_cpu"] = round(cdt / out["graph"]["ms_per_update"] * 1e3, 1)
    return out


class _FixedBatch:
    """A replay stand-in that hands out one device batch (graph-safe: the same tensors every call)."""
    graph_safe, idx, _full = True, 0, False

    def __init__(self, b):
        self.b = b
        self.prio = torch.zeros(b[0].shape[0], 1, device=b[0].device)

    def sample(self):
        return self.b

    def update_priorities(self, idxs, p):
        self.prio.copy_(p)


def pixel_learner_bench(dev, reps=10, modes=None):
    """The pixel learner (quadruped-run pixels: 9 x 84 x 84 frame stacks, conv encoder, batch 512, horizon 5;
    tdmpc.py:192-245 with RandomShiftsAug and the conv stack, helper.py:119-133, 250-283) on the learner engine
    (learner_conv.hip's conv kernels, HIP-graph replay) against the same update through autograd (PyTorch conv =
    MIOpen), one fixed device batch."""
    cfg = bench_cfg("quadruped-run-pixels", batch_size=512)
    cfg.device = str(dev)
    B, H, A = cfg.batch_size, cfg.horizon, cfg.action_dim
    shape = tuple(cfg.obs_shape)
    g = torch.Generator(device=dev).manual_seed(0)
    b = (torch.randint(0, 256, (B,) + shape, generator=g, device=dev).float(),
         torch.randint(0, 256, (H + 1, B) + shape, generator=g, device=dev).float(),
         torch.rand(H + 1, B, A, generator=g, device=dev) * 2 - 1, torch.randn(H + 1, B, 1, generator=g, device=dev),
         torch.arange(B, device=dev), torch.ones(B, device=dev))
    out = {"config": f"{cfg.task} pixels: batch {B}, horizon {H}, frames {shape}, latent {cfg.latent_dim}"}
    for mode, engine in (("engine_graph", "1"), ("autograd_miopen", "0")):
        if modes is not None and mode.split("_")[0] not in modes:
            continue
        os.environ["TDMPC_LEARNER_ENGINE"] = engine
        try:
            agent = TDMPC(cfg)
            agent.model.load_state_dict(synthetic_state_dict(cfg, 0))
            agent.model_target.load_state_dict(synthetic_state_dict(cfg, 1))
            agent.learner(graph=engine == "1", warmup=3)
            buf = _FixedBatch(b)
            for i in range(5):
                agent.update(buf, i + 1, sync_metrics=False)
            torch.cuda.synchronize()
            t = time.perf_counter()
            for i in range(reps):
                agent.update(buf, 6 + i, sync_metrics=False)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t) / reps
            out[mode] = {"value": round(1.0 / dt, 2), "unit": "updates/s", "ms_per_update": round(dt * 1e3, 3)}
            del agent
        finally:
            os.environ.pop("TDMPC_LEARNER_ENGINE", None)
    if "autograd_miopen" in out and "engine_graph" in out:
        out["engine_speedup_vs_autograd"] = round(out["autograd_miopen"]["ms_per_update"] /
                                                  out["engine_graph"]["ms_per_update"], 2)
    return out


def train_loop_bench(cfg, dev, reps=40):
    """The training loop's per-env-step GPU work (src/train.py:94-108 after the seed steps): one agent.plan(obs,
    step, t0) exactly as train.py calls it (TDMPC(cfg) defaults, host numpy obs, metrics synced to the host), then
    one agent.update(buffer, step) (batch 512 from a 50k-transition device replay buffer, HIP-graph replay; the
    update repacks the planner's weights from the learner's flat buffer inside that graph). Also each half alone,
    in the same process, in 4 interleaved rounds (medians): the loop's overhead over plan + update is what the
    hand-over between them costs."""
    from types import SimpleNamespace
    from tdmpc_amd.replay import ReplayBuffer
    lcfg = bench_cfg(args_config_for_learner(cfg), batch_size=512)
    lcfg.device = str(dev)
    L = 500
    rc = SimpleNamespace(**{**vars(lcfg), "train_steps": 50_000, "max_buffer_size": 10**6, "episode_length": L,
                            "env_horizon": lcfg.horizon})
    rs = np.random.RandomState(0)
    O, A = lcfg.obs_shape[0], lcfg.action_dim
    ep = SimpleNamespace(obs=torch.from_numpy(rs.standard_normal((L + 1, O)).astype(np.float32)),
                         action=torch.from_numpy(rs.uniform(-1, 1, (L, A)).astype(np.float32)),
                         reward=torch.from_numpy(rs.standard_normal(L).astype(np.float32)))
    agent = TDMPC(lcfg)
    agent.model.load_state_dict(synthetic_state_dict(lcfg, 0))
    agent.model_target.load_state_dict(synthetic_state_dict(lcfg, 1))
    agent.std = 0.05
    buf = ReplayBuffer(rc, latent_plan=True)
    for _ in range(50_000 // L - 1):
        buf.add(ep)
    obs = synthetic_obs(lcfg, 1, seed=0)[0]
    step = 10**6

    def plan(i):
        agent.plan(obs, step=step + i, t0=(i == 0))

    def update(i):
        agent.update(buf, step + i)

    def loop(i):
        plan(i)
        update(i)

    out = {"config": f"{lcfg.task}: plan N={lcfg.num_samples} H={lcfg.horizon} iters={lcfg.iterations} (1 env, "
                     f"train.py's call) + update batch {lcfg.batch_size} (replay 50k transitions)"}
    for i in range(8):   # warm-up: both graphs captured, the planner packed from the learner's buffer
        loop(i)
    torch.cuda.synchronize()
    # interleaved rounds (loop, plan alone, update alone), the median of each: a box's drift over the measurement
    # lands on all three alike
    samples = {"loop": [], "plan": [], "update": []}
    for r in range(4):
        for name, fn in (("loop", loop), ("plan", plan), ("update", update)):
            t = time.perf_counter()
            for i in range(reps // 4):
                fn(100 + 10 * reps * r + i)
            torch.cuda.synchronize()
            samples[name].append((time.perf_counter() - t) / (reps // 4) * 1e3)
    res = {k: float(np.median(v)) for k, v in samples.items()}
    loop_ms = res["loop"]
    out["ms_per_env_step"] = round(loop_ms, 4)
    out["value"] = round(1e3 / loop_ms, 2)
    out["unit"] = "env-steps/s"
    out["plan_ms"] = round(res["plan"], 4)
    out["update_ms"] = round(res["update"], 4)
    out["overhead_us"] = round((loop_ms - res["plan"] - res["update"]) * 1e3, 1)
    out["live_repack"] = bool(getattr(agent._learner, "_live_pack", False)) if hasattr(agent, "_learner") else None
    return out


def icem_bench(cfg, dev, cpu=True, steps=20):
    """the iCEM planner (TdICemSimMlp.plan) on the same task and N / H / iterations / K as the
    headline, iCEM defaults (N shrinking by 1.25 per iteration, 25 % of the elites reused, coloured noise), one
    env per call (the drop-in path), vs the oracle restatement of the reference planner on the host CPU."""
    from tdmpc_amd.icem import TdICEM
    icfg = bench_cfg(args_config_for_learner(cfg))
    icfg.device = str(dev)
    obs = synthetic_obs(icfg, 1)[0]
    step = 10**6

    def timed(rng):
        agent = TdICEM(icfg, rng=rng)
        agent.model.load_state_dict(synthetic_state_dict(icfg, 0, enc_norm=True))
        agent.std = 0.05
        for i in range(3):
            agent.plan(obs, step=step, t0=(i == 0))
        torch.cuda.synchronize()
        t = time.perf_counter()
        for i in range(steps):
            agent.plan(obs, step=step, t0=False)
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / steps, agent

    dt, agent = timed("device")
    dt_ref, _ = timed("reference")
    # vectorised: 32 envs per call (TdICEM.plan_batch), the chain kernels' regime
    Bv = 32
    ab = TdICEM(icfg, max_batch=Bv, rng="device")
    ab.model.load_state_dict(synthetic_state_dict(icfg, 0, enc_norm=True))
    ab.std = 0.05
    ob = torch.from_numpy(synthetic_obs(icfg, Bv, seed=0))
    for i in range(3):
        ab.plan_batch(ob, step=step, t0=(i == 0), sync_metrics=False)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for i in range(steps):
        ab.plan_batch(ob, step=step, t0=False, sync_metrics=False)
    torch.cuda.synchronize()
    dtb = (time.perf_counter() - t) / steps
    out = {"config": f"{icfg.task}: N={icfg.num_samples} (x1/{icfg.factor_decrease_num} per iteration) H={icfg.horizon} "
                     f"iters={icfg.iterations} K={icfg.num_elites} reuse={agent.E_max} elites, 1 env per call, "
                     "all noise drawn on the device (rng='device', inside the timed call)",
           "value": round(1.0 / dt, 2), "unit": "plan-steps/s", "ms_per_step": round(dt * 1e3, 3),
           "reference_rng": {"value": round(1.0 / dt_ref, 2), "ms_per_step": round(dt_ref * 1e3, 3),
                             "note": "noise drawn in the reference's order on torch's / numpy's global "
                                     "generators (host numpy coloured noise included)"},
           "batch32": {"value": round(Bv / dtb, 2), "unit": "plan-steps/s", "ms_per_step": round(dtb * 1e3, 3),
                       "note": "TdICEM.plan_batch, 32 envs per call, device RNG"}}
    if cpu:
        from oracle import icem_ref
        from oracle.tdmpc_ref import RefTOLD
        told = RefTOLD(synthetic_state_dict(icfg, 0, enc_norm=True), icfg)
        st = icem_ref.IcemState(0.05)
        times = []
        for i in range(40):
            nz = icem_ref.draw_icem_noise(icfg, st, step, i == 0, False)
            t0 = time.perf_counter()
            icem_ref.plan(told, icfg, st, obs, nz, eval_mode=False, step=step, t0=(i == 0))
            times.append(time.perf_counter() - t0)
            if i >= 3 and sum(times[2:]) > 6.0:
                break
        med = float(np.median(times[2:]))
        out["cpu_baseline"] = {"value": round(1.0 / med, 2), "unit": "plan-steps/s", "kind": "port",
                               "cores": torch.get_num_threads(),
                               "sample": f"{len(times) - 2} oracle iCEM plan() calls after 2 warm-up, median"}
        out["speedup_vs_cpu"] = round(med / dt, 1)
    return out


def args_config_for_learner(cfg):
    return {"humanoid": "humanoid-run", "cheetah": "cheetah-run", "dog": "dog-run",
            "cartpole": "cartpole-swingup"}.get(cfg.task, "humanoid-run")


def make_agent(cfg, B, rng, graph, seed, path="auto"):
    torch.manual_seed(seed)
    agent = TDMPC(cfg, max_batch=B, rng=rng, graph=graph, path=path)
    agent.model.load_state_dict(synthetic_state_dict(cfg, 0))
    agent.std = 0.05   # trained-regime value of std_schedule
    return agent


def step_roofline(cfg, B, agent, one_step, n_r, dev, pmc_prefix):
    """Roofline of the dominant kernel (the CEM rollout step, TOLD.next: 5 of every iteration's launches): HIP events
    around each t >= 1 step launch (t = 0 runs a reduced first layer, z0c_kernel, and is not timed) on the stream it
    is launched on, over an eager replay of `n_r` plan calls; FLOPs counted by the library per launch. PMC traffic /
    MFMA busy from profiles/pmc_*.json when a pass of the same kernel and shape was committed."""
    L = _lib.lib()
    graph = agent.graph
    agent.graph = False
    one_step(0)
    torch.cuda.synchronize()

    def timed(cfg_id, pro, kdim, rows):
        _lib.check(L.tdmpc_profile_begin(cfg_id, pro, kdim, rows, 8192), "profile_begin")
        for i in range(n_r):
            one_step(1 + i)
        n, ms, fl = C.c_int32(), C.c_double(), C.c_double()
        _lib.check(L.tdmpc_profile_end(C.byref(n), C.byref(ms), C.byref(fl)), "profile_end")
        return n.value, ms.value, fl.value

    rows = B * cfg.num_samples
    M, Lt, A = cfg.mlp_dim, cfg.latent_dim, cfg.action_dim
    n, ms, fl = timed(4, -1, 0, rows)
    peak = FP32_PEAK_TFLOPS
    if n > 0:
        name = L.tdmpc_profile_kernel().decode()   # the library names the kernel it launched
        wide = name.startswith("wide_step_kernel")
        x6 = wide or name.endswith(", x6>")
        rb = 16 if name.startswith("chain16") else 32
        if wide:
            peak = X6_PEAK_TFLOPS
            fold = ("; latent 512: x streamed through the ring (XS), the first layer folded to [W1a | W1z W3] on "
                    "h2 of the previous step and h2 stored instead of z' (OUTH: no layer 3; FLOPs counted as executed)"
                    if "OUTH" in name else "")
            kernel = (f"{name} (TOLD.next: dynamics + reward heads on 128-row "
                      f"workgroups, 8 waves x 16 rows x all {M} hidden columns in registers, layer 1 streamed into "
                      f"layer 2 by 64-column chunks, x6 weight fragments LDS-DMA'd once per workgroup into an LDS ring; "
                      f"{rows} rows x 2 heads per launch{fold}), fp32 products from a three-way bf16 split of both "
                      f"operands: 6 v_mfma_f32_16x16x32_bf16 per product, fp32 accumulation (peak = dense BF16 / 6)")
        elif x6:
            peak = X6_PEAK_TFLOPS
            kernel = (f"{name} (TOLD.next: dynamics + reward heads, {rb}-row blocks, hidden activations in LDS, weights streamed from L2; {rows} rows x 2 "
                      f"heads per launch), fp32 products from a three-way bf16 split of both operands: 6 "
                      f"{'v_mfma_f32_32x32x16_bf16' if rb == 32 else 'v_mfma_f32_16x16x32_bf16'} per product, fp32 "
                      f"accumulation (peak = dense BF16 / 6)")
        else:
            kernel = (f"{name} (TOLD.next: dynamics + reward heads, "
                      f"{rb}-row blocks, hidden activations in LDS, weights streamed from L2; {rows} rows x 2 heads per "
                      f"launch), fp32 {'v_mfma_f32_32x32x2_f32' if rb == 32 else 'v_mfma_f32_16x16x4_f32'}")
        kx = A + Lt
        alg_bytes = 4.0 * (rows * (kx + Lt + 2) + 2 * M * kx + 2 * M * M + M * Lt + M)
        pmc_key = f"{pmc_prefix}/" + ("wide_step" if wide else "chain_step" + ("_x6" if x6 else ""))
    else:
        n, ms, fl = timed(0, 0, M, rows)
        kernel = (f"linear_lds_kernel (128x128 LDS-staged tile): CEM rollout layer 2 (dynamics + reward "
                  f"hidden {M}x{M} Linear + ELU, {rows} rows x 2 problems), fp32 v_mfma_f32_32x32x2_f32")
        alg_bytes = 4.0 * (rows * 2 * M + 2 * M * M + rows * M)
        pmc_key = pmc_prefix
    agent.graph = graph
    avg_s = ms / max(n, 1) * 1e-3
    per_launch = fl / max(n, 1)
    achieved = per_launch / avg_s / 1e12
    roof = {"bound": "mfma", "achieved": round(achieved, 3), "peak": peak, "unit": "TFLOP/s",
            "frac": round(achieved / peak, 4), "frac_of_fp32_mfma_peak": round(achieved / FP32_PEAK_TFLOPS, 4),
            "traffic": None, "kernel": kernel,
            "launches": n, "avg_launch_us": round(avg_s * 1e6, 3), "flops_per_launch": per_launch,
            "algorithmic_bytes_per_launch": alg_bytes,
            "hbm_gbs_algorithmic": round(alg_bytes / avg_s / 1e9, 1)}
    mf = os.path.join(REPO, "profiles", "pmc_mfma.json")
    if os.path.exists(mf):
        try:
            t = json.load(open(mf)).get(pmc_key)
            if t:   # rocprofv3 PMC pass of the same kernel and shape (tools/gpu/suite.sh pmc, tools/pmc_mfma.py)
                roof["mfma_util_pmc"] = t.get("mfma_util")
                roof["clock_ghz_pmc"] = t.get("clock_ghz")
        except (OSError, ValueError):
            pass
    pmc = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc):
        try:
            t = json.load(open(pmc)).get(pmc_key)
            if t:
                roof["traffic"] = t.get("hbm_bytes_per_launch")
                roof["traffic_source"] = t.get("source")
        except (OSError, ValueError):
            pass
    # the HBM roofline the north star asks for, next to the binding MFMA one: algorithmic and PMC bytes per launch
    # over the measured launch time, as fractions of the 8 TB/s peak
    roof["hbm_frac_algorithmic"] = round(roof["hbm_gbs_algorithmic"] / HBM_PEAK_GBS, 4)
    if roof["traffic"]:
        roof["hbm_gbs_pmc"] = round(roof["traffic"] / avg_s / 1e9, 1)
        roof["hbm_frac_pmc"] = round(roof["hbm_gbs_pmc"] / HBM_PEAK_GBS, 4)
    if n > 0 and wide and "OUTH" in kernel:
        # the folded rollout runs no layer 3 between steps: the reference's FLOPs of the same TOLD.next (layer 3
        # included) over the same time, next to the executed-FLOP fraction above
        per_row_exec = 2.0 * (2 * ((Lt + A) * M + M * M) + M)
        roof["frac_algorithmic"] = round(achieved * (per_row_exec + 2.0 * M * Lt) / per_row_exec / peak, 4)
    if n > 0 and wide:
        # the wide kernel's weight stream: each workgroup fills its head's x6 weight fragments (3 KiB
        # each, 8 per step) from L2 into LDS once per launch -- 4 super-chunks x (G1 + 16) steps per head + 2 NB3
        # layer-3 steps of the dynamics head -- against the LDS-DMA rate measured with nothing else running
        # (tools/mb/dma_ring.hip: the kernel's own ring, 16.4-16.7 TB/s over the chip, profiles/r05/dma_ring_probe_*.txt)
        # (latent 512: mode XS streams each first-layer step's x beside the weights, 16 KiB per workgroup and step;
        # OUTH stores h2 for the folded first layer and runs no layer 3)
        fields = [v.strip() for v in name[name.index("<") + 1:name.index(">")].split(",")]
        g1, nb3 = int(fields[0]), int(fields[1])
        mode = fields[2] if len(fields) > 2 else ""
        nrb = -(-rows // 128)
        tail = 0 if "OUTH" in mode else (2 * nb3 if nb3 <= 8 else 16 * (nb3 // 8))
        fill = float(nrb * (4 * (g1 + 16) * 2 + tail) * 8 * 3072)
        if "XS" in mode:
            fill += float(nrb * 2 * 4 * g1 * 8 * 2048)
        tbs = fill / avg_s / 1e12
        roof["weight_stream"] = {
            "bytes_per_launch": fill, "achieved_tbs": round(tbs, 3), "ceiling_tbs": LDSDMA_CEILING_TBS,
            "frac": round(tbs / LDSDMA_CEILING_TBS, 4),
            "note": "L2 -> LDS x6 weight fills of all workgroups per launch. The probe with the kernel's ring: the "
                    "stream alone 0.38 us per step, its 48 MFMAs per wave alone 0.71, both 1.12 -- they do not "
                    "overlap (profiles/r05/dma_ring_probe_isolation.txt)"}
    return roof


def q_roofline(cfg, B, agent, one_step, n_r, cfg_id=6, rows=0):
    """The terminal heads (tdmpc.py:91-92): cfg_id 6 = helper.q (both Q heads, tdmpc.py:47-50) -- on the wide heads
    kernel the sampled rows' Q1 + Q2 launch, else the chain launch over the N + P rows of every env; cfg_id 5 with
    rows = B N = the wide heads kernel's mixed launch (the sampled rows' TOLD.pi beside the policy rows' Q1 + Q2).
    HIP events around the launches (library profiler), FLOPs counted by the library."""
    L = _lib.lib()
    graph = agent.graph
    agent.graph = False
    _lib.check(L.tdmpc_profile_begin(cfg_id, -1, 0, rows, 8192), "profile_begin")
    for i in range(n_r):
        one_step(1 + i)
    n, ms, fl = C.c_int32(), C.c_double(), C.c_double()
    _lib.check(L.tdmpc_profile_end(C.byref(n), C.byref(ms), C.byref(fl)), "profile_end")
    agent.graph = graph
    if n.value == 0:
        return None
    avg_s = ms.value / n.value * 1e-3
    per = fl.value / n.value
    return {"kernel": L.tdmpc_profile_kernel().decode(), "launches": n.value, "avg_launch_us": round(avg_s * 1e6, 3),
            "flops_per_launch": per, "achieved": round(per / avg_s / 1e12, 3),
            "frac_of_x6_peak": round(per / avg_s / 1e12 / X6_PEAK_TFLOPS, 4)}


def _sync():
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def time_steps(step_fn, warmup, steps, dist):
    """W untimed steps, then exactly `steps` timed ones bracketed by a barrier + device sync on both sides."""
    for i in range(warmup):
        step_fn(i)
    _sync()
    if dist is not None:
        dist.barrier()
    _sync()
    t0 = time.perf_counter()
    for i in range(steps):
        step_fn(warmup + i)
    _sync()
    if dist is not None:
        dist.barrier()
    _sync()
    return time.perf_counter() - t0


def job_rate(elapsed, units_per_rank, dist, device):
    """Whole-job throughput: the slowest rank's time (MAX over ranks) and every rank's units over it."""
    world = 1
    if dist is not None:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        world = dist.get_world_size()
    return elapsed, world * units_per_rank / elapsed


def summary_line(out, cfg):
    """A compact record of every leg (the driver keeps only the tail of the JSON line): per config its plan-steps/s,
    the dominant step kernel's fraction of its roof and helper.q's; then the single env, the learner, iCEM and the
    CPU speedup. Keys name the latent explicitly: BASELINE.json configs[2] says latent 512, the reference's
    cfgs/tasks/humanoid.yaml:6 says 100 -- both are measured."""
    def leg(v, roof):
        if v is None:
            return None
        r = roof or {}
        q = r.get("q_head") or {}
        return [round(v, 1), r.get("frac"), q.get("frac_of_x6_peak"), (r.get("kernel") or "").split(" (")[0]]
    s = {f"{out['config']['workload'].split(':')[0]} L{cfg.latent_dim} B{out['config']['envs_per_gpu']}":
         leg(out["value"], out.get("roofline"))}
    for k, v in (out.get("configs") or {}).items():
        s[k] = leg(v.get("value"), v.get("roofline"))
    s["_fields"] = "[plan-steps/s, step-kernel frac of x6 roof, helper.q frac, step kernel]"
    se = out.get("single_env") or {}
    s["single_env_plan"] = se.get("value")
    ln = out.get("learner") or {}
    s["learner_graph_ms"] = (ln.get("graph") or {}).get("ms_per_update") if isinstance(ln.get("graph"), dict) else ln.get("graph")
    ic = out.get("icem") or {}
    s["icem_single_b32"] = [ic.get("value"), (ic.get("batch32") or {}).get("value")]
    s["x_cpu"] = out.get("speedup_vs_cpu")
    return s


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="humanoid-run")
    ap.add_argument("--envs-per-gpu", type=int, default=32)
    ap.add_argument("--sweep", default="8", help="comma-separated extra envs-per-GPU batches timed at N=1")
    ap.add_argument("--rng", default="fused", choices=["fused", "reference"])
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=8.0, help="seconds of CPU work per thread count timed")
    ap.add_argument("--also", default="cheetah-run,dog-run@8,quadruped-run-pixels,humanoid-run-l512",
                    help="comma-separated other configs (name[@envs per call], default --envs-per-gpu) timed at N=1 "
                         "in the same run, each with its own roofline and cpu_baseline (reported under 'configs')")
    ap.add_argument("--cpu-budget-config", type=float, default=5.0,
                    help="seconds of CPU work for each --also config's cpu_baseline")
    ap.add_argument("--single-calls", type=int, default=200, help="literal plan() calls timed one by one (median)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--no-single", action="store_true")
    ap.add_argument("--no-replay", action="store_true")
    ap.add_argument("--no-learner", action="store_true")
    ap.add_argument("--no-icem", action="store_true")
    ap.add_argument("--no-exact", action="store_true", help="skip the exact-f32-MFMA comparison run")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    cfg = bench_cfg(args.config)
    cfg.device = f"cuda:{local}"
    B = args.envs_per_gpu
    graph = not args.no_graph
    np.random.seed(2 + rank)
    agent = make_agent(cfg, B, args.rng, graph, 1 + rank)
    # the global vectorised batch (identical on every rank); each rank plans its contiguous shard
    global_obs = torch.from_numpy(synthetic_obs(cfg, B * world, seed=0)).to(dev)
    sharded = EnvShardedPlanner(B * world, cfg.action_dim, agent=agent)
    obs = sharded.local_obs(global_obs)
    step = 10**6

    def one_step(i):
        return sharded.plan(global_obs, step, t0=(i % 100 == 0))

    elapsed = time_steps(one_step, args.warmup, args.steps, dist)
    elapsed, value = job_rate(elapsed, B * args.steps, dist, dev)
    ms_per_step = elapsed / args.steps * 1e3

    # ---- roofline of the dominant kernel class: HIP events around each launch, eager replay of the same
    # steps on the same stream (graph replays cannot carry the events)
    roof = None
    if not args.no_roofline:
        roof = step_roofline(cfg, B, agent, one_step, max(3, min(args.steps, 10)), dev, f"{args.config}/B{B}")
        roof["q_head"] = q_roofline(cfg, B, agent, one_step, max(3, min(args.steps, 10)))
        roof["pi_head"] = q_roofline(cfg, B, agent, one_step, max(3, min(args.steps, 10)), 5, B * cfg.num_samples)

    fl_alg = plan_flops(cfg, executed=False)
    fl_exec = plan_flops(cfg, executed=True)
    plan_roof = {"flop_per_plan_step_algorithmic": fl_alg, "flop_per_plan_step_executed": fl_exec,
                 "tflops_per_gpu_algorithmic": round(value / world * fl_alg / 1e12, 3),
                 "frac_of_fp32_peak": round(value / world * min(fl_alg, fl_exec) / 1e12 / FP32_PEAK_TFLOPS, 4),
                 "frac_of_x6_peak": round(value / world * min(fl_alg, fl_exec) / 1e12 / X6_PEAK_TFLOPS, 4)}

    # the same workload on the exact f32 MFMA chain kernels (path chain32: v_mfma_f32_32x32x2_f32), same run
    exact = None
    if not args.no_exact and world == 1 and cfg.mlp_dim == 512:
        ae = make_agent(cfg, B, args.rng, graph, 1 + rank, path="chain32")
        ke = max(10, args.steps // 2)
        ele = time_steps(lambda i: ae.plan_batch(obs, step=step, t0=(i % 100 == 0), sync_metrics=False), 3, ke, None)
        exact = {"value": round(B * ke / ele, 3), "unit": "plan-steps/s", "ms_per_step": round(ele / ke * 1e3, 4),
                 "frac_of_fp32_peak": round(B * ke / ele * min(plan_flops(cfg, False), plan_flops(cfg, True)) / 1e12
                                            / FP32_PEAK_TFLOPS, 4),
                 "note": "exact f32 MFMA (v_mfma_f32_32x32x2_f32) chain kernels, path chain32, same envs"}
        del ae

    single = None
    if not args.no_single and world == 1:
        # the literal drop-in call src/train.py:95 makes: TDMPC(cfg) with its default arguments, a host numpy
        # observation, agent.plan(obs, step=..., t0=...) -> (device action, metrics dict of Python floats)
        a1 = TDMPC(cfg)
        a1.model.load_state_dict(synthetic_state_dict(cfg, 0))
        a1.std = 0.05
        o1 = synthetic_obs(cfg, 1, seed=0)[0]
        # every call synchronises (metrics to the host), so each is timed on its own: the median of
        # --single-calls calls after a warm-up (a few slow calls -- host preemption -- do not move it)
        for i in range(10):
            a1.plan(o1, step=step, t0=(i == 0))
        per = []
        for i in range(args.single_calls):
            t1 = time.perf_counter()
            a1.plan(o1, step=step, t0=False)
            per.append(time.perf_counter() - t1)
        med = float(np.median(per))
        single = {"value": round(1.0 / med, 3), "unit": "plan-steps/s", "ms_per_step": round(med * 1e3, 4),
                  "calls": len(per), "ms_mean": round(float(np.mean(per)) * 1e3, 4),
                  "ms_p10_p90": [round(float(np.percentile(per, 10)) * 1e3, 4),
                                 round(float(np.percentile(per, 90)) * 1e3, 4)],
                  "note": "median over the timed calls of agent.plan(obs, step, t0) exactly as src/train.py:95 calls "
                          "it: TDMPC(cfg) defaults (reference-order RNG on torch's / numpy's global generators -- the "
                          "torch draws as one tdmpc_reference_normals launch, bitwise torch's -- HIP graph replay), "
                          "numpy obs copied to the device, metrics synced to the host; same GPU, same run"}
        ks = max(20, args.steps // 2)
        # the same env through the batch API with device RNG and graph replay (no host sync)
        ab1 = make_agent(cfg, 1, args.rng, graph, 7)
        ob1 = obs[:1].clone()
        el2 = time_steps(lambda i: ab1.plan_batch(ob1, step=step, t0=(i % 100 == 0), sync_metrics=False),
                         3, ks, None)
        single["batch_api"] = {"value": round(ks / el2, 3), "ms_per_step": round(el2 / ks * 1e3, 4),
                               "note": f"plan_batch(obs[1]), rng={args.rng}, hip_graph={graph}, no metrics sync"}
        del a1, ab1

    sweep = None
    if world == 1 and args.sweep:
        sweep = {}
        for bs in [int(x) for x in args.sweep.split(",") if x.strip()]:
            if bs == B:
                continue
            ab = make_agent(cfg, bs, args.rng, graph, 11)
            ob = torch.from_numpy(synthetic_obs(cfg, bs, seed=0)).to(dev)
            kb = max(10, args.steps // 2)
            elb = time_steps(lambda i: ab.plan_batch(ob, step=step, t0=(i % 100 == 0), sync_metrics=False),
                             3, kb, None)
            sweep[str(bs)] = {"value": round(bs * kb / elb, 3), "unit": "plan-steps/s",
                              "ms_per_step": round(elb / kb * 1e3, 4),
                              "frac_of_fp32_peak": round(bs * kb / elb * min(fl_alg, fl_exec) / 1e12 / FP32_PEAK_TFLOPS, 4)}
            del ab

    replay = None
    if not args.no_replay and world == 1:
        replay = replay_bench(cfg, dev, cpu=not args.no_cpu)

    learner = None
    if not args.no_learner and world == 1 and cfg.modality == "state":
        learner = learner_bench(cfg, dev, cpu=not args.no_cpu)

    loop = None
    if not args.no_learner and world == 1 and cfg.modality == "state":
        loop = train_loop_bench(cfg, dev)

    icem = None
    if not args.no_icem and world == 1 and cfg.modality == "state":
        icem = icem_bench(cfg, dev, cpu=not args.no_cpu)

    others = None
    if world == 1 and args.also:
        # the other BASELINE.json configs, timed by the same driver run
        others = {}
        for spec in [x.strip() for x in args.also.split(",") if x.strip()]:
            name, _, eb = spec.partition("@")
            eb = int(eb) if eb else B
            if name == args.config and eb == B:
                continue
            key = name if eb == B else f"{name}@{eb}"
            others[key] = config_leg(name, eb, args, dev, graph, cpu=not args.no_cpu)

    cpu = None
    if rank == 0 and not args.no_cpu and world == 1:
        cpu = cpu_baselines(cfg, args.cpu_budget)

    if rank == 0:
        out = {
            "metric": "plan-steps/sec (N=512, H=5, iters=6) at 1/2/4/8 MI355X vs CPU ref",
            "value": round(value, 3), "unit": "plan-steps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
            "fp32_products": ("three-way bf16 split of both operands, 6 bf16 MFMA products per fp32 product, fp32 "
                              "accumulation (x6 chain kernels; parity tests at the fp32 tolerance; max |G - G_fp64| "
                              "2.8e-6 vs 4.0e-6 for the exact f32 MFMA, tests/test_gpu_plan.py::"
                              "test_x6_accuracy_matches_f32_mfma)"
                              if cfg.mlp_dim == 512 and os.environ.get("TDMPC_X6", "3") != "0" else "f32 MFMA"),
            "data": "synthetic: seeded N(0,1/fan_in) TOLD weights, N(0,1) observations, noise drawn on device",
            "config": {"workload": f"{args.config}: TDMPC.plan N={cfg.num_samples} H={cfg.horizon} "
                                   f"iters={cfg.iterations} mixture={cfg.mixture_coef} K={cfg.num_elites} "
                                   f"L={cfg.latent_dim} A={cfg.action_dim}, {B} envs per GPU",
                       "envs_per_gpu": B, "global_envs": B * world,
                       "parallelism": f"env-shard x{world}" + (" + rccl all-gather of [envs, A+2]" if world > 1 else ""),
                       "rng": args.rng, "hip_graph": graph},
            "roofline": roof,
            "plan_roofline": plan_roof,
            "exact_f32_mfma": exact,
            "batch_sweep": sweep,
            "configs": others,
            "replay_sampler": replay,
            "learner": learner,
            "train_loop": loop,
            "icem": icem,
            "cpu_baseline": cpu,
        }
        if cpu:
            out["speedup_vs_cpu"] = round(value / world / cpu["value"], 2)
            if single:
                single["speedup_vs_cpu"] = round(single["value"] / cpu["value"], 2)
        out["single_env"] = single
        out["summary"] = summary_line(out, cfg)   # (last: the driver keeps the tail of the line)
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
