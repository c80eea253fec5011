"""Time the learner's grouped GEMM (tdmpc_lg_gemm) on its operand layouts (development tool).
    python tools/lg_gemm_bench.py [--small | --dw | --big]
C[m][n] = sum_k A(m, k) B(n, k): amode 0 A[m][k] (row-major activations), 1 A[k][m]; bmode 0 B[n][k] (a Linear weight
[out][in]), 1 B[k][n] (its transpose). --big: the macro tiles (3 / 4 / 5) against the register tiles and torch.mm
(hipBLASLt) on the heads' large products, single and grouped (2 / 3 jobs per launch)."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from tdmpc_amd import _lib

lib = _lib.lib()
dev = torch.device("cuda")
EXACT = 0x100


def _time(fn, reps):
    """GPU time per call: `reps` calls captured into one HIP graph and replayed (no host launch cost in the
    timing -- the learner replays its update as a graph too)."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.graph(g, stream=s):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def run(m, n, k, amode, bmode, tile, splits=1, reps=50, njobs=1, lda=None):
    lda = lda or (k if amode == 0 else m)
    As = [torch.randn((m if amode == 0 else k) * lda, device=dev) for _ in range(njobs)]
    Bs = [torch.randn(n * k, device=dev) for _ in range(njobs)]
    Cs = [torch.zeros(splits * m * n, device=dev) for _ in range(njobs)]
    arr = (_lib.LgJob * njobs)()
    for q in range(njobs):
        J = arr[q]
        J.seg[0].a, J.seg[0].b = As[q].data_ptr(), Bs[q].data_ptr()
        J.seg[0].lda = lda
        J.seg[0].ldb = k if bmode == 0 else n
        J.seg[0].k, J.seg[0].amode, J.seg[0].bmode, J.seg[0].ones_col = k, amode, bmode, -1
        J.nseg, J.m, J.n, J.epi, J.c, J.ldc = 1, m, n, 0, Cs[q].data_ptr(), n
        J.splits, J.slice = splits, m * n
    rc = lib.tdmpc_lg_gemm(arr, njobs, tile, C.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0, rc
    us = _time(lambda: lib.tdmpc_lg_gemm(arr, njobs, tile, C.c_void_p(torch.cuda.current_stream().cuda_stream)), reps)
    err = 0.0
    for q in range(njobs):
        A = As[q].view(m, lda)[:, :k] if amode == 0 else As[q].view(k, m).t()
        Bm = Bs[q].view(n, k).t() if bmode == 0 else Bs[q].view(k, n)
        ref = A.double() @ Bm.double()
        got = Cs[q].view(splits, m, n).sum(0).double()
        err = max(err, ((got - ref).abs().max() / ref.abs().max()).item())
    print(f"m {m:5d} n {n:4d} k {k:5d} amode {amode} bmode {bmode} tile {tile:#5x} splits {splits} jobs {njobs}: "
          f"{us:7.1f} us {2 * m * n * k * njobs / us / 1e6:6.1f} TFLOP/s  (rel err vs fp64 {err:.1e})", flush=True)
    return us


def run_torch(m, n, k, bmode, reps=50, njobs=1, lda=None):
    lda = lda or k
    torch.backends.cuda.matmul.allow_tf32 = False
    As = [torch.randn(m, lda, device=dev)[:, :k] for _ in range(njobs)]
    Ws = [torch.randn(n, k, device=dev) if bmode == 0 else torch.randn(k, n, device=dev) for _ in range(njobs)]
    Cs = [torch.empty(m, n, device=dev) for _ in range(njobs)]

    def fn():
        for q in range(njobs):
            torch.mm(As[q], Ws[q].t() if bmode == 0 else Ws[q], out=Cs[q])
    us = _time(fn, reps)
    print(f"m {m:5d} n {n:4d} k {k:5d} torch.mm bmode {bmode} jobs {njobs}: {us:7.1f} us "
          f"{2 * m * n * k * njobs / us / 1e6:6.1f} TFLOP/s", flush=True)


if "--roll" in sys.argv:   # the latent rollout's 512-row products (forward, then the backward's dX through W^T)
    for (m, n, k, am, bm, lda) in [(512, 512, 121, 0, 0, 124), (512, 512, 512, 0, 0, None), (512, 100, 512, 0, 0, None),
                                   (512, 512, 100, 0, 1, None), (512, 512, 512, 0, 1, None), (512, 100, 512, 0, 1, None)]:
        for tile in (1 | EXACT, 2 | EXACT):
            run(m, n, k, am, bm, tile, lda=lda)
    sys.exit(0)
if "--diag" in sys.argv:   # fixed costs of the register tile (TDMPC_LG_DIAG read once per process: one per run)
    print("TDMPC_LG_DIAG", os.environ.get("TDMPC_LG_DIAG", "0"))
    for (m, n, k) in [(512, 512, 512), (512, 512, 32), (32, 32, 32)]:
        run(m, n, k, 0, 0, 1 | EXACT)
    x = torch.zeros(4096, device=dev)
    us = _time(lambda: lib.tdmpc_lg_act(x.data_ptr(), None, 4096, 0, C.c_void_p(torch.cuda.current_stream().cuda_stream)), 50)
    print(f"tdmpc_lg_act on 4096 floats (one workgroup): {us:.2f} us")
    sys.exit(0)
if "--small" in sys.argv:
    for (m, n, k, am, bm) in [(512, 512, 512, 0, 0), (512, 512, 121, 0, 0), (512, 100, 512, 0, 0),
                              (512, 512, 100, 0, 1), (512, 512, 512, 0, 1), (512, 100, 512, 0, 1)]:
        for tile in (1, 2):
            run(m, n, k, am, bm, tile | EXACT)
    sys.exit(0)
if "--quick" in sys.argv:   # the macro tiles only (ring depth from TDMPC_LG_BIG_D)
    print("TDMPC_LG_BIG_D", os.environ.get("TDMPC_LG_BIG_D", "2"))
    for (m, n, k, bm, lda) in [(2560, 512, 512, 0, None), (3072, 512, 512, 1, None), (2560, 512, 121, 0, 121)]:
        for nj in (1, 3):
            run_torch(m, n, k, bm, njobs=nj, lda=lda)
            for tile in (1 | EXACT, 2 | EXACT, 3, 4):
                run(m, n, k, 0, bm, tile, njobs=nj, lda=lda)
    sys.exit(0)
if "--scan" in sys.argv:   # fixed cost vs size of the macro tiles
    for (m, n, k) in [(64, 64, 32), (256, 512, 32), (2560, 512, 32), (2560, 512, 128), (2560, 512, 512),
                      (2560, 64, 512), (320, 512, 512)]:
        run_torch(m, n, k, 0)
        for tile in (1 | EXACT, 3):
            run(m, n, k, 0, 0, tile)
    sys.exit(0)
if "--big" in sys.argv:
    shapes = [(2560, 512, 512, 0, None), (3072, 512, 512, 0, None), (2560, 512, 512, 1, None),
              (3072, 512, 512, 1, None), (2560, 512, 121, 0, 121), (3072, 512, 100, 0, None), (512, 512, 512, 0, None)]
    for (m, n, k, bm, lda) in shapes:
        for nj in (1, 2, 3):
            run_torch(m, n, k, bm, njobs=nj, lda=lda)
            for tile in (1 | EXACT, 2 | EXACT, 3, 4):
                run(m, n, k, 0, bm, tile, njobs=nj, lda=lda)
    sys.exit(0)
for (m, n, k) in ([] if "--dw" in sys.argv else [(2560, 512, 512), (3072, 512, 512), (512, 512, 512), (2560, 512, 121), (2560, 21, 512)]):
    for amode, bmode in [(0, 0), (0, 1), (1, 1)]:
        for tile in (1, 2):
            run(m, n, k, amode, bmode, tile | EXACT)
# weight-gradient shape: m = out, n = in + 1, k = rows (A = dY^T, B = X^T)
for tile in (1, 2):
    for sp in (1, 2, 4):
        run(512, 513, 2560, 1, 1, tile | EXACT, splits=sp)
        run(512, 122, 2560, 1, 1, tile | EXACT, splits=sp)
        run(21, 513, 3072, 1, 1, tile | EXACT, splits=sp)
