"""Time the learner's grouped GEMM (tdmpc_lg_gemm) on its operand layouts (development tool).
    python tools/lg_gemm_bench.py
C[m][n] = sum_k A(m, k) B(n, k): amode 0 A[m][k] (row-major activations), 1 A[k][m]; bmode 0 B[n][k] (a Linear weight
[out][in]), 1 B[k][n] (its transpose)."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from tdmpc_amd import _lib

lib = _lib.lib()
dev = torch.device("cuda")


def run(m, n, k, amode, bmode, tile, splits=1, reps=50):
    A = torch.randn(m * k, device=dev)
    B = torch.randn(n * k, device=dev)
    Cm = torch.zeros(splits * m * n, device=dev)
    arr = (_lib.LgJob * 1)()
    J = arr[0]
    J.seg[0].a, J.seg[0].b = A.data_ptr(), B.data_ptr()
    J.seg[0].lda = k if amode == 0 else m
    J.seg[0].ldb = k if bmode == 0 else n
    J.seg[0].k, J.seg[0].amode, J.seg[0].bmode, J.seg[0].ones_col = k, amode, bmode, -1
    J.nseg, J.m, J.n, J.epi, J.c, J.ldc = 1, m, n, 0, Cm.data_ptr(), n
    J.splits, J.slice = splits, m * n
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    for _ in range(3):
        lib.tdmpc_lg_gemm(arr, 1, tile, st)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        lib.tdmpc_lg_gemm(arr, 1, tile, st)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    ref = (A.view(m, k) if amode == 0 else A.view(k, m).t()) @ (B.view(n, k).t() if bmode == 0 else B.view(k, n))
    got = Cm.view(splits, m, n).sum(0)
    err = ((got - ref).abs().max() / ref.abs().max()).item()
    print(f"m {m:5d} n {n:4d} k {k:5d} amode {amode} bmode {bmode} tile {tile} splits {splits}: {us:7.1f} us "
          f"{2 * m * n * k / us / 1e6:6.1f} TFLOP/s  (rel err {err:.1e})", flush=True)


import sys as _s
if "--small" in _s.argv:
    for (m, n, k, am, bm) in [(512, 512, 512, 0, 0), (512, 512, 121, 0, 0), (512, 100, 512, 0, 0),
                              (512, 512, 100, 0, 1), (512, 512, 512, 0, 1), (512, 100, 512, 0, 1)]:
        for tile in (1, 2):
            run(m, n, k, am, bm, tile)
    _s.exit(0)
for (m, n, k) in ([] if "--dw" in _s.argv else [(2560, 512, 512), (3072, 512, 512), (512, 512, 512), (2560, 512, 121), (2560, 21, 512)]):
    for amode, bmode in [(0, 0), (0, 1), (1, 1)]:
        for tile in (1, 2):
            run(m, n, k, amode, bmode, tile)
# weight-gradient shape: m = out, n = in + 1, k = rows (A = dY^T, B = X^T)
for tile in (1, 2):
    for sp in (1, 2, 4):
        run(512, 513, 2560, 1, 1, tile, splits=sp)
        run(512, 122, 2560, 1, 1, tile, splits=sp)
        run(21, 513, 3072, 1, 1, tile, splits=sp)
