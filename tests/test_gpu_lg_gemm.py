"""GPU: tdmpc_lg_gemm's tiles against float64 torch (include/tdmpc_learner.h).

The learner's products (tdmpc.py:165-245 as learner_engine.py writes them out) run on tdmpc_lg_gemm: register tiles
(1 / 2, the exact f32 MFMA with TDMPC_LG_TILE_EXACT) and the LDS-staged macro tiles (3 / 4 / 5) for the large ones.
Every tile must give C = epi(sum over segments A B + bias + res) within fp32 accumulation error of the float64
product, bitwise the same on a second launch, for the operand forms the engine uses: row-major activations with
16-B aligned and unaligned row strides (121-float rows, and rows padded to 124 whose last quad straddles K), Linear weights [N][K] and their transpose [K][N],
K tails (100 / 121), two segments over one weight's column ranges, row counts and widths off the tile grid, and
several jobs of different shapes in one launch. Tolerance: |C - C64| <= 4e-6 (|A| |B| + |bias| + |res|) -- an f32
fma chain over K <= 1024 stays below ~1.5e-7 of that sum per the MI355X guide's measurement; the margin covers the
epilogue's own rounding.
"""
import ctypes as C

import pytest
import torch

from tdmpc_amd import _lib

pytestmark = pytest.mark.gpu

EXACT = 0x100
EPI_NONE, EPI_ELU, EPI_ELU_BWD = 0, 1, 3
TILES = [1 | EXACT, 2 | EXACT, 3, 4]


def _job(J, segs, m, n, c, ldc, epi=EPI_NONE, bias=None, res=None, aux=None):
    for s, (a, lda, b, ldb, k, bmode) in enumerate(segs):
        S = J.seg[s]
        S.a, S.b, S.lda, S.ldb, S.k, S.amode, S.bmode, S.ones_col = a, b, lda, ldb, k, 0, bmode, -1
    J.nseg, J.m, J.n, J.epi, J.c, J.ldc = len(segs), m, n, epi, c, ldc
    J.bias = bias.data_ptr() if bias is not None else None
    if res is not None:
        J.res, J.ldres = res.data_ptr(), res.stride(0)
    if aux is not None:
        J.aux, J.ldaux = aux.data_ptr(), aux.stride(0)
    J.splits, J.slice = 1, 0


def _case(g, m, n, parts, bmode, epi, lda_pad=0, bias=True, res=False):
    """parts: [(k, c0)] -- segments over weight columns [c0, c0 + k) of one weight W [N][K] (bmode 0) or
    [K][N] (bmode 1). Returns (segs, reference float64, scale, outputs, keepalive)."""
    dev = torch.device("cuda")
    K = max(c0 + k for k, c0 in parts)
    W = torch.randn(n, K, generator=g).to(dev) if bmode == 0 else torch.randn(K, n, generator=g).to(dev)
    xs = [torch.randn(m, k + lda_pad, generator=g).to(dev) for k, _ in parts]
    b = torch.randn(n, generator=g).to(dev) if bias else None
    r = torch.randn(m, n, generator=g).to(dev) if res else None
    aux = torch.nn.functional.elu(torch.randn(m, n, generator=g)).to(dev) if epi == EPI_ELU_BWD else None
    segs, ref, scale = [], torch.zeros(m, n, dtype=torch.float64, device=dev), torch.zeros(m, n, dtype=torch.float64,
                                                                                             device=dev)
    for x, (k, c0) in zip(xs, parts):
        if bmode == 0:
            segs.append((x.data_ptr(), x.stride(0), W.data_ptr() + 4 * c0, K, k, 0))
            Wk = W[:, c0:c0 + k].double().t()
        else:
            segs.append((x.data_ptr(), x.stride(0), W.data_ptr() + 4 * c0 * n, n, k, 1))
            Wk = W[c0:c0 + k].double()
        xd = x[:, :k].double()
        ref += xd @ Wk
        scale += xd.abs() @ Wk.abs()
    if b is not None:
        ref += b.double()
        scale += b.double().abs()
    if r is not None:
        ref += r.double()
        scale += r.double().abs()
    if epi == EPI_ELU:
        ref = torch.nn.functional.elu(ref)
    elif epi == EPI_ELU_BWD:
        a64 = aux.double()
        ref = ref * torch.where(a64 > 0, torch.ones_like(a64), a64 + 1)
        scale = scale * torch.where(a64 > 0, torch.ones_like(a64), (a64 + 1).abs())
    out = torch.full((m, n), float("nan"), device=dev)
    return segs, ref, scale, out, (W, xs, b, r, aux)


CASES = [
    # m, n, parts [(k, c0)], bmode, epi, lda_pad, bias, res
    (2560, 512, [(512, 0)], 0, EPI_NONE, 0, True, False),      # the heads' hidden layers (R = H B rows)
    (3072, 512, [(512, 0)], 1, EPI_ELU_BWD, 0, False, False),  # a dX through W (transpose) with ELU'
    (2560, 512, [(121, 0)], 0, EPI_ELU, 0, True, False),       # first layer over [z, a], unaligned rows, K tail
    (2560, 512, [(121, 0)], 0, EPI_NONE, 3, True, False),      # rows padded to 124: a 16-B quad straddles K
    (3072, 512, [(100, 0), (21, 100)], 0, EPI_NONE, 0, True, False),  # two segments over W's column ranges
    (1000, 100, [(512, 0)], 0, EPI_NONE, 3, True, True),       # off-grid rows / width, padded rows, residual
    (300, 21, [(512, 0)], 1, EPI_NONE, 0, False, False),       # a narrow output through W^T
    # the latent rollout's 512-row layers (tdmpc.py:203-205): [z, a] rows padded to 124 through W0 [512][121], the
    # hidden layer, the latent output; the backward's dX through W4^T, W2^T and W0[:, :100]^T (stride 121)
    (512, 512, [(121, 0)], 0, EPI_ELU, 3, True, False),
    (512, 512, [(512, 0)], 0, EPI_ELU, 0, True, False),
    (512, 100, [(512, 0)], 0, EPI_NONE, 0, True, False),
    (512, 512, [(100, 0)], 1, EPI_ELU_BWD, 0, False, False),
    (512, 512, [(512, 0)], 1, EPI_ELU_BWD, 0, False, False),
    (512, 100, [(512, 0)], 1, EPI_NONE, 0, False, True),
]


def _launch(L, tile, cases, idx, stream):
    arr = (_lib.LgJob * len(idx))()
    for J, q in zip(arr, idx):
        c = CASES[q]
        segs, ref, scale, out, keep = cases[q]
        W, xs, b, r, aux = keep
        _job(J, segs, c[0], c[1], out.data_ptr(), out.stride(0), epi=c[4], bias=b, res=r, aux=aux)
    _lib.check(L.tdmpc_lg_gemm(arr, len(idx), tile, stream), "tdmpc_lg_gemm")


@pytest.mark.parametrize("tile", TILES, ids=lambda t: f"tile{t & 0xff}{'x' if t & EXACT else ''}")
def test_gpu_lg_gemm_tiles_match_float64(tile):
    L = _lib.lib()
    g = torch.Generator().manual_seed(7)
    stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    cases = [_case(g, *c) for c in CASES]
    # one grouped launch per weight form (the macro tiles take one bmode per launch)
    groups = [[q for q, c in enumerate(CASES) if c[3] == bm] for bm in (0, 1)]

    def launch_all():
        for idx in groups:
            _launch(L, tile, cases, idx, stream)
        torch.cuda.synchronize()
    launch_all()
    firsts = [cs[3].clone() for cs in cases]
    for c, (segs, ref, scale, out, keep) in zip(CASES, cases):
        assert torch.isfinite(out).all(), c
        err = ((out.double() - ref).abs() / (scale + 1e-30)).max().item()
        assert err <= 4e-6, (c, tile, err)
    # a second launch: bitwise the same (fixed-order sums)
    for cs in cases:
        cs[3].fill_(float("nan"))
    launch_all()
    for f, cs in zip(firsts, cases):
        assert torch.equal(f, cs[3])


def test_gpu_lg_gemm_macro_tiles_refuse_unsupported_jobs():
    L = _lib.lib()
    dev = torch.device("cuda")
    a, w, out = (torch.zeros(64, 64, device=dev) for _ in range(3))
    arr = (_lib.LgJob * 1)()
    _job(arr[0], [(a.data_ptr(), 64, w.data_ptr(), 64, 64, 1)], 64, 64, out.data_ptr(), 64)
    arr[0].seg[0].amode = 1   # A transposed (the weight gradients): register tiles only
    for tile in (3, 4):
        assert L.tdmpc_lg_gemm(arr, 1, tile, None) == -1   # TDMPC_E_DIMS
    arr[0].seg[0].amode = 0
    arr[0].splits = 2          # split-K slices: register tiles only
    for tile in (3, 4):
        assert L.tdmpc_lg_gemm(arr, 1, tile, None) == -1   # TDMPC_E_DIMS
    arr2 = (_lib.LgJob * 2)()  # two weight forms in one launch: one per launch on the macro tiles
    _job(arr2[0], [(a.data_ptr(), 64, w.data_ptr(), 64, 64, 0)], 64, 64, out.data_ptr(), 64)
    _job(arr2[1], [(a.data_ptr(), 64, w.data_ptr(), 64, 64, 1)], 64, 64, out.data_ptr(), 64)
    for tile in (3, 4):
        assert L.tdmpc_lg_gemm(arr2, 2, tile, None) == -1   # TDMPC_E_DIMS
