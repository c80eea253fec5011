"""CPU check of the x6 arithmetic the chain kernels use (tdmpc_kernels.hip split3 / x6_group): fp32 operands split
exactly into three bf16 parts, products from six bf16 x bf16 terms accumulated in fp32. A numpy restatement
(bf16 = round-to-nearest-even of the fp32 bits, as v_cvt_pk_bf16_f32 does) -- no GPU needed."""
import numpy as np


def bf16(x):
    u = np.asarray(x, np.float32).view(np.uint32).astype(np.uint64)
    u = (u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000
    return u.astype(np.uint32).view(np.float32)


def split3(x):
    x = np.asarray(x, np.float32)
    hi = bf16(x)
    r1 = (x - hi).astype(np.float32)
    mid = bf16(r1)
    lo = bf16((r1 - mid).astype(np.float32))
    return hi, mid, lo


def test_split_is_exact_to_fp32():
    rs = np.random.RandomState(0)
    x = (rs.standard_normal(100000) * np.exp(rs.uniform(-20, 20, 100000))).astype(np.float32)
    hi, mid, lo = split3(x)
    rec = hi.astype(np.float64) + mid.astype(np.float64) + lo.astype(np.float64)
    # every part is a bf16 value, and the three reproduce x to within half an fp32 ulp
    for p in (hi, mid, lo):
        assert np.all(p.view(np.uint32) & 0xFFFF == 0)
    rel = np.abs(rec - x.astype(np.float64)) / np.abs(x.astype(np.float64))
    assert rel.max() <= 2.0 ** -24


def test_six_term_dot_is_as_accurate_as_fp32():
    """A K = 512 dot product (the M x M layer's inner dimension) from the six kept terms, accumulated in fp32, is
    within the error of a plain fp32 dot product of the float64 result."""
    rs = np.random.RandomState(1)
    worst_x6, worst_f32 = 0.0, 0.0
    for _ in range(200):
        a = rs.standard_normal(512).astype(np.float32)
        b = (rs.standard_normal(512) / np.sqrt(512)).astype(np.float32)
        ref = float(np.dot(a.astype(np.float64), b.astype(np.float64)))
        ah, am, al = split3(a)
        bh, bm, bl = split3(b)
        acc = np.float32(0)
        for k in range(512):   # the kernel's order inside a k step: small terms first, hi.hi last
            for u, v in ((am, bm), (al, bh), (ah, bl), (am, bh), (ah, bm), (ah, bh)):
                acc = np.float32(acc + np.float32(u[k]) * np.float32(v[k]))
        f32 = np.float32(0)
        for k in range(512):
            f32 = np.float32(f32 + a[k] * b[k])
        scale = float(np.abs(a.astype(np.float64) * b).sum())
        worst_x6 = max(worst_x6, abs(float(acc) - ref) / scale)
        worst_f32 = max(worst_f32, abs(float(f32) - ref) / scale)
    assert worst_x6 <= 4 * worst_f32 + 2.0 ** -24, (worst_x6, worst_f32)
