"""Gaussian noise with a power-law spectrum (1/f^beta), the iCEM planner's exploration noise.

The reference calls `colorednoise.powerlaw_psd_gaussian(exponent, size)` (tdmpc_icem_similarity_mlp.py:128-157).
`colorednoise` is neither vendored in /root/reference nor pinned (environment.yaml does not list it) and is
not installed here, so this is a restatement of its published algorithm (colorednoise 2.x,
`powerlaw_psd_gaussian`): frequencies f = rfftfreq(n) with the low cutoff fmin = 1/n, amplitude scale
f**(-beta/2), independent normal real and imaginary parts per frequency (the DC term and, for even n, the
Nyquist term real with their magnitude fixed by sqrt(2)), irfft, divided by the theoretical standard deviation
2 sqrt(sum(w^2)) / n. Parity of the generator itself is therefore unpinned; the iCEM planner is
pinned given its noise.

Two generators: `powerlaw_psd_gaussian(beta, size, rs)` on the host with a numpy RandomState (the reference draws
on the host; colorednoise 2.x seeds a fresh Generator from OS entropy per call, which no test could reproduce,
so here the caller's RandomState -- numpy's global one by default -- is used), and
`powerlaw_psd_gaussian_torch(beta, size, device)` on the device (rocFFT) for the fused-RNG path.
"""
from __future__ import annotations

import numpy as np
import torch


def _scales(beta, samples):
    f = np.fft.rfftfreq(samples)
    fmin = 1.0 / samples
    s_scale = f.copy()
    ix = int(np.sum(s_scale < fmin))
    if ix and ix < len(s_scale):
        s_scale[:ix] = s_scale[ix]
    s_scale = s_scale ** (-beta / 2.0)
    w = s_scale[1:].copy()
    w[-1] *= (1 + (samples % 2)) / 2.0
    sigma = 2 * np.sqrt(np.sum(w ** 2)) / samples
    return s_scale, sigma


def powerlaw_psd_gaussian(beta, size, rs=None):
    """size = (..., samples) -> float64 array of that shape (host, numpy RandomState `rs`, default global)."""
    rs = np.random if rs is None else rs
    size = list(size)
    samples = size[-1]
    s_scale, sigma = _scales(beta, samples)
    size[-1] = len(s_scale)
    s_scale = s_scale[(np.newaxis,) * (len(size) - 1) + (Ellipsis,)]
    sr = rs.normal(scale=s_scale, size=size)
    si = rs.normal(scale=s_scale, size=size)
    if not samples % 2:
        si[..., -1] = 0
        sr[..., -1] *= np.sqrt(2)
    si[..., 0] = 0
    sr[..., 0] *= np.sqrt(2)
    return np.fft.irfft(sr + 1j * si, n=samples, axis=-1) / sigma


def powerlaw_psd_gaussian_torch(beta, size, device, generator=None):
    """The same spectrum on the device (torch's generator, rocFFT), float32."""
    size = list(size)
    samples = size[-1]
    s_scale, sigma = _scales(beta, samples)
    size[-1] = len(s_scale)
    sc = torch.as_tensor(s_scale, dtype=torch.float32, device=device)
    sr = torch.randn(size, device=device, generator=generator) * sc
    si = torch.randn(size, device=device, generator=generator) * sc
    if not samples % 2:
        si[..., -1] = 0
        sr[..., -1] *= float(np.sqrt(2))
    si[..., 0] = 0
    sr[..., 0] *= float(np.sqrt(2))
    return torch.fft.irfft(torch.complex(sr, si), n=samples, dim=-1) / float(sigma)


def irfft_matrices(samples):
    """numpy's irfft(X, n=samples) as real matrices: y = Re(X) @ Cr + Im(X) @ Ci, Cr / Ci [F, samples] with
    F = samples // 2 + 1 (the imaginary parts of the DC and, for even n, Nyquist bins are ignored, as numpy does)."""
    L, F = samples, samples // 2 + 1
    t = np.arange(L)
    Cr = np.zeros((F, L))
    Ci = np.zeros((F, L))
    for k in range(F):
        w = 1.0 if k == 0 or (L % 2 == 0 and k == L // 2) else 2.0
        Cr[k] = w * np.cos(2 * np.pi * k * t / L) / L
        if w == 2.0:
            Ci[k] = -2.0 * np.sin(2 * np.pi * k * t / L) / L
    return Cr, Ci


def spectrum_rows(beta, samples):
    """Per-frequency factors of powerlaw_psd_gaussian folded into one row each for the real and imaginary
    normal draws (s_scale, the sqrt(2) of the DC / Nyquist real parts, zero imaginary parts there) and 1/sigma."""
    s_scale, sigma = _scales(beta, samples)
    re, im = s_scale.copy(), s_scale.copy()
    if not samples % 2:
        im[-1] = 0.0
        re[-1] *= np.sqrt(2)
    im[0] = 0.0
    re[0] *= np.sqrt(2)
    return re, im, 1.0 / sigma


class BatchedColoredNoise:
    """Every coloured-noise draw of one call as ONE batched device computation (fused-RNG paths): one normal draw
    [R, 2F] for the R = sum(n * A) sequences of all (beta, n) specs, per-row spectrum factors, the irfft as a
    matmul with irfft_matrices, 1/sigma, first H samples. The same distribution as powerlaw_psd_gaussian per
    spec (torch's generator); ~6 launches instead of ~10 per spec."""

    def __init__(self, specs, A, samples, H, device):
        F = samples // 2 + 1
        re_rows, im_rows, inv = [], [], []
        for beta, n in specs:
            re, im, isg = spectrum_rows(beta, samples)
            re_rows.append(np.broadcast_to(re, (n * A, F)))
            im_rows.append(np.broadcast_to(im, (n * A, F)))
            inv.append(np.full(n * A, isg))
        self.R = sum(n * A for _, n in specs)
        f32 = dict(dtype=torch.float32, device=device)
        self.re = torch.as_tensor(np.concatenate(re_rows) if re_rows else np.zeros((0, F)), **f32)
        self.im = torch.as_tensor(np.concatenate(im_rows) if im_rows else np.zeros((0, F)), **f32)
        Cr, Ci = irfft_matrices(samples)
        inv_sigma = np.concatenate(inv) if inv else np.zeros(0)
        # fold 1/sigma into the matrices per row is not possible (row-dependent): scale the factors instead
        self.re *= torch.as_tensor(inv_sigma, **f32)[:, None]
        self.im *= torch.as_tensor(inv_sigma, **f32)[:, None]
        self.C = torch.as_tensor(np.concatenate([Cr, Ci])[:, :H], **f32)   # [2F, H]
        self.F = F

    def draw(self, generator=None):
        """-> [R, H] float32: row r = sequence r (spec-major, then n, then A), its first H samples."""
        z = torch.randn(self.R, 2 * self.F, device=self.C.device, generator=generator)
        z[:, :self.F] *= self.re
        z[:, self.F:] *= self.im
        return z @ self.C
