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
