"""tdmpc_lg_adam (include/tdmpc_learner.h) against the pair the reference's update() runs
(/root/reference/src/algorithm/tdmpc.py:228-230: clip_grad_norm_(..., cfg.grad_clip_norm, error_if_nonfinite=False)
then optim.step()), with clip_grad_norm_ as the reference's PINNED torch 1.9 defines it (environment.yaml:6;
torch/nn/utils/clip_grad.py of 1.9: `clip_coef = max_norm / (total_norm + 1e-6); if clip_coef < 1: grad.mul_(clip_coef)`),
restated here because the installed torch (>= 1.13) clamps instead. Finite gradients above the clip norm agree to fp32
rounding (rtol 1e-5: the norm is reduced in another order). The non-finite patterns are pinned explicitly: a NaN
gradient entry makes the norm NaN, 1.9's `clip_coef < 1` test fails, nothing is scaled and ONLY that entry's parameter
turns NaN; an inf entry makes the coefficient 0 (inf * 0 = NaN in that entry, a zero gradient elsewhere)."""
import ctypes as C

import pytest
import torch

from tdmpc_amd import _lib

LR, B1, B2, EPS, MAX_NORM = 1e-3, 0.9, 0.999, 1e-8, 10.0


def _clip_grad_norm_19(p, max_norm):
    """torch 1.9's clip_grad_norm_ (norm_type 2) on one parameter."""
    total = torch.norm(torch.stack([torch.norm(p.grad.detach(), 2.0)]), 2.0)
    clip_coef = max_norm / (total + 1e-6)
    if clip_coef < 1:
        p.grad.detach().mul_(clip_coef)
    return total


def _torch_steps(p0, grads):
    p = torch.nn.Parameter(p0.clone())
    opt = torch.optim.Adam([p], lr=LR, betas=(B1, B2), eps=EPS, foreach=False)
    for g in grads:
        p.grad = g.clone()
        _clip_grad_norm_19(p, MAX_NORM)
        opt.step()
    return p.detach()


def _hip_steps(p0, grads):
    L = _lib.lib()
    dev = torch.device("cuda:0")
    p = p0.to(dev).clone()
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    step = torch.zeros(1, dtype=torch.int32, device=dev)
    norm_out = torch.zeros(1, device=dev)
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    for g in grads:
        gd = g.to(dev).contiguous()
        normp = (gd.double() ** 2).sum().float().reshape(1)   # one block's squared norm (lg_finalize's output)
        step += 1                                             # lg_finalize advances the step before lg_adam
        rc = L.tdmpc_lg_adam(C.c_void_p(p.data_ptr()), C.c_void_p(gd.data_ptr()), C.c_void_p(m.data_ptr()),
                             C.c_void_p(v.data_ptr()), p.numel(), C.c_void_p(normp.data_ptr()), 1,
                             C.c_void_p(step.data_ptr()), LR, B1, B2, EPS, MAX_NORM, C.c_void_p(norm_out.data_ptr()),
                             st)
        _lib.check(rc, "tdmpc_lg_adam")
    torch.cuda.synchronize()
    return p.cpu()


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["finite_clipped", "finite_unclipped", "nan_entry", "inf_entry", "finite_tail"])
def test_lg_adam_matches_torch_clip_and_adam(case):
    gen = torch.Generator().manual_seed(7)
    # > 256 x 256: several grid-stride rounds of the kernel; finite_tail: not a multiple of 4 (16-B body + element tail)
    n = 70_003 if case == "finite_tail" else 70_000
    p0 = torch.randn(n, generator=gen)
    scale = 1.0 if case != "finite_unclipped" else 1e-3
    grads = [torch.randn(n, generator=gen) * scale for _ in range(2)]
    if case == "nan_entry":
        grads[1][12_345] = float("nan")
    elif case == "inf_entry":
        grads[1][54_321] = float("inf")
    ref = _torch_steps(p0, grads)
    got = _hip_steps(p0, grads)
    assert torch.equal(torch.isnan(got), torch.isnan(ref))
    fin = torch.isfinite(ref)
    if case in ("nan_entry", "inf_entry"):   # exactly the non-finite gradient's entry (torch 1.9 semantics)
        bad = 12_345 if case == "nan_entry" else 54_321
        assert torch.nonzero(~torch.isfinite(got)).flatten().tolist() == [bad]
        assert torch.nonzero(~fin).flatten().tolist() == [bad]
    torch.testing.assert_close(got[fin], ref[fin], rtol=1e-5, atol=1e-7)
