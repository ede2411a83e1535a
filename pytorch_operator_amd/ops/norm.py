"""Fused RMSNorm (``csrc/kernels/rmsnorm.hip``) as an autograd op.

``rms_norm(x, w, eps)``: fp32 or bf16 activations ``[..., D]`` (D <= 8192), fp32 weight.
On a GPU the HIP kernels run (and their absence is an error, never a silent fallback);
on CPU the same math runs in PyTorch (used by the CPU tests and the gloo plumbing
config).  Statistics are fp32; the weight gradient is reduced deterministically.
"""
from __future__ import annotations

import ctypes

import torch

from . import _native

_DT = {torch.float32: 0, torch.bfloat16: 1}
_ROWS_PER_BLOCK = 16


def _stream(t: torch.Tensor):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def rms_norm_reference(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    return (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * w.float()).to(x.dtype)


class _RMSNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, eps):
        lib = _native.load()
        D = x.shape[-1]
        xc = x.contiguous()
        rows = xc.numel() // D
        y = torch.empty_like(xc)
        rstd = torch.empty(rows, device=x.device, dtype=torch.float32)
        _native.check(lib.pto_rmsnorm_fwd(xc.data_ptr(), w.data_ptr(), y.data_ptr(), rstd.data_ptr(), rows, D,
                                          float(eps), _DT[x.dtype], _stream(x)), "rmsnorm_fwd")
        ctx.save_for_backward(xc, w, rstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        lib = _native.load()
        xc, w, rstd = ctx.saved_tensors
        D = xc.shape[-1]
        rows = xc.numel() // D
        dyc = dy.contiguous().to(xc.dtype)
        dx = torch.empty_like(xc)
        dw = torch.empty(D, device=xc.device, dtype=torch.float32)
        parts = lib.pto_rmsnorm_bwd_parts(rows, _ROWS_PER_BLOCK)
        part = torch.empty((parts, D), device=xc.device, dtype=torch.float32)
        _native.check(lib.pto_rmsnorm_bwd(dyc.data_ptr(), xc.data_ptr(), w.data_ptr(), rstd.data_ptr(),
                                          dx.data_ptr(), dw.data_ptr(), part.data_ptr(), rows, D,
                                          _ROWS_PER_BLOCK, _DT[xc.dtype], _stream(xc)), "rmsnorm_bwd")
        return dx, dw.to(w.dtype), None


def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float = 1e-5) -> torch.Tensor:
    if not x.is_cuda:
        return rms_norm_reference(x, w, eps)
    if x.dtype not in _DT or w.dtype != torch.float32 or x.shape[-1] > 8192:
        raise ValueError("rms_norm: fp32/bf16 activations, fp32 weight, D <= 8192")
    return _RMSNorm.apply(x, w, eps)
