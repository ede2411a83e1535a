"""Fused RMSNorm (``csrc/kernels/rmsnorm.hip``) as an autograd op.

``rms_norm(x, w, eps, out_dtype=None)``: fp32 or bf16 activations ``[..., D]`` (D <= 8192),
fp32 weight.  ``out_dtype=torch.bfloat16`` with fp32 ``x`` writes a bf16 ``y`` straight from
the kernel (and takes a bf16 ``dy`` in the backward): the Llama blocks use it under bf16
autocast, where the next op is a bf16 matmul, so no separate cast kernels run.  On a GPU the HIP kernels run (and their absence is an error, never a silent fallback);
on CPU the same math runs in PyTorch (used by the CPU tests and the gloo plumbing
config).  Statistics are fp32; the weight gradient is reduced deterministically.
"""
from __future__ import annotations

import ctypes

import torch

from . import _native

_DT = {torch.float32: 0, torch.bfloat16: 1}
# (x dtype, y dtype) -> kernel dtype-pair code (csrc/kernels/rmsnorm.hip)
_PAIR = {(torch.float32, torch.float32): 0, (torch.bfloat16, torch.bfloat16): 1,
         (torch.float32, torch.bfloat16): 2}
_ROWS_PER_BLOCK = 8  # tools/llm_kernel_bench.py sweep at 8192x4096: 4/8/16/32 -> 82/75/80/121 us


def _stream(t: torch.Tensor):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def rms_norm_reference(x: torch.Tensor, w: torch.Tensor, eps: float, out_dtype=None) -> torch.Tensor:
    xf = x.float()
    return (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * w.float()).to(out_dtype or x.dtype)


class _RMSNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, eps, out_dtype):
        lib = _native.load()
        D = x.shape[-1]
        xc = x.contiguous()
        rows = xc.numel() // D
        y = torch.empty(xc.shape, device=x.device, dtype=out_dtype)
        rstd = torch.empty(rows, device=x.device, dtype=torch.float32)
        pair = _PAIR[(x.dtype, out_dtype)]
        _native.check(lib.pto_rmsnorm_fwd(xc.data_ptr(), w.data_ptr(), y.data_ptr(), rstd.data_ptr(), rows, D,
                                          float(eps), pair, _stream(x)), "rmsnorm_fwd")
        ctx.save_for_backward(xc, w, rstd)
        ctx.pair, ctx.out_dtype = pair, out_dtype
        return y

    @staticmethod
    def backward(ctx, dy):
        lib = _native.load()
        xc, w, rstd = ctx.saved_tensors
        D = xc.shape[-1]
        rows = xc.numel() // D
        dyc = dy.contiguous().to(ctx.out_dtype)
        dx = torch.empty_like(xc)
        dw = torch.empty(D, device=xc.device, dtype=torch.float32)
        parts = lib.pto_rmsnorm_bwd_parts(rows, _ROWS_PER_BLOCK)
        part = torch.empty((parts, D), device=xc.device, dtype=torch.float32)
        _native.check(lib.pto_rmsnorm_bwd(dyc.data_ptr(), xc.data_ptr(), w.data_ptr(), rstd.data_ptr(),
                                          dx.data_ptr(), dw.data_ptr(), part.data_ptr(), rows, D,
                                          _ROWS_PER_BLOCK, ctx.pair, _stream(xc)), "rmsnorm_bwd")
        return dx, dw.to(w.dtype), None, None


def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float = 1e-5, out_dtype=None) -> torch.Tensor:
    out_dtype = out_dtype or x.dtype
    if not x.is_cuda:
        return rms_norm_reference(x, w, eps, out_dtype)
    if (x.dtype, out_dtype) not in _PAIR or w.dtype != torch.float32 or x.shape[-1] > 8192:
        raise ValueError("rms_norm: fp32/bf16 activations (y fp32/bf16), fp32 weight, D <= 8192")
    return _RMSNorm.apply(x, w, eps, out_dtype)
