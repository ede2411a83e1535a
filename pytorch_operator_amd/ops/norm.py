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
    return ctypes.c_void_p(_native.current_stream_ptr(t.device))


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


# ------------------------------------------------------------------ residual-fused RMSNorm
class _AddRMSNorm(torch.autograd.Function):
    """(s, y) = (x + delta, rmsnorm(x + delta)): the transformer block's residual add folded
    into the next norm (one pass instead of add + norm), and in the backward the residual
    gradient sum folded into the norm's dx (which is also written in the branch dtype, the
    gradient of ``delta``): no separate add or cast kernels around the norms."""

    @staticmethod
    def forward(ctx, x, delta, w, eps, out_dtype):
        lib = _native.load()
        D = x.shape[-1]
        rows = x.numel() // D
        s = torch.empty_like(x)
        y = torch.empty(x.shape, device=x.device, dtype=out_dtype)
        rstd = torch.empty(rows, device=x.device, dtype=torch.float32)
        pair = _PAIR[(x.dtype, out_dtype)]
        _native.check(lib.pto_add_rmsnorm_fwd(x.data_ptr(), delta.data_ptr(), w.data_ptr(), y.data_ptr(),
                                              s.data_ptr(), rstd.data_ptr(), rows, D, float(eps), pair,
                                              _stream(x)), "add_rmsnorm_fwd")
        ctx.save_for_backward(s, w, rstd)
        ctx.pair, ctx.out_dtype, ctx.delta_dtype = pair, out_dtype, delta.dtype
        return s, y

    @staticmethod
    def backward(ctx, gs, gy):
        lib = _native.load()
        s, w, rstd = ctx.saved_tensors
        D = s.shape[-1]
        rows = s.numel() // D
        gy = torch.zeros(s.shape, device=s.device, dtype=ctx.out_dtype) if gy is None else \
            _aligned(gy.to(ctx.out_dtype))
        gs = None if gs is None else _aligned(gs.to(s.dtype))
        dx = torch.empty_like(s)
        dbranch = torch.empty(s.shape, device=s.device, dtype=ctx.out_dtype)
        dw = torch.empty(D, device=s.device, dtype=torch.float32)
        parts = lib.pto_rmsnorm_bwd_parts(rows, _ROWS_PER_BLOCK)
        part = torch.empty((parts, D), device=s.device, dtype=torch.float32)
        _native.check(lib.pto_add_rmsnorm_bwd(gy.data_ptr(), s.data_ptr(), w.data_ptr(), rstd.data_ptr(),
                                              gs.data_ptr() if gs is not None else None, dx.data_ptr(),
                                              dbranch.data_ptr(), dw.data_ptr(), part.data_ptr(), rows, D,
                                              _ROWS_PER_BLOCK, ctx.pair, _stream(s)), "add_rmsnorm_bwd")
        return dx, dbranch, dw.to(w.dtype), None, None


def _aligned(t: torch.Tensor) -> torch.Tensor:
    t = t.contiguous()
    return t if t.data_ptr() % 16 == 0 else t.clone()


def add_rms_norm(x: torch.Tensor, delta: torch.Tensor, w: torch.Tensor, eps: float = 1e-5, out_dtype=None):
    """Returns ``(s, y)`` with ``s = x + delta`` (dtype of x: the residual stream) and
    ``y = rms_norm(s)`` in ``out_dtype``.  Fused HIP kernels on a GPU when ``delta`` has the
    output dtype and D % 4 == 0; otherwise the unfused ops (CPU, odd shapes)."""
    out_dtype = out_dtype or x.dtype
    if (x.is_cuda and (x.dtype, out_dtype) in _PAIR and delta.dtype == out_dtype and w.dtype == torch.float32
            and x.shape == delta.shape and x.shape[-1] % 4 == 0 and x.shape[-1] <= 8192):
        return _AddRMSNorm.apply(_aligned(x), _aligned(delta), w, eps, out_dtype)
    s = x + delta
    return s, rms_norm(s, w, eps, out_dtype)
