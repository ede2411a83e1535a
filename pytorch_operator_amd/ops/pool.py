"""3x3 / stride 2 / pad 1 max-pool for channels-last bf16 activations (``csrc/kernels/pool.hip``).

The ResNet-50 stem pool: PyTorch stores an int64 index per output (as many bytes as the
411 MB input at B=256) and reads it back in the backward; here the forward keeps one tap byte
per output and the backward gathers the <= 4 covering windows per input pixel (no atomics, no
zero fill).  ``MaxPool3x3s2`` is a drop-in ``nn.MaxPool2d(3, 2, 1)``; on CPU, for other dtypes
or layouts it runs PyTorch's own op (the numerics reference of the tests).
"""
from __future__ import annotations

import ctypes

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _native


def supported(x: torch.Tensor) -> bool:
    return (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and x.shape[1] % 8 == 0
            and x.is_contiguous(memory_format=torch.channels_last))


class _MaxPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        N, C, H, W = x.shape
        OH, OW = (H - 1) // 2 + 1, (W - 1) // 2 + 1
        y = torch.empty((N, C, OH, OW), dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
        tap = torch.empty((N, OH, OW, C), dtype=torch.uint8, device=x.device)
        s = ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream)
        _native.check(_native.load().pto_maxpool3s2_fwd(x.data_ptr(), y.data_ptr(), tap.data_ptr(), N, H, W, C, s),
                      "maxpool3s2_fwd")
        ctx.save_for_backward(tap)
        ctx.shape = (N, C, H, W)
        return y

    @staticmethod
    def backward(ctx, dy):
        (tap,) = ctx.saved_tensors
        N, C, H, W = ctx.shape
        dy = dy.contiguous(memory_format=torch.channels_last)
        dx = torch.empty((N, C, H, W), dtype=dy.dtype, device=dy.device, memory_format=torch.channels_last)
        s = ctypes.c_void_p(torch.cuda.current_stream(dy.device).cuda_stream)
        _native.check(_native.load().pto_maxpool3s2_bwd(dy.data_ptr(), tap.data_ptr(), dx.data_ptr(), N, H, W, C, s),
                      "maxpool3s2_bwd")
        return dx


def max_pool_3x3_s2(x: torch.Tensor, impl: str = "hip") -> torch.Tensor:
    if impl == "hip" and supported(x):
        return _MaxPool.apply(x)
    return F.max_pool2d(x, 3, 2, 1)


class MaxPool3x3s2(nn.MaxPool2d):
    """``nn.MaxPool2d(3, stride=2, padding=1)`` with the HIP kernels for channels-last bf16."""

    def __init__(self):
        super().__init__(3, stride=2, padding=1)
        self.impl = "hip"

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return max_pool_3x3_s2(x, self.impl)
