"""Training-mode BatchNorm2d (+ residual add) (+ ReLU) on HIP kernels (``csrc/kernels/batchnorm.hip``).

The ResNet-50 worker's step is 58 % batch-norm and elementwise passes on the library path
(MIOpen mean/variance + normalise, then separate clamp / add / threshold-backward kernels:
``profiles/r2_resnet50_kernels.md``).  ``batch_norm_act`` fuses a bottleneck's
``relu(bn(x) [+ residual])`` into one statistics pass and one normalise pass, and its
backward into one reduction pass and one dx pass (the ReLU mask is recomputed from x when no
residual was added), for channels-last fp32/bf16 activations.

Residual gradient fusion (``link_output``): a bottleneck's output y feeds the next block twice
-- its conv1 and, as the identity, its residual add -- so autograd would sum the two incoming
gradients with an extra elementwise pass (2 reads + 1 write of the activation).  Here the
consumer's backward hands its residual gradient to the producer through a ``GradLink``
(returning no autograd gradient for that input, so the edge only orders the two backwards)
and the producer's backward kernels load both gradients and add them in fp32.

The first block of a stage uses its input twice through convolutions (conv1 and the
downsample conv): ``link_tap`` routes the downsample conv's input gradient through the same
link, so that sum is fused into the producer's backward as well.

``BatchNormAct2d`` is a drop-in ``nn.BatchNorm2d`` (same parameters, buffers and state dict)
whose forward takes an optional residual and applies the ReLU itself.  Its ``impl``
(``"hip"`` / ``"library"``) selects the HIP kernels or PyTorch's own ops on a GPU; on CPU, in
eval mode, for unsupported shapes (C/8 must divide 256) or cumulative-average momentum it
always runs the PyTorch ops -- the numerics reference of the tests.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _native

_DT = {torch.float32: 0, torch.bfloat16: 1}
MASK_BITS = True  # residual+ReLU backward masks from the forward's bit image (False: re-read y)


def _stream(t: torch.Tensor):
    return ctypes.c_void_p(_native.current_stream_ptr(t.device))


def supported(x: torch.Tensor) -> bool:
    C = x.shape[1] if x.dim() == 4 else 0
    return x.is_cuda and x.dim() == 4 and x.dtype in _DT and C % 8 == 0 and 8 <= C <= 2048 and 256 % (C // 8) == 0


def reference(x, weight, bias, running_mean, running_var, training, momentum, eps, relu, residual):
    y = F.batch_norm(x, running_mean, running_var, weight, bias, training, momentum, eps)
    if residual is not None:
        y = y + residual
    return F.relu(y) if relu else y


def _nhwc(t: torch.Tensor, dtype) -> torch.Tensor:
    return t.to(dtype).contiguous(memory_format=torch.channels_last)


def _ptr(t: Optional[torch.Tensor]) -> int:
    return 0 if t is None else t.data_ptr()


def _plan(lib, M: int, C: int):
    rpb = ctypes.c_int(0)
    G = lib.pto_bn_plan(M, C, ctypes.byref(rpb))
    if G <= 0:
        raise ValueError(f"batch_norm_act: unsupported channel count {C}")
    return G, rpb.value


class GradLink:
    """Out-of-band second gradient of a ``BatchNormAct2d`` output (see the module docstring).
    ``claimed``: a consumer took the residual role; ``dz``: the gradient it left for the
    producer's backward (consumed, then cleared, there)."""
    __slots__ = ("claimed", "dz")

    def __init__(self):
        self.claimed = False
        self.dz = None


class _BNAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, residual, running_mean, running_var, nbt, momentum, eps, relu,
                res_link=None, out_link=None):
        lib = _native.load()
        N, C, H, W = x.shape
        M = N * H * W
        xc = _nhwc(x, x.dtype)
        z = _nhwc(residual, x.dtype) if residual is not None else None
        y = torch.empty_like(xc, memory_format=torch.channels_last)
        G, rpb = _plan(lib, M, C)
        f32 = dict(device=x.device, dtype=torch.float32)
        part = torch.empty(G * (2 * C + 1), **f32)
        stats = torch.empty(4 * C, **f32)  # mean | rstd | scale | shift
        ctx.mask = 0 if not relu else (2 if residual is not None else 1)
        # ReLU after a residual add: the backward's mask comes from a 1-bit image written here
        # (M*C/8 bytes) instead of re-reading y in both backward passes
        bits = torch.empty(M * C // 8, dtype=torch.uint8, device=x.device) if ctx.mask == 2 and MASK_BITS else None
        _native.check(lib.pto_bn_fwd_train(
            xc.data_ptr(), _ptr(z), y.data_ptr(), weight.data_ptr(), bias.data_ptr(), _ptr(running_mean),
            _ptr(running_var), _ptr(nbt), stats.data_ptr(), stats[C:].data_ptr(), stats[2 * C:].data_ptr(),
            part.data_ptr(), M, C, G, rpb, float(momentum), float(eps), _DT[x.dtype], int(relu), _ptr(bits),
            _stream(x)), "bn_fwd_train")
        if bits is not None:
            ctx.mask = 3
        ctx.has_res = residual is not None
        ctx.res_dtype = residual.dtype if residual is not None else None
        ctx.plan = (M, C, G, rpb)
        ctx.res_link, ctx.out_link = res_link, out_link
        ctx.save_for_backward(xc, y if ctx.mask == 2 else bits, weight, stats)
        return y

    @staticmethod
    def backward(ctx, dy):
        lib = _native.load()
        xc, y, weight, stats = ctx.saved_tensors
        M, C, G, rpb = ctx.plan
        dyc = _nhwc(dy, xc.dtype)
        dy2 = None
        if ctx.out_link is not None and ctx.out_link.dz is not None:
            dy2, ctx.out_link.dz = _nhwc(ctx.out_link.dz, xc.dtype), None
        dx = torch.empty_like(xc, memory_format=torch.channels_last)
        dz = torch.empty_like(xc, memory_format=torch.channels_last) if ctx.has_res else None
        f32 = dict(device=xc.device, dtype=torch.float32)
        part = torch.empty(G * 2 * C, **f32)
        coef = torch.empty(3 * C, **f32)
        dgb = torch.empty(2 * C, **f32)
        _native.check(lib.pto_bn_bwd(
            dyc.data_ptr(), _ptr(dy2), xc.data_ptr(), _ptr(y), weight.data_ptr(), stats.data_ptr(), stats[C:].data_ptr(),
            stats[2 * C:].data_ptr(), dgb.data_ptr(), dgb[C:].data_ptr(), dx.data_ptr(), _ptr(dz), part.data_ptr(),
            coef.data_ptr(), M, C, G, rpb, _DT[xc.dtype], ctx.mask, _stream(xc)), "bn_bwd")
        dgamma, dbeta = dgb[:C].to(weight.dtype), dgb[C:].to(weight.dtype)
        if dz is not None and ctx.res_link is not None:
            # the producer of the residual adds this in its own backward kernels; the
            # autograd edge only orders the two backwards (no gradient sum pass)
            ctx.res_link.dz, dz = dz, None
        if dz is not None and dz.dtype != ctx.res_dtype:
            dz = dz.to(ctx.res_dtype)
        return dx, dgamma, dbeta, dz, None, None, None, None, None, None, None, None


class _LinkTap(torch.autograd.Function):
    """Identity whose backward hands the incoming gradient to ``link`` instead of autograd:
    the second consumer of a linked ``BatchNormAct2d`` output (e.g. a stage's downsample
    conv next to its conv1) leaves its input gradient for the producer's backward kernels,
    which add it to the first consumer's in fp32 (no separate gradient-sum pass)."""

    @staticmethod
    def forward(ctx, x, link):
        ctx.link = link
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        ctx.link.dz = g
        return None, None


def link_tap(x: torch.Tensor) -> torch.Tensor:
    """``x`` for a second consumer: if ``x`` is a linked ``batch_norm_act`` output whose link
    is unclaimed, the gradient flowing back through the result is summed inside the
    producer's backward; otherwise ``x`` itself (autograd sums the gradients as usual)."""
    link = getattr(x, "_pto_link", None)
    if link is None or link.claimed or not torch.is_grad_enabled() or not x.requires_grad:
        return x
    link.claimed = True
    return _LinkTap.apply(x, link)


def batch_norm_act(x, weight, bias, running_mean=None, running_var=None, num_batches_tracked=None,
                   training=True, momentum=0.1, eps=1e-5, relu=False, residual=None, impl="hip",
                   link_output=False):
    """``relu(batch_norm(x) [+ residual])`` (training statistics when ``training``).

    ``link_output``: the result carries a ``GradLink`` so that a later ``batch_norm_act``
    taking it as ``residual`` returns its residual gradient through the link and this op's
    backward sums it in-kernel.  A residual that carries a link is claimed by its first such
    consumer only (any other use goes through autograd as usual)."""
    if (impl != "hip" or not training or momentum is None or not supported(x) or weight is None
            or weight.dtype != torch.float32):
        if training and num_batches_tracked is not None:
            num_batches_tracked.add_(1)
        return reference(x, weight, bias, running_mean, running_var, training, momentum, eps, relu, residual)
    res_link = None
    if residual is not None and torch.is_grad_enabled() and residual.requires_grad:
        link = getattr(residual, "_pto_link", None)
        if (link is not None and not link.claimed and residual.dtype == x.dtype and residual.shape == x.shape
                and residual.is_contiguous(memory_format=torch.channels_last)):
            link.claimed, res_link = True, link
    out_link = GradLink() if link_output and torch.is_grad_enabled() else None
    y = _BNAct.apply(x, weight, bias, residual, running_mean, running_var, num_batches_tracked, momentum, eps,
                     relu, res_link, out_link)
    if out_link is not None:
        y._pto_link = out_link
    return y


class BatchNormAct2d(nn.BatchNorm2d):
    """``nn.BatchNorm2d`` + optional residual add + optional ReLU, one fused op on MI355X."""

    def __init__(self, num_features: int, relu: bool = False, link_output: bool = False, **kw):
        super().__init__(num_features, **kw)
        self.relu = relu
        self.impl = "hip"
        self.link_output = link_output  # output's second gradient summed in-kernel (GradLink)

    def forward(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None) -> torch.Tensor:
        training = self.training or not self.track_running_stats
        momentum = self.momentum
        if momentum is None and training and self.track_running_stats:
            return self._cumulative(x, residual)
        rm = self.running_mean if (not self.training or self.track_running_stats) else None
        rv = self.running_var if (not self.training or self.track_running_stats) else None
        nbt = self.num_batches_tracked if (self.training and self.track_running_stats) else None
        return batch_norm_act(x, self.weight, self.bias, rm, rv, nbt, training, momentum if momentum is not None else 0.0,
                              self.eps, self.relu, residual, self.impl, self.link_output)

    def _cumulative(self, x, residual):
        self.num_batches_tracked.add_(1)
        f = 1.0 / float(self.num_batches_tracked)
        return reference(x, self.weight, self.bias, self.running_mean, self.running_var, True, f, self.eps,
                         self.relu, residual)

    def extra_repr(self) -> str:
        return super().extra_repr() + f", relu={self.relu}"
