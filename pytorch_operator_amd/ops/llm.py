"""Fused RoPE and SwiGLU (``csrc/kernels/llm_fused.hip``) as autograd ops for the Llama worker.

``rope(x, cos, sin)``: ``x`` [B, S, H, D] (fp32 or bf16, contiguous), tables [S, D/2] fp32;
rotates adjacent pairs like Meta's complex formulation.  The backward is the same kernel
with the rotation negated.  ``swiglu(a, b)`` = ``silu(a) * b`` with a one-pass backward.

On a GPU the HIP kernels run (a missing library is an error, never a silent fallback); on
CPU the same math runs in PyTorch (CPU tests and the gloo plumbing config).
"""
from __future__ import annotations

import ctypes

import torch
import torch.nn.functional as F

from . import _native

_DT = {torch.float32: 0, torch.bfloat16: 1}


def _stream(t: torch.Tensor):
    return ctypes.c_void_p(_native.current_stream_ptr(t.device))


def _aligned(t: torch.Tensor) -> torch.Tensor:
    t = t.contiguous()
    return t if t.data_ptr() % 16 == 0 else t.clone()


# ------------------------------------------------------------------------------------ rope
def rope_reference(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    xf = x.float().reshape(*x.shape[:-1], -1, 2)
    x0, x1 = xf[..., 0], xf[..., 1]
    c = cos[None, :, None, :]
    s = sin[None, :, None, :]
    out = torch.stack((x0 * c - x1 * s, x0 * s + x1 * c), dim=-1)
    return out.flatten(-2).type_as(x)


def _rope_launch(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, sign: float) -> torch.Tensor:
    B, S, H, D = x.shape
    y = torch.empty_like(x)
    _native.check(_native.load().pto_rope(x.data_ptr(), cos.data_ptr(), sin.data_ptr(), y.data_ptr(), B * S * H, H,
                                          S, D, sign, _DT[x.dtype], _stream(x)), "rope")
    return y


class _Rope(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, cos, sin):
        ctx.save_for_backward(cos, sin)
        return _rope_launch(x, cos, sin, 1.0)

    @staticmethod
    def backward(ctx, dy):
        cos, sin = ctx.saved_tensors
        return _rope_launch(_aligned(dy), cos, sin, -1.0), None, None


def rope(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    if not x.is_cuda:
        return rope_reference(x, cos, sin)
    if x.dim() != 4 or x.dtype not in _DT or x.shape[-1] % 8 or cos.shape != (x.shape[1], x.shape[3] // 2):
        raise ValueError(f"rope: x [B,S,H,D] fp32/bf16 with D % 8 == 0 and tables [S, D/2]; got {tuple(x.shape)}")
    return _Rope.apply(_aligned(x), _aligned(cos.float()), _aligned(sin.float()))


# --------------------------------------------------------------------------------- rope_qkv
def rope_qkv_reference(qkv: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, hq: int, hkv: int):
    B, S, W = qkv.shape
    D = W // (hq + 2 * hkv)
    q, k, v = qkv.split([hq * D, hkv * D, hkv * D], dim=-1)
    return (rope_reference(q.reshape(B, S, hq, D), cos, sin), rope_reference(k.reshape(B, S, hkv, D), cos, sin),
            v.reshape(B, S, hkv, D))


def _rope_qkv_launch(packed, q, k, v, cos, sin, S, hq, hkv, D, direction):
    _native.check(_native.load().pto_rope_qkv(packed.data_ptr(), q.data_ptr(), k.data_ptr(), v.data_ptr(),
                                              cos.data_ptr(), sin.data_ptr(), packed.numel() // packed.shape[-1],
                                              S, hq, hkv, D, direction, _DT[packed.dtype], _stream(packed)),
                  "rope_qkv")


class _RopeQKV(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, cos, sin, hq, hkv):
        B, S, W = qkv.shape
        D = W // (hq + 2 * hkv)
        q = qkv.new_empty(B, S, hq, D)
        k = qkv.new_empty(B, S, hkv, D)
        v = qkv.new_empty(B, S, hkv, D)
        _rope_qkv_launch(qkv, q, k, v, cos, sin, S, hq, hkv, D, 0)
        ctx.save_for_backward(cos, sin)
        ctx.dims = (B, S, W, hq, hkv, D)
        return q, k, v

    @staticmethod
    def backward(ctx, dq, dk, dv):
        cos, sin = ctx.saved_tensors
        B, S, W, hq, hkv, D = ctx.dims
        ref = next(t for t in (dq, dk, dv) if t is not None)
        dq = _aligned(dq) if dq is not None else ref.new_zeros(B, S, hq, D)
        dk = _aligned(dk) if dk is not None else ref.new_zeros(B, S, hkv, D)
        dv = _aligned(dv) if dv is not None else ref.new_zeros(B, S, hkv, D)
        dt = dq.dtype
        dk, dv = dk.to(dt), dv.to(dt)
        dqkv = dq.new_empty(B, S, W)
        _rope_qkv_launch(dqkv, dq, dk, dv, cos, sin, S, hq, hkv, D, 1)
        return dqkv, None, None, None, None


def rope_qkv(qkv: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, hq: int, hkv: int):
    """Split the fused QKV projection's output [B, S, (hq + 2 hkv) * D] into contiguous
    q [B, S, hq, D], k, v [B, S, hkv, D] with RoPE applied to q and k -- one HBM pass, and
    one pass back to a packed d(qkv) in the backward (so the three input-gradient matmuls
    become one and no gradient sum is needed)."""
    if not qkv.is_cuda:
        return rope_qkv_reference(qkv, cos, sin, hq, hkv)
    B, S, W = qkv.shape
    if qkv.dtype not in _DT or W % (hq + 2 * hkv) or (W // (hq + 2 * hkv)) % 8 or \
            cos.shape != (S, W // (hq + 2 * hkv) // 2):
        raise ValueError(f"rope_qkv: bad shapes qkv {tuple(qkv.shape)} cos {tuple(cos.shape)} hq {hq} hkv {hkv}")
    return _RopeQKV.apply(_aligned(qkv), _aligned(cos.float()), _aligned(sin.float()), hq, hkv)


# ---------------------------------------------------------------------------------- swiglu
def swiglu_reference(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    return F.silu(a) * b


class _SwiGLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        y = torch.empty_like(a)
        _native.check(_native.load().pto_swiglu_fwd(a.data_ptr(), b.data_ptr(), y.data_ptr(), a.numel(),
                                                    _DT[a.dtype], _stream(a)), "swiglu_fwd")
        ctx.save_for_backward(a, b)
        return y

    @staticmethod
    def backward(ctx, dy):
        a, b = ctx.saved_tensors
        dy = _aligned(dy.to(a.dtype))
        da, db = torch.empty_like(a), torch.empty_like(b)
        _native.check(_native.load().pto_swiglu_bwd(dy.data_ptr(), a.data_ptr(), b.data_ptr(), da.data_ptr(),
                                                    db.data_ptr(), a.numel(), _DT[a.dtype], _stream(a)),
                      "swiglu_bwd")
        return da, db


def swiglu(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    if not a.is_cuda:
        return swiglu_reference(a, b)
    if a.shape != b.shape or a.dtype != b.dtype or a.dtype not in _DT:
        raise ValueError("swiglu: a and b must share shape and dtype (fp32/bf16)")
    return _SwiGLU.apply(_aligned(a), _aligned(b))


def swiglu_packed_reference(x: torch.Tensor) -> torch.Tensor:
    a, b = x.chunk(2, dim=-1)
    return F.silu(a) * b


class _SwiGLUPacked(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        F2 = x.shape[-1]
        y = x.new_empty(*x.shape[:-1], F2 // 2)
        _native.check(_native.load().pto_swiglu_packed_fwd(x.data_ptr(), y.data_ptr(), x.numel() // F2, F2 // 2,
                                                           _DT[x.dtype], _stream(x)), "swiglu_packed_fwd")
        ctx.save_for_backward(x)
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        dy = _aligned(dy.to(x.dtype))
        dx = torch.empty_like(x)
        F2 = x.shape[-1]
        _native.check(_native.load().pto_swiglu_packed_bwd(dy.data_ptr(), x.data_ptr(), dx.data_ptr(),
                                                           x.numel() // F2, F2 // 2, _DT[x.dtype], _stream(x)),
                      "swiglu_packed_bwd")
        return dx


def swiglu_packed(x: torch.Tensor) -> torch.Tensor:
    """``silu(a) * b`` of the fused W1|W3 projection's output x = [a | b] (last dim 2F)."""
    if not x.is_cuda:
        return swiglu_packed_reference(x)
    if x.dtype not in _DT or x.shape[-1] % 16:
        raise ValueError(f"swiglu_packed: fp32/bf16 with last dim % 16 == 0, got {tuple(x.shape)} {x.dtype}")
    return _SwiGLUPacked.apply(_aligned(x))


# ---------------------------------------------------------------------------- cross-entropy
_IGNORE = -100


def cross_entropy_reference(logits: torch.Tensor, targets: torch.Tensor) -> torch.Tensor:
    return F.cross_entropy(logits.float(), targets, ignore_index=_IGNORE)


class _CrossEntropy(torch.autograd.Function):
    """Mean cross-entropy of [N, V] logits: the forward reads the logits once (per-row lse,
    per-row loss).  The backward writes d(logits) into a fresh tensor, or -- ``overwrite``,
    the Llama training path -- over the saved logits in place (an intermediate only this op
    consumes there: the lm-head matmul's backward needs its input and weight, not its output;
    saves one [N, V] buffer, 1 GB at Llama-3 8B batch 4).  In place, the logits' version
    counter is bumped, so autograd rejects any later use of the overwritten tensor."""

    @staticmethod
    def forward(ctx, logits, targets, overwrite):
        N, V = logits.shape
        lse = torch.empty(N, device=logits.device, dtype=torch.float32)
        loss = torch.empty(N, device=logits.device, dtype=torch.float32)
        tgt = targets.contiguous().long()
        _native.check(_native.load().pto_xent_fwd(logits.data_ptr(), tgt.data_ptr(), lse.data_ptr(),
                                                  loss.data_ptr(), N, V, _IGNORE, _DT[logits.dtype],
                                                  _stream(logits)), "xent_fwd")
        count = (tgt != _IGNORE).sum().clamp_min(1).float()
        ctx.save_for_backward(logits, tgt, lse, count)
        ctx.overwrite = bool(overwrite)
        return loss.sum() / count

    @staticmethod
    def backward(ctx, g):
        if getattr(ctx, "consumed", False):
            raise RuntimeError("fused cross_entropy(overwrite_logits=True): the logits were overwritten by the "
                               "first backward (retain_graph double backward is not supported)")
        logits, tgt, lse, count = ctx.saved_tensors
        N, V = logits.shape
        scale = (g.float() / count).reshape(1).contiguous()
        out = logits if ctx.overwrite else torch.empty_like(logits)
        _native.check(_native.load().pto_xent_bwd(logits.data_ptr(), tgt.data_ptr(), lse.data_ptr(),
                                                  scale.data_ptr(), out.data_ptr(), N, V, _IGNORE,
                                                  _DT[logits.dtype], _stream(logits)), "xent_bwd")
        if ctx.overwrite:
            ctx.consumed = True
            torch.autograd.graph.increment_version(logits)  # the kernel wrote it behind autograd's back
        return out, None, None


def cross_entropy(logits: torch.Tensor, targets: torch.Tensor, *, overwrite_logits: bool = False) -> torch.Tensor:
    """Mean token cross-entropy (ignore_index -100) over [N, V] logits in their own dtype
    (fp32 math inside the kernels).  GPU: the fused HIP kernels; CPU: PyTorch.

    ``overwrite_logits=True`` lets the backward write d(logits) over ``logits`` (no extra
    [N, V] buffer); only for callers that never read the logits after backward."""
    if logits.is_cuda and logits.dtype in _DT and logits.shape[-1] % 8 == 0 and logits.dim() == 2:
        return _CrossEntropy.apply(_aligned(logits), targets, overwrite_logits)
    return cross_entropy_reference(logits, targets)


# ---------------------------------------------------------------------------- TN linear
def transpose2d(x: torch.Tensor) -> torch.Tensor:
    """Contiguous transpose of a 2-D bf16 matrix (HIP LDS-tiled kernel when both dims are
    multiples of 64, PyTorch's copy otherwise)."""
    R, C = x.shape
    if not x.is_cuda or x.dtype != torch.bfloat16 or R % 64 or C % 64 or R // 64 > 65535:
        return x.t().contiguous()
    x = _aligned(x)
    out = torch.empty((C, R), device=x.device, dtype=x.dtype)
    _native.check(_native.load().pto_transpose16(x.data_ptr(), out.data_ptr(), R, C, _stream(x)), "transpose16")
    return out


class _LinearTN(torch.autograd.Function):
    """y = x.W^T whose backward GEMMs are issued with both operands K-contiguous -- the
    layout hipBLASLt runs fastest on MI355X (tools/gemm_layout_probe.py) -- instead of
    autograd's dy.W (W K-strided) and dy^T.x (both K-strided): dX = dy.(W^T)^T and
    dW = (dy^T).(x^T)^T, with the transposed copies made by one LDS-tiled pass each."""

    @staticmethod
    def forward(ctx, x, w):
        x2 = x.reshape(-1, x.shape[-1])
        ctx.save_for_backward(x2, w)
        ctx.xshape = x.shape
        # a gradient sink (parallel/zero.py, gradient-as-bucket-view): dW is written by the
        # GEMM straight into the optimizer's bucket slot -- no .grad tensor, no copy pass
        ctx.sink = getattr(w, "_pto_grad_sink", None)
        return F.linear(x2, w).view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, w = ctx.saved_tensors
        dy2 = _aligned(dy.reshape(-1, w.shape[0]).to(x2.dtype))
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = F.linear(dy2, transpose2d(w)).view(ctx.xshape)
        if ctx.needs_input_grad[1]:
            sink = ctx.sink
            if sink is not None and sink.dtype == x2.dtype and sink.shape == tuple(w.shape):
                torch.mm(transpose2d(dy2), transpose2d(x2).t(), out=sink.view)
                sink.ready()
            else:
                dw = F.linear(transpose2d(dy2), transpose2d(x2))
        return dx, dw


def linear_tn(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """``F.linear(x, w)`` (no bias) with K-contiguous backward GEMMs on a GPU; under bf16
    autocast both operands are taken in bf16 (as autocast's linear would)."""
    if not x.is_cuda:
        return F.linear(x, w)
    if torch.is_autocast_enabled("cuda"):
        dt = torch.get_autocast_dtype("cuda")
        with torch.autocast(device_type="cuda", enabled=False):
            return _LinearTN.apply(x.to(dt), w.to(dt))
    if x.dtype != torch.bfloat16 or w.dtype != torch.bfloat16:
        return F.linear(x, w)
    return _LinearTN.apply(x, w)
