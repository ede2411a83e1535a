"""Flash attention (``csrc/kernels/attention.hip``) as an autograd op for the Llama worker.

``flash_attention(q, k, v, causal=True)``: q [B, S, Hq, D], k/v [B, S, Hkv, D] (GQA when
Hkv < Hq), token-major like the projections that produce them, so no transposes or copies
surround the kernels; returns o [B, S, Hq, D] (``o.reshape(B, S, Hq * D)`` feeds the output
projection).  Scale 1/sqrt(D).

The HIP path covers the Llama-3 attention shapes: bf16, D = 128, S a multiple of 128
(``hip_supported``).  The forward keeps lse2 = log2-sum-exp of the scaled scores per query
row; the backward is two launches (dQ with delta = rowsum(dO * O), then dK/dV), both
deterministic.  On CPU the same math runs in PyTorch (``attention_reference``); a GPU call
with an unsupported shape raises instead of falling back silently.
"""
from __future__ import annotations

import ctypes
import math

import torch
import torch.nn.functional as F

from . import _native

HEAD_DIM = 128
SEQ_MULTIPLE = 128


def _stream(t: torch.Tensor):
    return ctypes.c_void_p(_native.current_stream_ptr(t.device))


def _c(t: torch.Tensor) -> torch.Tensor:
    t = t.contiguous()
    return t if t.data_ptr() % 16 == 0 else t.clone()


def hip_supported(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor) -> bool:
    if not (q.is_cuda and k.is_cuda and v.is_cuda) or q.dim() != 4:
        return False
    B, S, Hq, D = q.shape
    return (q.dtype == k.dtype == v.dtype == torch.bfloat16 and D == HEAD_DIM and S % SEQ_MULTIPLE == 0
            and k.shape == v.shape and k.shape[0] == B and k.shape[1] == S and k.shape[3] == D
            and Hq % k.shape[2] == 0)


def attention_reference(q, k, v, causal: bool = True, return_lse: bool = False):
    """fp32 math on [B, S, H, D] tensors; lse in natural-log units of the scaled scores."""
    B, S, Hq, D = q.shape
    G = Hq // k.shape[2]
    qf = q.float().transpose(1, 2)
    kf = k.float().repeat_interleave(G, dim=2).transpose(1, 2)
    vf = v.float().repeat_interleave(G, dim=2).transpose(1, 2)
    s = (qf @ kf.transpose(-1, -2)) / math.sqrt(D)
    if causal:
        s = s.masked_fill(torch.ones(S, S, dtype=torch.bool, device=q.device).triu(1), float("-inf"))
    lse = torch.logsumexp(s, dim=-1)
    o = (torch.softmax(s, dim=-1) @ vf).transpose(1, 2).to(q.dtype)
    return (o, lse) if return_lse else o


class _FlashAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, causal):
        B, S, Hq, D = q.shape
        Hkv = k.shape[2]
        o = torch.empty_like(q)
        lse2 = torch.empty(B, Hq, S, dtype=torch.float32, device=q.device)
        scale = 1.0 / math.sqrt(D)
        _native.check(_native.load().pto_attn_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(),
                                                  lse2.data_ptr(), B, S, Hq, Hkv, D, scale, int(causal),
                                                  _stream(q)), "attn_fwd")
        ctx.save_for_backward(q, k, v, o, lse2)
        ctx.causal = causal
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse2 = ctx.saved_tensors
        B, S, Hq, D = q.shape
        Hkv = k.shape[2]
        do = _c(do.to(q.dtype))
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        delta = torch.empty_like(lse2)
        _native.check(_native.load().pto_attn_bwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(),
                                                  do.data_ptr(), lse2.data_ptr(), delta.data_ptr(), dq.data_ptr(),
                                                  dk.data_ptr(), dv.data_ptr(), B, S, Hq, Hkv, D,
                                                  1.0 / math.sqrt(D), int(ctx.causal), _stream(q)), "attn_bwd")
        return dq, dk, dv, None


def flash_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, causal: bool = True) -> torch.Tensor:
    if not q.is_cuda:
        return attention_reference(q, k, v, causal)
    if not hip_supported(q, k, v):
        raise ValueError(f"flash_attention: HIP path needs bf16 [B,S,H,{HEAD_DIM}] with S % {SEQ_MULTIPLE} == 0 "
                         f"and Hq % Hkv == 0; got q {tuple(q.shape)} {q.dtype}, k {tuple(k.shape)}")
    return _FlashAttention.apply(_c(q), _c(k), _c(v), bool(causal))


def sdpa_bshd(q, k, v, causal: bool = True) -> torch.Tensor:
    """The library path on the same [B, S, H, D] layout (A/B baseline and non-HIP shapes)."""
    o = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), is_causal=causal,
                                       enable_gqa=k.shape[2] != q.shape[2])
    return o.transpose(1, 2)
