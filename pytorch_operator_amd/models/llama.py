"""Llama-3 decoder for the BASELINE "Llama-3 8B DDP bf16" PyTorchJob config.

Not part of the reference (MNIST only); BASELINE.json names it as the large-model job
shape: Master=1 Worker=7, 288 GB HBM sizing, OnFailure restarts + gang scheduling.
Plain DDP fits on MI355X: 8.0 B parameters in fp32 (32 GB) + fp32 grads (32 GB) + AdamW
moments (64 GB) + bf16 activations for a 2 k-token sequence stay well inside 288 GB, so
no sharding is needed -- every rank keeps the whole model and only gradients cross xGMI.

Architecture (Meta's reference layout): token embedding, ``n_layers`` x [RMSNorm ->
GQA attention with RoPE (theta 500 000) -> residual, RMSNorm -> SwiGLU FFN -> residual],
final RMSNorm, untied output projection.  Matmuls run in bf16 under autocast
(hipBLASLt); attention runs the hand-written HIP flash attention (``ops.attention``, forward
and backward on MFMA, token-major [B, S, H, D] in and out, so no transposes around it) for
bf16 head_dim-128 shapes and ``scaled_dot_product_attention`` otherwise (``impl`` = "sdpa"
forces the library path for A/B runs).
The elementwise work between the matmuls runs as hand-written HIP kernels on a GPU:
RMSNorm (``ops.norm``, fp32 statistics over the fp32 residual stream, bf16 output under
autocast so the next matmul reads it directly), RoPE and SwiGLU (``ops.llm``, one HBM pass
each, fwd and bwd).  On CPU the same math runs in PyTorch.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F


@dataclass
class LlamaConfig:
    dim: int = 4096
    n_layers: int = 32
    n_heads: int = 32
    n_kv_heads: int = 8
    vocab_size: int = 128256
    ffn_hidden: int = 14336
    norm_eps: float = 1e-5
    rope_theta: float = 500000.0
    max_seq_len: int = 8192

    @property
    def head_dim(self) -> int:
        return self.dim // self.n_heads

    def num_params(self) -> int:
        d, f, v, L = self.dim, self.ffn_hidden, self.vocab_size, self.n_layers
        kv = self.n_kv_heads * self.head_dim
        per_layer = d * d * 2 + d * kv * 2 + 3 * d * f + 2 * d
        return L * per_layer + 2 * v * d + d


CONFIGS = {
    "llama3-8b": LlamaConfig(),
    "llama3-1b": LlamaConfig(dim=2048, n_layers=16, n_heads=32, n_kv_heads=8, ffn_hidden=8192),
    "llama-tiny": LlamaConfig(dim=64, n_layers=2, n_heads=4, n_kv_heads=2, vocab_size=256, ffn_hidden=128,
                              max_seq_len=256),
    # smallest config with the 8B model's head_dim (128): exercises the HIP flash attention
    "llama-mini": LlamaConfig(dim=512, n_layers=2, n_heads=4, n_kv_heads=2, vocab_size=512, ffn_hidden=1024,
                              max_seq_len=1024),
}


def rope_tables(head_dim: int, seq_len: int, theta: float, device=None):
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, device=device, dtype=torch.float32) / head_dim))
    t = torch.arange(seq_len, device=device, dtype=torch.float32)
    ang = torch.outer(t, inv)  # [S, D/2]
    return torch.cos(ang), torch.sin(ang)


def apply_rope(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    """x [B, S, H, D]; rotates adjacent pairs (x0, x1) like Meta's complex formulation."""
    from ..ops.llm import rope
    return rope(x, cos, sin)


class RMSNorm(nn.Module):
    def __init__(self, dim: int, eps: float = 1e-5):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(dim))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        from ..ops.norm import rms_norm
        out_dtype = None
        if x.is_cuda and x.dtype == torch.float32 and torch.is_autocast_enabled("cuda"):
            out_dtype = torch.get_autocast_dtype("cuda")  # consumed by a bf16 matmul next
        return rms_norm(x, self.weight, self.eps, out_dtype)

    fuse_residual = True  # False: plain add + norm (A/B of the residual-fused kernels)

    def add_forward(self, x: torch.Tensor, delta: Optional[torch.Tensor]):
        """(x + delta, norm(x + delta)) -- the residual add fused into this norm."""
        if delta is None:
            return x, self(x)
        if not self.fuse_residual:
            s = x + delta
            return s, self(s)
        from ..ops.norm import add_rms_norm
        out_dtype = None
        if x.is_cuda and x.dtype == torch.float32 and torch.is_autocast_enabled("cuda"):
            out_dtype = torch.get_autocast_dtype("cuda")
        return add_rms_norm(x, delta, self.weight, self.eps, out_dtype)


class TNLinear(nn.Linear):
    """Bias-free projection whose backward GEMMs take K-contiguous operands (``ops.llm.linear_tn``)
    when ``impl == "tn"``; ``"autograd"`` is the plain ``nn.Linear`` backward (A/B)."""

    impl = "tn"

    def __init__(self, fin: int, fout: int):
        super().__init__(fin, fout, bias=False)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.impl == "tn" and x.is_cuda:
            from ..ops.llm import linear_tn
            return linear_tn(x, self.weight)
        return super().forward(x)


class Attention(nn.Module):
    impl = "auto"  # "auto": HIP flash attention where it applies; "sdpa": library kernels

    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.nh, self.nkv, self.hd = cfg.n_heads, cfg.n_kv_heads, cfg.head_dim
        # one fused Q|K|V projection: one GEMM (N = (Hq + 2 Hkv) * D) forward and one for
        # the input gradient backward, instead of three plus a gradient sum
        self.wqkv = TNLinear(cfg.dim, (self.nh + 2 * self.nkv) * self.hd)
        self.wo = TNLinear(self.nh * self.hd, cfg.dim)

    def forward(self, x, cos, sin):
        B, S, _ = x.shape
        from ..ops import attention as A
        from ..ops.llm import rope_qkv
        q, k, v = rope_qkv(self.wqkv(x), cos, sin, self.nh, self.nkv)
        if self.impl != "sdpa" and A.hip_supported(q, k, v):
            o = A.flash_attention(q, k, v, causal=True)  # [B, S, H, D], no transposes
        else:
            o = A.sdpa_bshd(q, k, v, causal=True)
        return self.wo(o.reshape(B, S, self.nh * self.hd))


class FeedForward(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        # fused W1|W3 (gate | up) projection: one GEMM each way, packed SwiGLU between
        self.w13 = TNLinear(cfg.dim, 2 * cfg.ffn_hidden)
        self.w2 = TNLinear(cfg.ffn_hidden, cfg.dim)

    def forward(self, x):
        from ..ops.llm import swiglu_packed
        return self.w2(swiglu_packed(self.w13(x)))


class Block(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.attention_norm = RMSNorm(cfg.dim, cfg.norm_eps)
        self.attention = Attention(cfg)
        self.ffn_norm = RMSNorm(cfg.dim, cfg.norm_eps)
        self.feed_forward = FeedForward(cfg)

    def forward(self, x, delta, cos, sin):
        """x: residual stream entering the block minus the previous block's FFN output
        ``delta`` (None for the first block): each residual add happens inside the next
        RMSNorm.  Returns (residual stream before the FFN add, FFN output)."""
        h, y = self.attention_norm.add_forward(x, delta)
        h, y = self.ffn_norm.add_forward(h, self.attention(y, cos, sin))
        return h, self.feed_forward(y)


class Llama(nn.Module):
    def __init__(self, cfg: LlamaConfig, checkpoint_layers: bool = False):
        super().__init__()
        self.cfg = cfg
        self.checkpoint_layers = checkpoint_layers
        self.tok_embeddings = nn.Embedding(cfg.vocab_size, cfg.dim)
        self.layers = nn.ModuleList(Block(cfg) for _ in range(cfg.n_layers))
        self.norm = RMSNorm(cfg.dim, cfg.norm_eps)
        self.output = nn.Linear(cfg.dim, cfg.vocab_size, bias=False)
        self.reset_parameters()

    @torch.no_grad()
    def reset_parameters(self, std: float = 0.02):
        for m in self.modules():
            if isinstance(m, (nn.Linear, nn.Embedding)):
                nn.init.normal_(m.weight, std=std)
        # scaled init of the residual projections (GPT-2 / Llama practice)
        for blk in self.layers:
            nn.init.normal_(blk.attention.wo.weight, std=std / math.sqrt(2 * self.cfg.n_layers))
            nn.init.normal_(blk.feed_forward.w2.weight, std=std / math.sqrt(2 * self.cfg.n_layers))

    def forward(self, tokens: torch.Tensor, targets: Optional[torch.Tensor] = None):
        B, S = tokens.shape
        cos, sin = rope_tables(self.cfg.head_dim, S, self.cfg.rope_theta, tokens.device)
        h, d = self.tok_embeddings(tokens), None
        for blk in self.layers:
            if self.checkpoint_layers and self.training:
                h, d = torch.utils.checkpoint.checkpoint(blk, h, d, cos, sin, use_reentrant=False)
            else:
                h, d = blk(h, d, cos, sin)
        logits = self.output(self.norm.add_forward(h, d)[1])
        if targets is None:
            return logits
        from ..ops.llm import cross_entropy
        # the logits are this op's own intermediate: d(logits) may overwrite them
        return cross_entropy(logits.reshape(-1, logits.shape[-1]), targets.reshape(-1), overwrite_logits=True)
