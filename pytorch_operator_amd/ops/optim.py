"""Mixed-precision AdamW with fp32 master weights (``csrc/kernels/adamw.hip``).

``to_bf16_matmul_weights(model)`` turns every ``nn.Linear`` weight into bf16 -- the
tensors the bf16 autocast matmuls read directly, so the per-step fp32->bf16 weight casts
and bf16->fp32 gradient casts disappear -- and ``MasterAdamW`` keeps an fp32 master copy
of those weights plus fp32 moments.  Other parameters (embedding, RMSNorm weights) stay
fp32 and are their own master.  One fused HIP pass per parameter updates master, m, v
and rewrites the bf16 weight.  Update rule = ``torch.optim.AdamW`` (decoupled decay,
bias-corrected moments), applied to the fp32 master.

On CPU the same update runs in PyTorch (CPU tests, gloo plumbing).
"""
from __future__ import annotations

import ctypes
import math

import torch
import torch.nn as nn

from . import _native


def to_bf16_matmul_weights(model: nn.Module) -> int:
    """Cast ``nn.Linear`` weights (and biases) of ``model`` to bf16 in place; returns #params cast."""
    n = 0
    for mod in model.modules():
        if isinstance(mod, nn.Linear):
            for p in mod.parameters(recurse=False):
                if p.dtype == torch.bfloat16:
                    continue
                master = p.data.float()
                p.data = p.data.to(torch.bfloat16)
                p._pto_master = master  # exact fp32 init for MasterAdamW (dropped once it takes over)
                n += p.numel()
    return n


class MasterAdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))

    def _state(self, p):
        st = self.state[p]
        if not st:
            st["step"] = 0
            if p.dtype != torch.float32:
                st["master"] = getattr(p, "_pto_master", None)
                if st["master"] is None:
                    st["master"] = p.detach().float().clone()
                else:
                    del p._pto_master
            else:
                st["master"] = None
            st["exp_avg"] = torch.zeros(p.shape, dtype=torch.float32, device=p.device)
            st["exp_avg_sq"] = torch.zeros(p.shape, dtype=torch.float32, device=p.device)
        return st

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            lr, (b1, b2), eps, wd = group["lr"], group["betas"], group["eps"], group["weight_decay"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.dtype not in (torch.float32, torch.bfloat16):
                    raise TypeError(f"MasterAdamW: fp32/bf16 parameters only, got {p.dtype}")
                st = self._state(p)
                st["step"] += 1
                master = st["master"] if st["master"] is not None else p
                # the DDP fp32 comm hook's reduced gradient (harness/ddp_train.py), else .grad
                g32 = getattr(p, "_pto_grad32", None)
                if g32 is not None:
                    del p._pto_grad32
                g = g32 if g32 is not None else p.grad
                if p.is_cuda:
                    self._step_hip(p, g, master, st, lr, b1, b2, eps, wd)
                else:
                    self._step_reference(p, g, master, st, lr, b1, b2, eps, wd)
        return loss

    @staticmethod
    def _step_reference(p, g, master, st, lr, b1, b2, eps, wd):
        g = g.float()
        t = st["step"]
        master.mul_(1 - lr * wd)
        st["exp_avg"].lerp_(g, 1 - b1)
        st["exp_avg_sq"].mul_(b2).addcmul_(g, g, value=1 - b2)
        denom = (st["exp_avg_sq"].sqrt() / math.sqrt(1 - b2 ** t)).add_(eps)
        master.addcdiv_(st["exp_avg"], denom, value=-lr / (1 - b1 ** t))
        if master is not p:
            p.copy_(master)

    @staticmethod
    def _step_hip(p, g, master, st, lr, b1, b2, eps, wd):
        if not g.is_contiguous() or g.data_ptr() % 16:
            g = g.contiguous().clone()
        if g.dtype not in (torch.float32, torch.bfloat16) or not p.is_contiguous():
            raise TypeError("MasterAdamW: contiguous fp32/bf16 parameters and gradients only")
        out = p.data_ptr() if master is not p else None
        stream = ctypes.c_void_p(torch.cuda.current_stream(p.device).cuda_stream)
        _native.check(_native.load().pto_adamw_step(
            master.data_ptr(), st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr(), g.data_ptr(), out,
            p.numel(), 1 if g.dtype == torch.bfloat16 else 0, lr, b1, b2, eps, wd, st["step"], stream),
            "adamw_step")
