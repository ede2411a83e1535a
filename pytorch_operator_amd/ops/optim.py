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
    """``overlap=True`` (GPU): ``step()`` enqueues the updates on a side stream, in parameter
    order, and returns at once; each parameter gets a ready event, and ``install_overlap
    (model)`` makes every module wait (on the compute stream) for its own parameters' events
    just before its forward.  The next step's forward then starts while the updates of the
    later layers are still streaming -- the memory-bound optimizer (~11 % of a Llama-3 8B
    step) runs under the compute-bound forward GEMMs instead of after them."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, overlap=False):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self.overlap = overlap
        self._side = None

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
        side = None
        for group in self.param_groups:
            for p in group["params"]:
                if self.overlap and p.is_cuda and p.grad is not None:
                    if self._side is None:
                        self._side = torch.cuda.Stream(device=p.device)
                    side = self._side
                    side.wait_stream(torch.cuda.current_stream(p.device))  # gradients complete
                break
            if side is not None:
                break
        if side is None:
            self._step_all(None)
        else:
            with torch.cuda.stream(side):
                self._step_all(side)
        return loss

    def _step_all(self, side):
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
                    if side is not None:
                        g.record_stream(side)  # the next backward may reuse the memory otherwise
                    self._step_hip(p, g, master, st, lr, b1, b2, eps, wd)
                    if side is not None:
                        ev = torch.cuda.Event()
                        ev.record(side)
                        p._pto_ready = ev
                else:
                    self._step_reference(p, g, master, st, lr, b1, b2, eps, wd)


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


def install_overlap(model: nn.Module) -> int:
    """Forward pre-hooks: each module with parameters of its own makes the current stream wait
    for those parameters' optimizer-update events (``MasterAdamW(overlap=True)``); returns the
    number of hooked modules."""
    def hook(mod, _inputs):
        for p in mod.parameters(recurse=False):
            ev = getattr(p, "_pto_ready", None)
            if ev is not None:
                torch.cuda.current_stream(p.device).wait_event(ev)
    n = 0
    for mod in model.modules():
        if any(True for _ in mod.parameters(recurse=False)):
            mod.register_forward_pre_hook(hook)
            n += 1
    return n
