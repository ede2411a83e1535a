"""Data-parallel gradient synchronisation designed for 8x MI355X over xGMI.

The reference wraps its model in ``nn.parallel.DistributedDataParallel``
(examples/mnist/mnist.py:133-138): per-parameter autograd hooks fill 25 MB
buckets and each full bucket is all-reduced.  On one 8-GPU MI355X node every GPU
pair has its own xGMI link (7 links x ~153 GB/s per GPU), so the collective for
this model (431 080 fp32 = 1.72 MB) is latency-bound, not bandwidth-bound: the
right shape is *as few collectives as possible, as early as possible*.

``FlatGradAllReduce`` is the fused-trainer path: gradients already live in one
flat buffer, split into exactly two buckets in backward-production order -- the
fc bucket (fc1+fc2, 93.9 % of the bytes, ready after the fc1 backward launch) and
the conv bucket (ready after the conv backward launch).  The fc all-reduce is
issued on RCCL's stream while the conv backward kernel still runs; SGD waits for
both (``finish``) and folds the 1/world average into its update.

At world 1 the collectives are skipped unless ``force`` (or ``PTO_FORCE_COLLECTIVES=1``) is
set: then both bucket all-reduces are really issued on the (single-rank) process group, so the
RCCL step forms -- stream-launched pieces and the one-graph ``graph-comm`` step -- run under a
real RCCL communicator on a one-GPU box (their single-rank floor; ``tools/rccl_w1_check.py``).

``BucketedDDP`` is the generic path for arbitrary ``nn.Module`` s (the ResNet /
Llama configs, the CPU gloo plumbing): gradient hooks copy each parameter's grad
into a flat bucket buffer in reverse-registration order and launch the bucket's
all-reduce the moment it fills, exactly one collective per bucket.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional

import torch
import torch.distributed as dist
import torch.nn as nn


def forced_collectives() -> bool:
    """``PTO_FORCE_COLLECTIVES=1``: issue the gradient collectives even at world 1."""
    return os.environ.get("PTO_FORCE_COLLECTIVES", "0") not in ("", "0")


class FlatGradAllReduce:
    """Two-bucket overlapped all-reduce hooks for ``FusedMnistTrainer``."""

    def __init__(self, group=None, compress_bf16: bool = False, force: Optional[bool] = None):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.compress_bf16 = compress_bf16
        if force is None:
            force = forced_collectives()
        if force and not dist.is_initialized():
            raise RuntimeError("force=True needs an initialised process group (init_from_env(force_pg=True))")
        # active: the bucket all-reduces are issued (always at world > 1; at world 1 only forced)
        self.active = self.world > 1 or bool(force)
        self._works: List = []
        self._pending_copies: List = []
        self.issued = 0  # bucket all-reduces issued from the host (a captured one counts once)

    def _launch(self, t: torch.Tensor) -> None:
        if not self.active:
            return
        self.issued += 1
        if self.compress_bf16:
            tmp = t.to(torch.bfloat16)
            w = dist.all_reduce(tmp, group=self.group, async_op=True)
            self._works.append(w)
            self._pending_copies.append((tmp, t))
        else:
            self._works.append(dist.all_reduce(t, group=self.group, async_op=True))

    def fc_ready(self, t: torch.Tensor) -> None:
        self._launch(t)

    def conv_ready(self, t: torch.Tensor) -> None:
        self._launch(t)

    def all_ready(self, t: torch.Tensor) -> None:
        """The whole flat gradient at once (the fused step completes both buckets together): one
        all-reduce instead of two."""
        self._launch(t)

    def finish(self) -> float:
        for w in self._works:
            w.wait()
        self._works.clear()
        for tmp, dst in self._pending_copies:
            dst.copy_(tmp)
        self._pending_copies.clear()
        return 1.0 / self.world


class BucketedDDP(nn.Module):
    """Minimal DistributedDataParallel with flat, size-capped gradient buckets.

    * parameters are broadcast from rank 0 at construction (reference DDP does the same);
    * buckets are filled in reverse parameter order (the order backward produces
      gradients) and all-reduced asynchronously as soon as every gradient of a
      bucket has arrived;
    * ``bucket_cap_mb`` defaults to 25 like torch DDP; for the MNIST model on xGMI a
      single bucket is optimal (one latency-bound collective per step).
    """

    def __init__(self, module: nn.Module, group=None, bucket_cap_mb: float = 25.0,
                 broadcast_buffers: bool = True):
        super().__init__()
        self.module = module
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        params = [p for p in module.parameters() if p.requires_grad]
        if self.world > 1:
            with torch.no_grad():
                for t in list(module.parameters()) + (list(module.buffers()) if broadcast_buffers else []):
                    dist.broadcast(t.data, 0, group=group)
        cap = int(bucket_cap_mb * 1024 * 1024)
        self._buckets: List[List[nn.Parameter]] = []
        cur, cur_bytes = [], 0
        for p in reversed(params):
            nbytes = p.numel() * p.element_size()
            if cur and cur_bytes + nbytes > cap:
                self._buckets.append(cur)
                cur, cur_bytes = [], 0
            cur.append(p)
            cur_bytes += nbytes
        if cur:
            self._buckets.append(cur)
        self._flat: List[torch.Tensor] = []
        self._slot: Dict[int, tuple] = {}
        for bi, bucket in enumerate(self._buckets):
            dtype = bucket[0].dtype
            n = sum(p.numel() for p in bucket)
            flat = torch.zeros(n, dtype=dtype, device=bucket[0].device)
            self._flat.append(flat)
            off = 0
            for p in bucket:
                self._slot[id(p)] = (bi, off)
                off += p.numel()
        self._pending = [0] * len(self._buckets)
        self._works: List = [None] * len(self._buckets)
        self._hooks = []
        if self.world > 1:
            for p in params:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))
        self._reset()

    def _reset(self):
        self._pending = [len(b) for b in self._buckets]
        self._works = [None] * len(self._buckets)

    def _on_grad(self, p: torch.Tensor) -> None:
        bi, off = self._slot[id(p)]
        flat = self._flat[bi]
        if p.grad is None:  # hooks also run when a backward returned no gradient for the leaf
            flat[off:off + p.numel()].zero_()
        else:
            flat[off:off + p.numel()].copy_(p.grad.reshape(-1))
        self._pending[bi] -= 1
        if self._pending[bi] == 0:
            self._works[bi] = dist.all_reduce(flat, group=self.group, async_op=True)

    def forward(self, *args, **kwargs):
        if self.world > 1:
            self._reset()
        return self.module(*args, **kwargs)

    def finish_gradient_sync(self) -> None:
        """Wait for all bucket all-reduces and write averaged grads back (call before optimizer.step)."""
        if self.world == 1:
            return
        for bi, bucket in enumerate(self._buckets):
            w = self._works[bi]
            if w is None:
                # parameters that received no grad this step: reduce zeros to stay in lockstep
                flat = self._flat[bi]
                for p in bucket:
                    b, off = self._slot[id(p)]
                    src = p.grad.reshape(-1) if p.grad is not None else torch.zeros_like(p).reshape(-1)
                    flat[off:off + p.numel()].copy_(src)
                w = dist.all_reduce(flat, group=self.group, async_op=True)
            w.wait()
            flat = self._flat[bi]
            flat.div_(self.world)
            for p in bucket:
                _, off = self._slot[id(p)]
                g = flat[off:off + p.numel()].view_as(p)
                if p.grad is None:
                    p.grad = g.clone()
                else:
                    p.grad.copy_(g)
