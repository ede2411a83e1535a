"""ZeRO-1 data parallelism for bf16 master-weight training (the Llama DDP worker, ``--zero 1``).

The reference's DDP contract (``examples/mnist/mnist.py:136-138``: every replica steps the
same model on its own data, gradients averaged) is kept; what changes is where the optimizer
state lives.  ``DistributedDataParallel`` + ``MasterAdamW`` keeps, on EVERY rank, fp32
masters + both AdamW moments (12 B/param: 96 GB for Llama-3 8B) and runs the memory-bound
update over all of them (~40 ms of a 360 ms step on one MI355X,
``profiles/r2_llama3_8b_step_kernels.md``).  Here each rank owns 1/W of every bucket:

* backward: each gradient is copied (fp32) into its flat bucket as soon as autograd has
  accumulated it (post-accumulate hook; the bf16 ``.grad`` is freed right away), the bucket
  is scaled by 1/W and **reduce-scattered** (fp32 sum) asynchronously while backward goes on;
* ``step()``: fused HIP AdamW (``csrc/kernels/adamw.hip``) on the rank's shard only
  (master, m, v, grad shard -> new master + the bf16 weight shard, in place in the flat
  weight bucket), then an async in-place **all-gather** of the bucket's weights;
* next forward: a pre-hook per module waits (stream-side) for the all-gather of the buckets
  holding that module's weights, so later buckets' all-gathers run under earlier layers.

Bytes per rank and step over xGMI: reduce-scatter 4 B x (W-1)/W + all-gather 2 B x (W-1)/W
per parameter, against 2 x 4 B x (W-1)/W for the fp32 all-reduce it replaces; optimizer state
and update time are divided by W.  Buckets are large (``bucket_mb``, default 256 MB of
fp32 gradient): few collectives, each well into RCCL's bandwidth regime on point-to-point
xGMI links.

``reduce_dtype=torch.bfloat16`` (``--allreduce-dtype bf16``; at world 1, where nothing is
reduced, every bucket takes its parameters' dtype) halves the reduce-scatter bytes, like DDP's
``bf16_compress_hook``, and enables **gradient-as-bucket-view** (``grad_view``): every bf16
matmul weight gets a ``_pto_grad_sink`` whose view IS its bucket slot, and ``linear_tn``'s
backward GEMM writes dW there directly (``ops/llm.py``) -- no bf16 ``.grad`` allocation and no
deposit copy pass (the round-2 world-1 cost: 389 vs 365 ms/step and +30 GB).  Such buckets
hold the unscaled gradient sum; the 1/W rides on the AdamW kernel (exact for W = 2^k).

Numerics (fp32 reduction) equal ``DDP(fp32 comm hook) + MasterAdamW``: the same fp32 sum of the same
``grad / W`` terms, the same AdamW per element (tests/test_harness.py pins the parameter
digest of both paths equal on gloo).
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional

import torch
import torch.distributed as dist
import torch.nn as nn

_ALIGN = 64  # shard lengths are multiples of this (16-byte aligned fp32 / bf16 shard pointers)


class _Sink:
    """Destination of a weight gradient written in place by a backward GEMM: its slot of the
    bucket (allocated when the bucket's first gradient arrives, see ``_Bucket.grad32``)."""
    __slots__ = ("bucket", "off", "shape", "dtype", "ready")

    def __init__(self, bucket, off: int, shape, ready):
        self.bucket, self.off, self.shape, self.ready = bucket, off, shape, ready
        self.dtype = bucket.gdt

    @property
    def view(self) -> torch.Tensor:
        n = 1
        for d in self.shape:
            n *= d
        return self.bucket.grad32[self.off:self.off + n].view(self.shape)


class _Bucket:
    def __init__(self, params: List[nn.Parameter], world: int, rank: int, reduce_dtype=torch.float32):
        self.params = params
        self.dtype = params[0].dtype
        dev = params[0].device
        n = sum(p.numel() for p in params)
        self.shard = -(-n // (world * _ALIGN)) * _ALIGN
        self.npad = self.shard * world
        self.lo = rank * self.shard
        self.flat_w = torch.zeros(self.npad, dtype=self.dtype, device=dev)
        # gradient bucket: the reduce dtype; at world 1 (nothing is reduced) the parameters' own
        # dtype, i.e. exactly the .grad autograd would have produced
        self.gdt = reduce_dtype if world > 1 else self.dtype
        self.n = n
        self.world = world
        # the full gradient bucket lives only from its first gradient of a backward to the end of
        # its reduce-scatter (world 1: to the end of step()): allocated at the first arrival, then
        # released, so it never coexists with the forward's activation peak -- the peak memory of
        # a step stays that of .grad-based training (the caching allocator recycles the block)
        self._g: Optional[torch.Tensor] = None
        self._dev = dev
        self._gshard = None if world == 1 else torch.zeros(self.shard, dtype=self.gdt, device=dev)
        self.slot: Dict[int, int] = {}
        masters = torch.zeros(self.npad, dtype=torch.float32, device=dev) if self.dtype != torch.float32 else None
        off = 0
        with torch.no_grad():
            for p in params:
                k = p.numel()
                self.slot[id(p)] = off
                self.flat_w[off:off + k].copy_(p.detach().reshape(-1))
                if masters is not None:
                    init = getattr(p, "_pto_master", None)  # exact fp32 init (ops/optim.py)
                    masters[off:off + k].copy_((init if init is not None else p.detach()).reshape(-1))
                    if init is not None:
                        del p._pto_master
                p.data = self.flat_w[off:off + k].view(p.shape)
                off += k
        # fp32 master of the owned shard (None: fp32 weights are their own master)
        self.master = masters[self.lo:self.lo + self.shard].clone() if masters is not None else None
        del masters
        self.exp_avg = torch.zeros(self.shard, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(self.shard, dtype=torch.float32, device=dev)
        self.pending = len(params)
        self.arrived: set = set()  # ids of the parameters whose gradient was deposited this step
        self.rs_work = None
        self.ag_work = None
        self.unscaled = False  # grad_view bucket: holds sum(g), AdamW applies 1/W

    def w_shard(self) -> torch.Tensor:
        return self.flat_w[self.lo:self.lo + self.shard]

    @property
    def grad32(self) -> torch.Tensor:
        if self._g is None:
            # every slot is written before use (gradient copy / in-place GEMM, or zeroed by
            # step() for a parameter without a gradient); only the alignment padding is cleared
            self._g = torch.empty(self.npad, dtype=self.gdt, device=self._dev)
            if self.npad > self.n:
                self._g[self.n:].zero_()
        return self._g

    @property
    def gshard(self) -> torch.Tensor:
        # world 1: the shard IS the bucket (no reduce-scatter, no copy)
        return self.grad32 if self.world == 1 else self._gshard

    def release_grad(self) -> None:
        self._g = None


class ZeroAdamW:
    """Replaces ``DDP(model) + MasterAdamW``: construct on the (unwrapped) model after
    ``to_bf16_matmul_weights``; call ``zero_grad`` / forward / backward / ``step`` as usual.
    Weights are broadcast from rank 0 at construction (DDP constructor semantics)."""

    def __init__(self, model: nn.Module, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2,
                 group=None, bucket_mb: float = 256.0, reduce_dtype=torch.float32, grad_view: bool = True):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.lr, self.betas, self.eps, self.weight_decay = lr, betas, eps, weight_decay
        self.t = 0
        # per-parameter AdamW step counts (bias correction), as MasterAdamW's st["step"]: at world 1
        # a parameter that gets no gradient skips the step and its count stays behind
        self.pstep: Dict[int, int] = {}
        if reduce_dtype not in (torch.float32, torch.bfloat16):
            raise TypeError("reduce_dtype: float32 or bfloat16")
        self.reduce_dtype = reduce_dtype
        params = [p for p in model.parameters() if p.requires_grad]
        if self.world > 1:
            with torch.no_grad():
                for p in params:
                    dist.broadcast(p.data, 0, group=group)
                    init = getattr(p, "_pto_master", None)
                    if init is not None:
                        dist.broadcast(init, 0, group=group)
        # buckets in backward order (reverse registration), <= bucket_mb of fp32 each; one open
        # bucket per dtype, so the small fp32 norm weights between the bf16 projections share
        # buckets instead of each cutting a bf16 run into a tiny collective
        cap = int(bucket_mb * 2 ** 20) // 4
        self.buckets: List[_Bucket] = []
        open_: Dict[torch.dtype, List[nn.Parameter]] = {}
        size: Dict[torch.dtype, int] = {}
        for p in reversed(params):
            cur = open_.setdefault(p.dtype, [])
            if cur and size[p.dtype] + p.numel() > cap:
                self.buckets.append(_Bucket(cur, self.world, self.rank, reduce_dtype))
                cur = open_[p.dtype] = []
                size[p.dtype] = 0
            cur.append(p)
            size[p.dtype] = size.get(p.dtype, 0) + p.numel()
        for cur in open_.values():
            if cur:
                self.buckets.append(_Bucket(cur, self.world, self.rank, reduce_dtype))
        self._of: Dict[int, _Bucket] = {id(p): b for b in self.buckets for p in b.params}
        for p in params:
            p.register_post_accumulate_grad_hook(self._on_grad)
        self.sinks = 0
        if grad_view:
            for b in self.buckets:
                if b.gdt != b.dtype or not b.flat_w.is_cuda:
                    continue
                b.unscaled = True
                for p in b.params:
                    if p.dim() == 2:
                        p._pto_grad_sink = _Sink(b, b.slot[id(p)], tuple(p.shape),
                                                 lambda p=p, b=b: self._arrive(b, p))
                        self.sinks += 1
        self._hooked = 0
        for mod in model.modules():
            own = [self._of[id(p)] for p in mod.parameters(recurse=False) if id(p) in self._of]
            if own:
                uniq = list({id(b): b for b in own}.values())
                mod.register_forward_pre_hook(lambda _m, _i, bs=uniq: self._wait_weights(bs))
                self._hooked += 1

    # ------------------------------------------------------------------ backward side
    def _on_grad(self, p: torch.Tensor) -> None:
        if p.grad is None:
            # autograd runs post-accumulate hooks even when the backward returned no gradient
            # for the leaf -- the case of a weight whose gradient sink was written in place
            # (it arrived through _arrive already) or of no gradient at all (step() fills it)
            return
        b = self._of[id(p)]
        if b.pending < 0:
            raise RuntimeError("ZeroAdamW: a second backward before step() -- gradient accumulation "
                               "across backward passes is not supported (the bucket was already reduced)")
        off = b.slot[id(p)]
        self._deposit(b.grad32[off:off + p.numel()], p.grad.reshape(-1), b.unscaled)
        p.grad = None
        self._arrive(b, p)

    def _arrive(self, b: _Bucket, p: torch.Tensor) -> None:
        if b.pending < 0:
            raise RuntimeError("ZeroAdamW: a second backward before step() -- gradient accumulation "
                               "across backward passes is not supported (the bucket was already reduced)")
        if id(p) in b.arrived:
            raise RuntimeError("ZeroAdamW: a parameter received two gradients in one backward (a weight "
                               "used twice cannot write its gradient in place; construct with grad_view=False)")
        b.arrived.add(id(p))
        b.pending -= 1
        if b.pending == 0:
            self._reduce_scatter(b)

    def _deposit(self, dst: torch.Tensor, g: torch.Tensor, unscaled: bool = False) -> None:
        """dst = g / W in the bucket dtype -- the comm hooks' ``grad / W`` before the sum.  For a
        power-of-two W the scale is exact, so it rides on the cast copy (one pass).  ``unscaled``
        (grad_view buckets): plain copy, the 1/W is applied by AdamW."""
        w = self.world
        if w == 1 or unscaled:
            dst.copy_(g)
        elif w & (w - 1) == 0:
            src = g if dst.dtype == torch.float32 else g.to(dst.dtype)  # (out= never downcasts)
            torch.mul(src, 1.0 / w, out=dst)
        else:
            dst.copy_(g)
            dst.div_(w)

    def _reduce_scatter(self, b: _Bucket) -> None:
        if self.world == 1:
            b.rs_work = None
        else:
            b.rs_work = dist.reduce_scatter_tensor(b.gshard, b.grad32, group=self.group, async_op=True)
        b.pending = -1  # launched

    def zero_grad(self, set_to_none: bool = True) -> None:  # noqa: ARG002 -- grads never persist
        for b in self.buckets:
            for p in b.params:
                p.grad = None

    # ------------------------------------------------------------------ optimizer side
    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        self.t += 1
        skip: Dict[int, set] = {}
        for b in self.buckets:
            if b.pending >= 0:
                # some parameter of this bucket got no gradient through the hook this step.  Only
                # the slots that never arrived are filled (zeros, or a gradient set outside
                # backward); deposited gradients are kept.  At world > 1 a missing gradient
                # contributes zeros to the sum (DDP's find_unused_parameters semantics); at world 1
                # a parameter without any gradient is left untouched, as MasterAdamW /
                # torch.optim.AdamW skip it.
                for p in b.params:
                    if id(p) in b.arrived:
                        continue
                    off = b.slot[id(p)]
                    if p.grad is None:
                        b.grad32[off:off + p.numel()].zero_()
                        if self.world == 1:
                            skip.setdefault(id(b), set()).add(id(p))
                    else:
                        self._deposit(b.grad32[off:off + p.numel()], p.grad.reshape(-1), b.unscaled)
                        p.grad = None
                self._reduce_scatter(b)
        # forward order (the last bucket holds the first layers): their all-gathers go first
        for b in reversed(self.buckets):
            if b.rs_work is not None:
                b.rs_work.wait()
                b.rs_work = None
            if self.world > 1:
                b.release_grad()  # the shard holds what AdamW needs (stream-ordered after the wait)
            # parameters grouped by their step count after this step (world > 1: every parameter
            # steps -- a missing gradient is a zero contribution, DDP's semantics); each group is
            # one AdamW pass over the bucket with the other ranges saved and restored around it
            skipped = skip.get(id(b), set())
            groups: Dict[int, List[nn.Parameter]] = {}
            for p in b.params:
                if id(p) not in skipped:
                    t = self.pstep[id(p)] = self.pstep.get(id(p), self.t - 1) + 1
                    groups.setdefault(t, []).append(p)
            if self.world > 1 and len(groups) > 1:
                # _save_ranges / _restore_ranges index bucket-absolute offsets, valid only when the
                # shard is the whole bucket (world 1); at world > 1 every parameter steps together
                raise RuntimeError("ZeroAdamW: parameters of one bucket diverged in step count at world > 1")
            for t, members in groups.items():
                ids = {id(p) for p in members}
                keep = self._save_ranges(b, [(b.slot[id(p)], p.numel()) for p in b.params if id(p) not in ids])
                self._adamw(b, t)
                self._restore_ranges(b, keep)
            if self.world == 1:
                b.release_grad()
            if self.world > 1:
                src = b.w_shard() if b.flat_w.is_cuda else b.w_shard().clone()
                b.ag_work = dist.all_gather_into_tensor(b.flat_w, src, group=self.group, async_op=True)
            b.pending = len(b.params)
            b.arrived.clear()
        return loss

    @staticmethod
    def _save_ranges(b: _Bucket, ranges) -> list:
        """Copies of the optimizer state + weights of the bucket ranges AdamW must not touch
        (world 1 only: the shard is the whole bucket)."""
        out = []
        for off, n in ranges:
            sl = slice(off, off + n)
            out.append((sl, b.flat_w[sl].clone(), b.exp_avg[sl].clone(), b.exp_avg_sq[sl].clone(),
                        b.master[sl].clone() if b.master is not None else None))
        return out

    @staticmethod
    def _restore_ranges(b: _Bucket, saved) -> None:
        for sl, w, m, v, ms in saved:
            b.flat_w[sl].copy_(w)
            b.exp_avg[sl].copy_(m)
            b.exp_avg_sq[sl].copy_(v)
            if ms is not None:
                b.master[sl].copy_(ms)

    def _adamw(self, b: _Bucket, t: int) -> None:
        b1, b2 = self.betas
        w = b.w_shard()
        master = b.master if b.master is not None else w
        if w.is_cuda:
            from ..ops import _native
            stream = ctypes.c_void_p(torch.cuda.current_stream(w.device).cuda_stream)
            out = w.data_ptr() if b.master is not None else None
            _native.check(_native.load().pto_adamw_step_scaled(
                master.data_ptr(), b.exp_avg.data_ptr(), b.exp_avg_sq.data_ptr(), b.gshard.data_ptr(), out,
                b.shard, 1 if b.gshard.dtype == torch.bfloat16 else 0, self.lr, b1, b2, self.eps,
                self.weight_decay, t, 1.0 / self.world if b.unscaled else 1.0, stream), "adamw_step")
        else:
            from ..ops.optim import MasterAdamW
            st = {"step": t, "exp_avg": b.exp_avg, "exp_avg_sq": b.exp_avg_sq}
            MasterAdamW._step_reference(w, b.gshard, master, st, self.lr, b1, b2, self.eps, self.weight_decay)

    def _wait_weights(self, buckets) -> None:
        for b in buckets:
            if b.ag_work is not None:
                b.ag_work.wait()  # stream-side wait on GPU backends
                b.ag_work = None

    def synchronize(self) -> None:
        """Wait for every outstanding weight all-gather (before reading the weights)."""
        self._wait_weights(self.buckets)

    # ------------------------------------------------------------------ checkpoint (utils/train_ckpt.py)
    def shard_state_dict(self) -> dict:
        """This rank's optimizer shard: step count + fp32 master / moments of each bucket's slice
        (the weights themselves are in the model's state_dict)."""
        return {"t": self.t, "world": self.world, "rank": self.rank,
                "buckets": [{"npad": b.npad, "master": b.master, "exp_avg": b.exp_avg,
                             "exp_avg_sq": b.exp_avg_sq,
                             "pstep": [self.pstep.get(id(p), self.t) for p in b.params]} for b in self.buckets]}

    @torch.no_grad()
    def load_shard_state_dict(self, sd: dict) -> None:
        if sd["world"] != self.world or sd["rank"] != self.rank or len(sd["buckets"]) != len(self.buckets):
            raise ValueError("ZeRO shard checkpoint was written by a different world / rank / bucket layout")
        for b, s in zip(self.buckets, sd["buckets"]):
            if s["npad"] != b.npad or (s["master"] is None) != (b.master is None):
                raise ValueError("ZeRO shard checkpoint bucket layout differs")
            if b.master is not None:
                b.master.copy_(s["master"])
            b.exp_avg.copy_(s["exp_avg"])
            b.exp_avg_sq.copy_(s["exp_avg_sq"])
            for p, n in zip(b.params, s.get("pstep") or [int(sd["t"])] * len(b.params)):
                self.pstep[id(p)] = int(n)
        self.t = int(sd["t"])

    # ------------------------------------------------------------------ inspection
    def state_bytes(self) -> int:
        """Optimizer-state bytes held by this rank (masters + moments of its shards)."""
        n = 0
        for b in self.buckets:
            n += (b.exp_avg.numel() + b.exp_avg_sq.numel()) * 4
            n += b.master.numel() * 4 if b.master is not None else 0
        return n

    def full_masters_digest(self) -> Optional[str]:
        """sha1 of every bucket's fp32 masters gathered in rank order (all ranks must call)."""
        import hashlib
        h = hashlib.sha1()
        for b in self.buckets:
            m = b.master if b.master is not None else b.w_shard().float()
            full = torch.zeros(b.npad, dtype=torch.float32, device=m.device)
            if self.world > 1:
                dist.all_gather_into_tensor(full, m.contiguous(), group=self.group)
            else:
                full.copy_(m)
            h.update(full.cpu().numpy().tobytes())
        return h.hexdigest()
