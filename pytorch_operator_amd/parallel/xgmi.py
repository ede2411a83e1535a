"""Peer-memory (xGMI) gradient all-reduce fused with SGD -- the DDP hot path on one node.

``XgmiAllReduce`` wraps ``csrc/kernels/xgmi_allreduce.hip``: every rank exports an
uncached device buffer through a HIP IPC handle, the handles are exchanged once over the
process group, and each training step then runs ONE kernel per rank that

1. pushes every gradient element into the buffer of the rank that owns it (posted
   stores over xGMI, then a step-numbered flag per sender block),
2. reduces shard ``rank`` across all senders (fixed rank order) and applies SGD to it,
   then pushes the updated parameters into every peer's buffer (+ a flag per chunk),
3. copies the other shards' parameters from its own buffer once their flags arrive.

Remote traffic is stores only and every wait polls local memory, one lane per flag.
No host involvement per step, so the whole DDP step (forward, backward, all-reduce,
optimizer) is one hipGraph.  This replaces the reference's implicit DDP all-reduce
(examples/mnist/mnist.py:136-138 -> NCCL ring) with the direct two-shot exchange that
suits 7 point-to-point xGMI links: 2 x 1.7 MB / W bytes per link per step.

Safety: every wait inside the kernel is bounded; ``self_test()`` compares the kernel with
``torch.distributed.all_reduce`` on random data for several steps (covering both parity
buffers) and every rank adopts the path only if ALL ranks passed -- otherwise the caller
falls back to RCCL (``FlatGradAllReduce``).
"""
from __future__ import annotations

import ctypes
import json
import os
import socket
from typing import Optional

import torch
import torch.distributed as dist

from ..ops import _native


class XgmiUnavailable(RuntimeError):
    pass


def physical_gpu(device: torch.device) -> tuple:
    """The GPU behind ``device``, independent of the process's visible-device list: its PCI
    (domain, bus, device) ids.  Pods that each see one GPU as ``cuda:0`` (the kubelet emulator's
    ``HIP_VISIBLE_DEVICES``) then count as sharing a GPU only when they really do."""
    try:
        p = torch.cuda.get_device_properties(device)
        bus = getattr(p, "pci_bus_id", None)
        if bus is not None:
            return ("pci", int(getattr(p, "pci_domain_id", 0)), int(bus), int(getattr(p, "pci_device_id", 0)))
    except (RuntimeError, AssertionError, AttributeError):
        pass
    return ("index", device.index)


class XgmiAllReduce:
    """Rank-local handle on the shared exchange buffers (world 2..8, one GPU per rank)."""

    def __init__(self, n: int, group=None, nblk: int = 0, timeout_s: float = 5.0,
                 device: Optional[torch.device] = None):
        if not dist.is_initialized():
            raise XgmiUnavailable("needs an initialised process group")
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if not 2 <= self.world <= 8:
            raise XgmiUnavailable(f"world size {self.world} outside 2..8")
        if n % 4:
            raise ValueError("n must be a multiple of 4")
        self.n = int(n)
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.prebarrier = False
        where = (socket.gethostname(),) + physical_gpu(self.device)
        peers = [None] * self.world
        dist.all_gather_object(peers, where, group=group)
        self.ranks_on_device = sum(1 for p in peers if p == where)
        if nblk <= 0:
            # one workgroup per CU when every rank owns its GPU (the kernel's phase 1 reduces
            # the conv backward's slab -- 1.6 MB of 4-sample chunk rows + per-sample rows of the
            # small conv grads at B = 64 -- across more CUs: 256 workgroups measured faster than
            # 128 on the emulated W=2 exchange, 16.7 vs 18.2 us/launch, when the slab was the
            # round-2 6.5 MB per-sample form); 128 when ranks share a device (1-GPU
            # rehearsals), where every rank's blocks must be resident at once
            nblk = 256 if len(set(peers)) == self.world else 128
        self.nblk = int(nblk)
        # the other ranks on this GPU can hold a spinning exchange workgroup on every CU: order every
        # exchange behind a rank barrier (set_prebarrier; never on one rank per GPU)
        self.crowded = (self.ranks_on_device - 1) * self.nblk >= 256
        self.lib = _native.load()
        self._ctx = ctypes.c_void_p()
        handle = ctypes.create_string_buffer(64)
        rc = self.lib.pto_xar_create(self.rank, self.world, self.n, nblk, timeout_s,
                                     ctypes.byref(self._ctx), handle)
        handles = [None] * self.world
        dist.all_gather_object(handles, handle.raw if rc == 0 else b"", group=group)
        if rc != 0 or any(len(h) != 64 for h in handles):
            self._ctx = None
            raise XgmiUnavailable(f"pto_xar_create failed on some rank (local rc={rc})")
        blob = b"".join(handles)
        rc = self.lib.pto_xar_open(self._ctx, blob)
        flags = [None] * self.world
        dist.all_gather_object(flags, rc, group=group)
        if any(f != 0 for f in flags):
            raise XgmiUnavailable(f"hipIpcOpenMemHandle failed: {flags}")
        self.alloc_kind = int(self.lib.pto_xar_alloc_kind(self._ctx))
        self.npad = int(self.lib.pto_xar_npad(self._ctx))
        if self.crowded:
            self.set_prebarrier(True)
        # PTO_XAR_FENCE=full|light (diagnostics): force the exchange's fence flavour
        fence = {"full": 0, "light": 1}.get(os.environ.get("PTO_XAR_FENCE", ""), -1)
        if fence >= 0:
            _native.check(self.lib.pto_xar_fence(self._ctx, fence), "pto_xar_fence")

    # ------------------------------------------------------------------ ops
    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def allreduce_mean(self, inp: torch.Tensor, out: torch.Tensor) -> None:
        self._check(inp)
        self._check(out)
        _native.check(self.lib.pto_xar_allreduce(self._ctx, inp.data_ptr(), out.data_ptr(),
                                                  1.0 / self.world, self._stream()), "pto_xar_allreduce")

    def allreduce_sgd_(self, grads: torch.Tensor, params: torch.Tensor, momentum_buf: torch.Tensor, *,
                       lr: float, momentum: float, dampening: float = 0.0, weight_decay: float = 0.0,
                       nesterov: bool = False, first_step: bool = False,
                       step_counter: Optional[torch.Tensor] = None,
                       slab: Optional[torch.Tensor] = None, slab_rows: int = 0, conv_n: int = 0,
                       slab_big: Optional[tuple] = None, skip: Optional[tuple] = None) -> None:
        """SGD with the mean gradient over ranks.  With ``slab`` ([rows, stride] fp32), the
        first ``conv_n`` gradient entries are the sum of its first ``slab_rows`` rows
        (fused deterministic reduction of the conv backward's partials); ``grads`` then
        only needs to hold the entries after ``conv_n``.  ``slab_big = (rows, lo, hi)``: the
        entries [lo, hi) (conv2.weight, written per 4-sample chunk by conv_bwd4) sum only
        their first ``rows`` rows.  ``skip = (lo, hi)``: gradient entries [lo, hi) a producer
        launch of this step already pushed into their owners' receive buffers (fc1_bwd with
        ``xpush``, ``push_info``); they must still be in ``grads`` (the degraded fallback's
        local SGD reads them)."""
        for t in (grads, params, momentum_buf):
            self._check(t)
        sc = step_counter.data_ptr() if step_counter is not None else None
        sp, stride = None, 0
        if slab is not None:
            if not (slab.is_cuda and slab.dtype == torch.float32 and slab.is_contiguous() and slab.dim() == 2
                    and slab_rows <= slab.shape[0] and conv_n <= slab.shape[1]):
                raise ValueError("slab must be a contiguous fp32 CUDA [rows, stride] tensor")
            sp, stride = slab.data_ptr(), slab.shape[1]
        big_rows, big_lo, big_hi = slab_big if slab_big is not None else (max(1, slab_rows), 0, 0)
        _native.check(self.lib.pto_xar_allreduce_sgd(
            self._ctx, grads.data_ptr(), params.data_ptr(), momentum_buf.data_ptr(), lr, momentum,
            dampening, weight_decay, 1.0 / self.world, int(nesterov), int(first_step), sc,
            sp, int(slab_rows), int(stride), int(conv_n), int(big_rows), int(big_lo), int(big_hi),
            int(skip[0]) if skip else 0, int(skip[1]) if skip else 0, self._stream()), "pto_xar_allreduce_sgd")

    def allreduce_sgd_fc_(self, grads: torch.Tensor, params: torch.Tensor, momentum_buf: torch.Tensor, *,
                          lr: float, momentum: float, dampening: float = 0.0, weight_decay: float = 0.0,
                          nesterov: bool = False, first_step: bool = False,
                          step_counter: Optional[torch.Tensor] = None, slab: torch.Tensor, slab_rows: int,
                          conv_n: int, slab_big: Optional[tuple], fc: tuple) -> None:
        """The fused DDP step's exchange: ``allreduce_sgd_`` with the conv slab, and the fully
        connected layers' gradients computed inside the exchange from the step's activations --
        ``fc = (dh [B,500], a2 [B,800], dlogits [B,10], h [B,500], per_sample [B,2], stats, loss_scale,
        (fc1.weight, fc1.bias, fc2.weight, fc2.bias float offsets in the flat gradient))`` -- and
        deposited straight with their owners; the loss statistics land in ``stats``.  Nothing of
        the fc range is read from ``grads``."""
        for t in (grads, params, momentum_buf):
            self._check(t)
        if not (slab.is_cuda and slab.dtype == torch.float32 and slab.is_contiguous() and slab.dim() == 2
                and slab_rows <= slab.shape[0] and conv_n <= slab.shape[1]):
            raise ValueError("slab must be a contiguous fp32 CUDA [rows, stride] tensor")
        dh, a2, dlog, h, per_sample, stats, loss_scale, offs = fc
        B = int(dh.shape[0])
        for t, shape in ((dh, (B, 500)), (a2, (B, 800)), (dlog, (B, 10)), (h, (B, 500)), (per_sample, (B, 2))):
            if tuple(t.shape) != shape or t.dtype != torch.float32 or not t.is_contiguous() or not t.is_cuda:
                raise ValueError(f"fc operand must be contiguous fp32 CUDA {shape}")
        sc = step_counter.data_ptr() if step_counter is not None else None
        big_rows, big_lo, big_hi = slab_big if slab_big is not None else (max(1, slab_rows), 0, 0)
        _native.check(self.lib.pto_xar_allreduce_sgd_fc(
            self._ctx, grads.data_ptr(), params.data_ptr(), momentum_buf.data_ptr(), lr, momentum,
            dampening, weight_decay, 1.0 / self.world, int(nesterov), int(first_step), sc,
            slab.data_ptr(), int(slab_rows), int(slab.shape[1]), int(conv_n), int(big_rows), int(big_lo),
            int(big_hi), dh.data_ptr(), a2.data_ptr(), dlog.data_ptr(), h.data_ptr(), per_sample.data_ptr(),
            stats.data_ptr(), float(loss_scale), B, *[int(o) for o in offs], self._stream()),
            "pto_xar_allreduce_sgd_fc")

    def push_info(self):
        """(bases, rank, world, shard4) for a producer kernel that pushes gradient float4s into
        their owners' receive buffers itself (``ops.mnist.fc1_bwd(xpush=...)``)."""
        if getattr(self, "_push_info", None) is None:
            bases = (ctypes.c_void_p * 8)()
            rank, world, shard4 = ctypes.c_int(), ctypes.c_int(), ctypes.c_long()
            _native.check(self.lib.pto_xar_push_info(self._ctx, bases, ctypes.byref(rank), ctypes.byref(world),
                                                     ctypes.byref(shard4)), "pto_xar_push_info")
            self._push_info = (bases, rank.value, world.value, shard4.value)
        return self._push_info

    def err_ptr(self) -> int:
        """Device address of the exchange's error word (a pushing producer stops once it is set)."""
        return int(self.lib.pto_xar_err_ptr(self._ctx) or 0)

    def gather_sharded_(self, t: torch.Tensor) -> None:
        """Reassemble a tensor each rank only kept for its own shard (e.g. the momentum
        buffer after fused steps) so every rank holds the full, identical copy."""
        shard = self.npad // self.world
        lo, hi = self.rank * shard, min(self.n, (self.rank + 1) * shard)
        full = torch.zeros_like(t)
        if hi > lo:
            full[lo:hi] = t[lo:hi]
        dist.all_reduce(full, group=self.group)
        t.copy_(full)

    def error(self) -> int:
        return int(self.lib.pto_xar_error(self._ctx))

    def reset(self) -> None:
        """Restart the protocol after a failed exchange: this rank's flags, step counters and error
        word back to zero.  Collective -- every rank calls it while no exchange is in flight on
        any rank (synchronise and barrier before and after; ``autotune._restart_exchange``)."""
        _native.check(self.lib.pto_xar_reset(self._ctx), "pto_xar_reset")

    def fits_shared_gpu(self, fc: bool) -> bool:
        """Whether the exchange workgroups of every rank on this GPU can be resident at once (the
        fused form's kernel with ``fc``).  Ranks sharing a GPU finish an exchange only then; one
        rank per GPU always fits."""
        if self.ranks_on_device <= 1:
            return True
        resident = int(self.lib.pto_xar_resident_blocks(self._ctx, 1 if fc else 0))
        return resident >= self.ranks_on_device * self.nblk

    def set_prebarrier(self, on: bool = True) -> None:
        """Ranks sharing one GPU: a one-wave rank barrier before every later (or later-captured)
        exchange launch, so no rank's exchange spins on the CUs while a peer still runs its step
        kernels (csrc/kernels/xgmi_allreduce.hip ``xar_prebarrier_kernel``).  One rank per GPU
        never needs it."""
        _native.check(self.lib.pto_xar_prebarrier(self._ctx, 1 if on else 0), "pto_xar_prebarrier")
        self.prebarrier = bool(on)

    def enable_stamps(self, ring: int = 16) -> torch.Tensor:
        """Diagnostics: every later (or later-captured) launch records, per workgroup, its step,
        wall_clock64 stamps (100 MHz, one clock for every process on the GPU) at start / flag1
        raised / flag2 raised / end, the error word at the end and, after a phase-2 timeout, the
        first sender flag still missing (q * nblk + j + 1) -- into a ring of the last ``ring``
        launches, [ring, nblk, 8] int64.  A launch that starts degraded writes nothing, so the
        record of the launch that timed out survives."""
        self.stamps = torch.zeros((ring, self.nblk, 8), dtype=torch.int64, device=self.device)
        _native.check(self.lib.pto_xar_stamps(self._ctx, ctypes.c_void_p(self.stamps.data_ptr()), int(ring)),
                      "pto_xar_stamps")
        return self.stamps

    def _check(self, t: torch.Tensor) -> None:
        if not (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous() and t.numel() == self.n):
            raise ValueError(f"expected contiguous fp32 CUDA tensor of {self.n} elements")
        if t.data_ptr() % 16:
            raise ValueError("tensor must be 16-byte aligned")

    # ------------------------------------------------------------------ validation
    def self_test(self, steps: int = 12, seed: int = 1234) -> bool:
        """Kernel vs ``dist.all_reduce`` on random data (mean and fused SGD); all ranks agree."""
        ok = True
        report = []
        g = torch.Generator(device="cpu").manual_seed(seed + self.rank)
        # diagnostics: PTO_XAR_SELFTEST_STAMPS=<dir> keeps every launch's per-block stamps (step,
        # wall-clock phases, error word) and writes them there as rank<r>.json after the test
        stamp_dir = os.environ.get("PTO_XAR_SELFTEST_STAMPS")
        if stamp_dir:
            self.enable_stamps(ring=2 * steps)
        for i in range(steps):
            xc = torch.randn(self.n, generator=g)
            x = xc.to(self.device)
            ref = x.clone()
            dist.all_reduce(ref, group=self.group)  # collectives first: never skipped by a failure
            ref /= self.world
            # every rank's input, to tell which side is off when a check fails: host tensors over
            # gloo (not its GPU-tensor path, which the reference above takes), device ones otherwise
            host = dist.get_backend(self.group) == "gloo"
            xs = [torch.empty(self.n) if host else torch.empty_like(x) for _ in range(self.world)]
            dist.all_gather(xs, xc if host else x, group=self.group)
            try:
                out = torch.empty_like(x)
                self.allreduce_mean(x, out)
                torch.cuda.synchronize(self.device)
                # fused SGD (first step: buf = mean grad, p -= lr * buf) on every rank
                p = torch.linspace(-1, 1, self.n, device=self.device)
                buf = torch.zeros_like(p)
                p_ref = p - 0.1 * ref
                self.allreduce_sgd_(x, p, buf, lr=0.1, momentum=0.5, first_step=True)
                torch.cuda.synchronize(self.device)
                # momentum lives only on the shard this rank owns (ZeRO-1 style update)
                lo = self.rank * (self.npad // self.world)
                hi = min(self.n, lo + self.npad // self.world)
                errs = {"mean": float((out - ref).abs().max()), "param": float((p - p_ref).abs().max()),
                        "momentum": float((buf[lo:hi] - ref[lo:hi]).abs().max()) if hi > lo else 0.0}
                bad = {k: v for k, v in errs.items() if not v <= 1e-5}
                if bad:  # both sides against the float64 mean of every rank's input
                    truth = torch.stack([t.cpu() for t in xs]).double().mean(0).float()
                    ok = False
                    idx = int((out - ref).abs().argmax())
                    report.append({"step": i, **bad, "argmax_mean": idx,
                                   "xgmi_vs_host_mean": float((out.cpu() - truth).abs().max()),
                                   "gloo_vs_host_mean": float((ref.cpu() - truth).abs().max())})
            except Exception as e:  # noqa: BLE001 -- any failure means "do not use this path"
                ok = False
                report.append({"step": i, "exception": repr(e)})
        try:
            if self.error():
                ok = False
                report.append({"kernel_error": self.error()})
        except Exception as e:  # noqa: BLE001
            ok = False
            report.append({"exception": repr(e)})
        self.last_report = report
        if stamp_dir:
            os.makedirs(stamp_dir, exist_ok=True)
            with open(os.path.join(stamp_dir, f"rank{self.rank}.json"), "w") as f:
                json.dump({"rank": self.rank, "report": report, "stamps": self.stamps.cpu().tolist()}, f)
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=self.device)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.group)
        return bool(flag.item())

    def close(self) -> None:
        if self._ctx:
            self.lib.pto_xar_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


class XgmiEmulation:
    """``world`` ranks of the same kernel on ONE device in one launch (grid.y = rank).

    Every block of every emulated rank is co-resident, so the protocol runs exactly as on
    a node (flags, pushes, step counters, bounded waits) with local HBM in place of the
    xGMI links: a world-8 correctness test and the protocol's latency floor on a 1-GPU box.
    """

    def __init__(self, world: int, n: int, nblk: int = 128, timeout_s: float = 2.0, alloc_kind: int = 0,
                 fence: int = -1):
        self.lib = _native.load()
        self.world, self.n = int(world), int(n)
        self._ctx = ctypes.c_void_p()
        rc = self.lib.pto_xar_emu_create(self.world, self.n, nblk, timeout_s, alloc_kind, fence,
                                         ctypes.byref(self._ctx))
        if rc != 0:
            self._ctx = None
            raise XgmiUnavailable(f"pto_xar_emu_create failed ({rc})")
        self.npad = int(self.lib.pto_xar_emu_npad(self._ctx))
        self.nblk = nblk
        # threads per emulated workgroup: 256 as on a node, or one wave when W x nblk > 1024
        # (W = 8 x 256, the production geometry, fits the device only with 1-wave workgroups)
        self.threads = int(self.lib.pto_xar_emu_threads(self._ctx))
        self.stamps = None

    def enable_stamps(self) -> torch.Tensor:
        """Per (rank, block): wall_clock64 at start / flags1 sent / flags2 sent / end (call
        before ``configure``)."""
        self.stamps = torch.zeros(self.world * self.nblk * 4, dtype=torch.int64, device="cuda")
        self.lib.pto_xar_emu_stamps(self._ctx, ctypes.c_void_p(self.stamps.data_ptr()))
        return self.stamps

    def _ptrs(self, ts):
        if ts is None:
            return None
        assert len(ts) == self.world
        return (ctypes.c_longlong * self.world)(*[t.data_ptr() for t in ts])

    def configure(self, mode: int, inputs, dst, mbuf=None, slab=None, slab_rows: int = 0, conv_n: int = 0,
                  lr: float = 0.0, momentum: float = 0.0, dampening: float = 0.0, weight_decay: float = 0.0,
                  nesterov: bool = False, first_step: bool = False, slab_big: Optional[tuple] = None,
                  skip: Optional[tuple] = None) -> None:
        """``skip = (lo, hi)``: gradient entries a producer pushes itself (``prepush`` emulates
        fc1_bwd's dW_fc1 push); the exchange's phase 1 skips them."""
        for t in list(inputs) + list(dst) + list(mbuf or []):
            if not (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous() and t.numel() == self.n
                    and t.data_ptr() % 16 == 0):
                raise ValueError(f"expected aligned contiguous fp32 CUDA tensors of {self.n} elements")
        stride = slab[0].shape[1] if slab is not None else 0
        big_rows, big_lo, big_hi = slab_big if slab_big is not None else (max(1, slab_rows), 0, 0)
        self._keep = (inputs, dst, mbuf, slab)  # the kernel holds raw pointers
        _native.check(self.lib.pto_xar_emu_set(
            self._ctx, int(mode), self._ptrs(inputs), self._ptrs(dst), self._ptrs(mbuf), self._ptrs(slab),
            int(slab_rows), int(stride), int(conv_n), int(big_rows), int(big_lo), int(big_hi), lr, momentum,
            dampening, weight_decay, int(nesterov), int(first_step), int(skip[0]) if skip else 0,
            int(skip[1]) if skip else 0), "pto_xar_emu_set")

    def configure_fc(self, dh, a2, dlog, h, per_sample, stats, B: int, loss_scale: float, offsets) -> None:
        """The fused DDP step's exchange on top of ``configure(mode=1, skip=(fc1.weight offset, n))``:
        per emulated rank the step's activations (lists of ``world`` tensors), from which the
        exchange computes dW_fc1 / db_fc1 / dW_fc2 / db_fc2 and the loss statistics itself.
        ``offsets``: flat-layout offsets of fc1.weight, fc1.bias, fc2.weight, fc2.bias."""
        w1, b1, w2, b2 = (int(o) for o in offsets)
        self._keep_fc = (dh, a2, dlog, h, per_sample, stats)
        _native.check(self.lib.pto_xar_emu_set_fc(
            self._ctx, self._ptrs(dh), self._ptrs(a2), self._ptrs(dlog), self._ptrs(h), self._ptrs(per_sample),
            self._ptrs(stats), int(B), float(loss_scale), w1, b1, w2, b2), "pto_xar_emu_set_fc")
        self.threads = int(self.lib.pto_xar_emu_threads(self._ctx))

    def prepush(self) -> None:
        _native.check(self.lib.pto_xar_emu_prepush(
            self._ctx, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)), "pto_xar_emu_prepush")

    def launch(self) -> None:
        _native.check(self.lib.pto_xar_emu_launch(
            self._ctx, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)), "pto_xar_emu_launch")

    def error(self) -> int:
        return int(self.lib.pto_xar_emu_error(self._ctx))

    def close(self) -> None:
        if self._ctx:
            self.lib.pto_xar_emu_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


class XgmiGradSync:
    """``grad_sync`` for ``FusedMnistTrainer``: the all-reduce and SGD are one kernel,
    issued from the trainer's step tail (capturable, so the step graph holds everything).
    ``push_fc1``: fc1_bwd pushes dW_fc1 into its owners' receive buffers itself and the
    exchange skips it (default; ``PTO_XGMI_PUSH_FC1=0`` turns it off for A/B)."""

    fused_sgd = True
    push_fc1 = os.environ.get("PTO_XGMI_PUSH_FC1", "1") != "0"

    def __init__(self, xar: XgmiAllReduce):
        self.xar = xar
        self.world = xar.world

    def fc_ready(self, t):  # the exchange runs once, at the step tail
        pass

    def conv_ready(self, t):
        pass

    def all_ready(self, t):
        pass

    def finish(self) -> float:
        return 1.0 / self.world


def try_xgmi(n: int, device, required: bool = False, log=print,
             timeout_s: float = 5.0) -> Optional[XgmiGradSync]:
    """The self-tested xGMI gradient path, or None (RCCL then carries the gradients).

    Only used under RCCL (one GPU per rank) unless ``required`` or ``PTO_XGMI_ANY_BACKEND=1``
    -- which let the 1-GPU rehearsal run it under gloo with ranks sharing a device (the
    latter keeps the start-up race against the gloo bucket path, ``--allreduce auto``)."""
    if not required and dist.get_backend() != "nccl" and os.environ.get("PTO_XGMI_ANY_BACKEND") != "1":
        return None
    # PTO_XGMI_TIMEOUT_S: the exchange's bounded wait (crowded one-GPU rehearsals, where a rank
    # sharing the host's CPUs with many others can arrive seconds late)
    timeout_s = float(os.environ.get("PTO_XGMI_TIMEOUT_S", timeout_s))
    try:
        xar = XgmiAllReduce(n, device=device, timeout_s=timeout_s)
    except XgmiUnavailable as e:
        if required:
            raise
        log(f"xgmi all-reduce unavailable ({e}); using RCCL")
        return None
    if xar.self_test():
        return XgmiGradSync(xar)
    errs = [r for r in xar.last_report if "kernel_error" in r or "exception" in r]
    log(f"xgmi all-reduce self-test failed ({errs + xar.last_report[:2]}); using RCCL")
    xar.close()
    if required:
        raise XgmiUnavailable("xgmi path requested but its self-test failed")
    return None
