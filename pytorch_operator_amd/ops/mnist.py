"""Python bindings for the fused MNIST kernels (csrc/kernels/mnist_kernels.hip).

Each function validates shapes/dtypes/devices on the host (the kernels' grids
assume them) and launches on the current torch stream, so calls compose with
``torch.cuda`` streams, events and graph capture.

Reference op sequence (jiaqianjing/pytorch-operator examples/mnist/mnist.py:25-33,
37-43): conv1 -> relu -> pool -> conv2 -> relu -> pool -> fc1 -> relu -> fc2 ->
log_softmax -> nll_loss -> backward -> SGD.step.
"""
from __future__ import annotations

from typing import Optional

import torch

from . import _native

MNIST_MEAN = 0.1307
MNIST_STD = 0.3081
U8_SCALE = 1.0 / (255.0 * MNIST_STD)
U8_SHIFT = -MNIST_MEAN / MNIST_STD


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _stream() -> int:
    return _native.current_stream_ptr()


def _req(t: torch.Tensor, shape, dtype, name: str) -> None:
    if not t.is_cuda:
        raise ValueError(f"{name} must be a CUDA (HIP) tensor")
    if t.dtype != dtype:
        raise ValueError(f"{name} must be {dtype}, got {t.dtype}")
    if tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name} must have shape {tuple(shape)}, got {tuple(t.shape)}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


class BatchSource:
    """Where a batch's pixels/labels come from (mirrors ``pto::BatchSrc``).

    ``x``: [N,784] (or [N,1,28,28]) uint8 raw pixels or fp32 values.
    ``perm``: optional int32 [N] order; the batch is ``perm[offset : offset+B]``
    (wrapping), with ``offset = cursor[0]*B % N`` when a device ``cursor`` is given
    (graph replay) or ``host_offset`` otherwise.  Without ``perm`` the batch is
    rows ``0..B-1`` of ``x``.
    """

    def __init__(self, x: torch.Tensor, labels: Optional[torch.Tensor] = None,
                 perm: Optional[torch.Tensor] = None, cursor: Optional[torch.Tensor] = None,
                 host_offset: int = 0, normalize: Optional[bool] = None):
        if not x.is_cuda or not x.is_contiguous():
            raise ValueError("x must be a contiguous CUDA tensor")
        if x.numel() % 784 != 0:
            raise ValueError("x must hold 28x28 images")
        self.x = x
        self.n_total = x.numel() // 784
        self.is_u8 = x.dtype == torch.uint8
        if not self.is_u8 and x.dtype != torch.float32:
            raise ValueError("x must be uint8 or float32")
        if normalize is None:
            normalize = self.is_u8
        if self.is_u8 and normalize:
            self.scale, self.shift = U8_SCALE, U8_SHIFT
        elif normalize:
            self.scale, self.shift = 1.0 / MNIST_STD, -MNIST_MEAN / MNIST_STD
        else:
            self.scale, self.shift = 1.0, 0.0
        if labels is not None:
            if labels.dtype != torch.int32 or not labels.is_cuda or labels.numel() != self.n_total:
                raise ValueError("labels must be int32 CUDA [N]")
        self.labels = labels
        if perm is not None:
            if perm.dtype != torch.int32 or perm.numel() != self.n_total or not perm.is_cuda:
                raise ValueError("perm must be int32 CUDA [N]")
        self.perm = perm
        if cursor is not None and (cursor.dtype != torch.int32 or not cursor.is_cuda):
            raise ValueError("cursor must be an int32 CUDA tensor")
        self.cursor = cursor
        self.host_offset = int(host_offset)

    def check_batch(self, B: int) -> None:
        if self.perm is None and B > self.n_total:
            raise ValueError(f"batch {B} larger than dataset {self.n_total}")


def conv1_fwd(src: BatchSource, w: torch.Tensor, b: torch.Tensor, B: int,
              out: Optional[torch.Tensor] = None, idx: Optional[torch.Tensor] = None,
              zero: Optional[torch.Tensor] = None, xn: Optional[torch.Tensor] = None,
              lab: Optional[torch.Tensor] = None):
    """relu(maxpool2(conv1(normalize(x)))).

    Returns ``(a1 [B,20,12,12] f32, idx1 uint8 argmax, xn [B,784] normalised batch,
    lab [B] int32 gathered labels or None)``.  ``zero`` (optional) is zero-filled by
    the same launch.
    """
    lib = _native.load()
    src.check_batch(B)
    _req(w, (20, 1, 5, 5), torch.float32, "conv1.weight")
    _req(b, (20,), torch.float32, "conv1.bias")
    dev = w.device
    out = torch.empty((B, 20, 12, 12), device=dev) if out is None else out
    idx = torch.empty((B, 20, 12, 12), device=dev, dtype=torch.uint8) if idx is None else idx
    xn = torch.empty((B, 784), device=dev) if xn is None else xn
    if src.labels is not None and lab is None:
        lab = torch.empty((B,), device=dev, dtype=torch.int32)
    _req(out, (B, 20, 12, 12), torch.float32, "a1")
    _req(idx, (B, 20, 12, 12), torch.uint8, "idx1")
    _req(xn, (B, 784), torch.float32, "xn")
    if lab is not None:
        if src.labels is None:
            raise ValueError("lab output requested but BatchSource has no labels")
        _req(lab, (B,), torch.int32, "lab")
    zn = 0
    if zero is not None:
        if zero.dtype != torch.float32 or not zero.is_contiguous():
            raise ValueError("zero must be contiguous fp32")
        zn = zero.numel()
    rc = lib.pto_mnist_conv1_fwd(
        src.x.data_ptr(), int(src.is_u8), _ptr(src.labels), _ptr(src.perm), _ptr(src.cursor),
        src.host_offset, src.n_total, src.scale, src.shift, w.data_ptr(), b.data_ptr(),
        out.data_ptr(), idx.data_ptr(), B, _ptr(zero), zn, xn.data_ptr(), _ptr(lab), _stream())
    _native.check(rc, "conv1_fwd")
    return out, idx, xn, lab


def conv2_fwd(a1: torch.Tensor, w: torch.Tensor, b: torch.Tensor,
              out: Optional[torch.Tensor] = None, idx: Optional[torch.Tensor] = None):
    """relu(maxpool2(conv2(a1))) flattened -> (a2 [B,800], idx2 uint8 [B,800])."""
    lib = _native.load()
    B = a1.shape[0]
    _req(a1, (B, 20, 12, 12), torch.float32, "a1")
    _req(w, (50, 20, 5, 5), torch.float32, "conv2.weight")
    _req(b, (50,), torch.float32, "conv2.bias")
    if w.data_ptr() % 16:
        raise ValueError("conv2.weight must be 16-byte aligned")
    out = torch.empty((B, 800), device=a1.device) if out is None else out
    idx = torch.empty((B, 800), device=a1.device, dtype=torch.uint8) if idx is None else idx
    _req(out, (B, 800), torch.float32, "a2")
    _req(idx, (B, 800), torch.uint8, "idx2")
    rc = lib.pto_mnist_conv2_fwd(a1.data_ptr(), w.data_ptr(), b.data_ptr(), out.data_ptr(),
                                 idx.data_ptr(), B, _stream())
    _native.check(rc, "conv2_fwd")
    return out, idx


class BatchStage:
    """Device staging slot for the NEXT step's batch (uint8 pixels [B, 784], int32 labels,
    and the step number they belong to).  ``fc1_bwd(..., stage=)`` fills it during step t for
    step t + 1; ``conv12_fwd(..., stage=)`` then reads the batch with one load instead of the
    cursor -> permutation -> pixel chain, and falls back to the gather on its own whenever the
    tag is not the current cursor (first step, or the cursor was moved from the host)."""

    def __init__(self, B: int, device):
        self.B = int(B)
        self.x = torch.zeros((self.B, 784), dtype=torch.uint8, device=device)
        self.lab = torch.zeros((self.B,), dtype=torch.int32, device=device)
        self.tag = torch.full((1,), -1, dtype=torch.int32, device=device)

    def invalidate(self) -> None:
        """Forget the staged batch (call after changing the source's permutation in place)."""
        self.tag.fill_(-1)

    @staticmethod
    def supported(src: "BatchSource") -> bool:
        return src.is_u8 and src.perm is not None and src.cursor is not None and src.labels is not None


def conv12_fwd(src: BatchSource, w1: torch.Tensor, b1: torch.Tensor, w2: torch.Tensor,
               b2: torch.Tensor, B: int, a1=None, idx1=None, xn=None, lab=None, a2=None,
               idx2=None, stage: Optional[BatchStage] = None):
    """conv1+pool+conv2+pool fused (one launch): returns (a1, idx1, xn, lab, a2, idx2).
    ``stage``: take the batch from a ``BatchStage`` when its tag matches the cursor."""
    lib = _native.load()
    src.check_batch(B)
    _req(w1, (20, 1, 5, 5), torch.float32, "conv1.weight")
    _req(b1, (20,), torch.float32, "conv1.bias")
    _req(w2, (50, 20, 5, 5), torch.float32, "conv2.weight")
    _req(b2, (50,), torch.float32, "conv2.bias")
    dev = w1.device
    a1 = torch.empty((B, 20, 12, 12), device=dev) if a1 is None else a1
    idx1 = torch.empty((B, 20, 12, 12), device=dev, dtype=torch.uint8) if idx1 is None else idx1
    xn = torch.empty((B, 784), device=dev) if xn is None else xn
    if src.labels is not None and lab is None:
        lab = torch.empty((B,), device=dev, dtype=torch.int32)
    a2 = torch.empty((B, 800), device=dev) if a2 is None else a2
    idx2 = torch.empty((B, 800), device=dev, dtype=torch.uint8) if idx2 is None else idx2
    _req(a1, (B, 20, 12, 12), torch.float32, "a1")
    _req(idx1, (B, 20, 12, 12), torch.uint8, "idx1")
    _req(xn, (B, 784), torch.float32, "xn")
    _req(a2, (B, 800), torch.float32, "a2")
    _req(idx2, (B, 800), torch.uint8, "idx2")
    if lab is not None:
        if src.labels is None:
            raise ValueError("lab output requested but BatchSource has no labels")
        _req(lab, (B,), torch.int32, "lab")
    if stage is not None:
        if not BatchStage.supported(src):
            raise ValueError("a staged batch needs a uint8 source with labels, perm and a device cursor")
        if stage.B < B:
            raise ValueError("stage holds fewer samples than B")
    rc = lib.pto_mnist_conv12_fwd(
        src.x.data_ptr(), int(src.is_u8), _ptr(src.labels), _ptr(src.perm), _ptr(src.cursor),
        src.host_offset, src.n_total, src.scale, src.shift, w1.data_ptr(), b1.data_ptr(),
        w2.data_ptr(), b2.data_ptr(), a1.data_ptr(), idx1.data_ptr(), xn.data_ptr(), _ptr(lab),
        a2.data_ptr(), idx2.data_ptr(), B, _ptr(stage.x if stage else None),
        _ptr(stage.lab if stage else None), _ptr(stage.tag if stage else None), _stream())
    _native.check(rc, "conv12_fwd")
    return a1, idx1, xn, lab, a2, idx2


def fc1_fwd(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor,
            out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """relu(x @ w.T + b) for x [B,800], w [500,800]."""
    lib = _native.load()
    B = x.shape[0]
    _req(x, (B, 800), torch.float32, "x")
    _req(w, (500, 800), torch.float32, "fc1.weight")
    _req(b, (500,), torch.float32, "fc1.bias")
    out = torch.empty((B, 500), device=x.device) if out is None else out
    _req(out, (B, 500), torch.float32, "h1")
    rc = lib.pto_mnist_fc1_fwd(x.data_ptr(), w.data_ptr(), b.data_ptr(), out.data_ptr(), B,
                               _stream())
    _native.check(rc, "fc1_fwd")
    return out


FC1_KS = 2  # K split of the training-path fc1 (FC1_KS of mnist_kernels.hip)


def fc1_split() -> int:
    """K split of the training-path fc1: 2 (256 workgroups)."""
    return FC1_KS


def fc1_fwd_parts(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None,
                  out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Split-K fc1 forward: the pre-activation partials ``out[z] = x[:, Kz] @ w[:, Kz].T`` over
    2 K slices (2 x 400) as fp32 [2, B, 500], ``bias`` added to ``out[0]``; ``head(...,
    h_second=out[1], h_out=h)`` and ``fc1_bwd_head`` finish ``h = relu(out[0] + out[1])``.  256
    workgroups instead of 128: half the operand bytes per CU on the latency-bound load phase."""
    lib = _native.load()
    B = x.shape[0]
    ks = fc1_split()
    _req(x, (B, 800), torch.float32, "x")
    _req(w, (500, 800), torch.float32, "fc1.weight")
    if bias is not None:
        _req(bias, (500,), torch.float32, "fc1.bias")
    out = torch.empty((ks, B, 500), device=x.device) if out is None else out
    _req(out, (ks, B, 500), torch.float32, "fc1 partials")
    rc = lib.pto_mnist_fc1_fwd_parts(x.data_ptr(), w.data_ptr(), _ptr(bias), out.data_ptr(), B, _stream())
    _native.check(rc, "fc1_fwd_parts")
    return out


def head(h: torch.Tensor, w: torch.Tensor, b: torch.Tensor, lab: torch.Tensor, *,
         grad_scale: float = 0.0, loss_scale: float = 1.0, want_grad: bool = True,
         want_logp: bool = False, stats: Optional[torch.Tensor] = None,
         per_sample: Optional[torch.Tensor] = None, dlogits: Optional[torch.Tensor] = None,
         dh: Optional[torch.Tensor] = None, logp: Optional[torch.Tensor] = None,
         h_second: Optional[torch.Tensor] = None, h_out: Optional[torch.Tensor] = None):
    """fc2 + log_softmax + nll (+ d(logits), dh with the fc1 ReLU mask).

    ``lab``: int32 [B] targets (``conv1_fwd`` gathers them).  ``per_sample`` (fp32
    [B,2]) receives (loss, correct) per sample; ``stats`` (fp32 [>=2]) accumulates
    ``sum(loss)*loss_scale`` and the correct count atomically.  With ``h_second``
    (``fc1_fwd_parts``), ``h`` is the first split-K half: the kernel forms
    ``relu(h + h_second)`` (``h`` holds the bias) and writes it to ``h_out``.
    """
    lib = _native.load()
    B = h.shape[0]
    _req(h, (B, 500), torch.float32, "h1")
    if h_second is not None:
        _req(h_second, (B, 500), torch.float32, "h_second")
        if h_out is None:
            raise ValueError("h_second needs h_out")
        _req(h_out, (B, 500), torch.float32, "h_out")
    _req(w, (10, 500), torch.float32, "fc2.weight")
    _req(b, (10,), torch.float32, "fc2.bias")
    _req(lab, (B,), torch.int32, "lab")
    dev = h.device
    if want_grad:
        dlogits = torch.empty((B, 10), device=dev) if dlogits is None else dlogits
        dh = torch.empty((B, 500), device=dev) if dh is None else dh
        _req(dlogits, (B, 10), torch.float32, "dlogits")
        _req(dh, (B, 500), torch.float32, "dh")
    else:
        dlogits = dh = None
    if want_logp:
        logp = torch.empty((B, 10), device=dev) if logp is None else logp
        _req(logp, (B, 10), torch.float32, "logp")
    else:
        logp = None
    if per_sample is not None:
        _req(per_sample, (B, 2), torch.float32, "per_sample")
    if stats is not None and (stats.dtype != torch.float32 or stats.numel() < 2):
        raise ValueError("stats must be fp32 with >= 2 elements")
    rc = lib.pto_mnist_head(h.data_ptr(), w.data_ptr(), b.data_ptr(), lab.data_ptr(), B,
                            float(grad_scale), float(loss_scale), _ptr(dlogits), _ptr(dh),
                            _ptr(logp), _ptr(per_sample), _ptr(stats), _ptr(h_second),
                            _ptr(h_out), _stream())
    _native.check(rc, "head")
    return dlogits, dh, logp


FC1_BWD_WGRAD = 1   # dW_fc1, db_fc1
FC1_BWD_DGRAD = 2   # dz2 (input grad, un-pooled + ReLU-masked)
FC1_BWD_FC2 = 4     # dW_fc2, db_fc2, loss statistics
FC1_BWD_ALL = 7


def fc1_bwd(dh, a2, idx2, w1, dlogits, h, gw1, gb1, gw2, gb2, dz2=None, per_sample=None,
            stats=None, loss_scale: float = 1.0, jobs: int = FC1_BWD_ALL,
            src: Optional[BatchSource] = None, stage: Optional["BatchStage"] = None, stage_adv: int = 1,
            xpush: Optional[tuple] = None, dpool: Optional[torch.Tensor] = None):
    """fc1/fc2 weight+bias grads and dz2 [B,50,8,8] (un-pooled, ReLU-masked).

    With ``dpool`` ([B, 800] fp32) the input-gradient job writes d(a2) there, still pooled and
    ReLU-masked, instead of dz2 (``conv_bwd4(..., dpool=, idx2=)`` un-pools it); returns dpool.

    ``jobs`` selects which of the three independent parts to launch (so the weight
    gradients can run on a side stream concurrently with the input gradient).
    With ``per_sample`` (head output) and ``stats``, job FC2 also writes
    ``stats[0] = sum(loss)*loss_scale`` and ``stats[1] = #correct``.
    With ``src`` + ``stage`` (all jobs), ceil(B/4) extra blocks stage the batch of step
    ``cursor + stage_adv`` for the next conv12_fwd.
    ``xpush = (bases, rank, world, shard4, w1_offset[, err_ptr])`` (DDP over xGMI, all jobs): dW_fc1 is also
    pushed into the owning ranks' receive buffers (``XgmiAllReduce.push_info``; ``w1_offset`` =
    float offset of fc1.weight in the flat gradient); the exchange then skips that range.
    """
    lib = _native.load()
    B = dh.shape[0]
    _req(dh, (B, 500), torch.float32, "dh")
    _req(a2, (B, 800), torch.float32, "a2")
    _req(idx2, (B, 800), torch.uint8, "idx2")
    _req(w1, (500, 800), torch.float32, "fc1.weight")
    _req(dlogits, (B, 10), torch.float32, "dlogits")
    _req(h, (B, 500), torch.float32, "h1")
    _req(gw1, (500, 800), torch.float32, "grad fc1.weight")
    _req(gb1, (500,), torch.float32, "grad fc1.bias")
    _req(gw2, (10, 500), torch.float32, "grad fc2.weight")
    _req(gb2, (10,), torch.float32, "grad fc2.bias")
    if dpool is not None:
        _req(dpool, (B, 800), torch.float32, "dpool")
        if dz2 is not None:
            raise ValueError("dz2 and dpool are exclusive")
    else:
        dz2 = torch.empty((B, 50, 8, 8), device=dh.device) if dz2 is None else dz2
        _req(dz2, (B, 50, 8, 8), torch.float32, "dz2")
    out = dpool if dpool is not None else dz2
    if per_sample is not None:
        _req(per_sample, (B, 2), torch.float32, "per_sample")
    if stage is not None:
        if jobs not in (FC1_BWD_ALL, FC1_BWD_DGRAD | FC1_BWD_FC2) or src is None or not BatchStage.supported(src):
            raise ValueError("staging needs jobs DGRAD|FC2 (+WGRAD) and a uint8 BatchSource with labels, perm, cursor")
        if stage.B < B or src.x.data_ptr() % 16:
            raise ValueError("stage too small or unaligned source")
        rc = lib.pto_mnist_fc1_bwd_stage(
            dh.data_ptr(), a2.data_ptr(), idx2.data_ptr(), w1.data_ptr(), dlogits.data_ptr(), h.data_ptr(),
            gw1.data_ptr(), gb1.data_ptr(), gw2.data_ptr(), gb2.data_ptr(), _ptr(dz2), _ptr(per_sample),
            _ptr(stats), float(loss_scale), B, src.x.data_ptr(), src.labels.data_ptr(), src.perm.data_ptr(),
            src.cursor.data_ptr(), src.n_total, int(stage_adv), int(jobs), stage.x.data_ptr(), stage.lab.data_ptr(),
            stage.tag.data_ptr(), _ptr(dpool), _stream())
        _native.check(rc, "fc1_bwd(stage)")
        return out
    if xpush is not None:
        if stage is not None or jobs != FC1_BWD_ALL:
            raise ValueError("xpush runs every job and no staging")
        bases, rank, world, shard4, w1_off = xpush[:5]
        err = xpush[5] if len(xpush) > 5 else None  # the exchange's error word: no push once set
        if w1_off % 4:
            raise ValueError("fc1.weight must start on a float4 boundary of the flat gradient")
        rc = lib.pto_mnist_fc1_bwd_push(
            dh.data_ptr(), a2.data_ptr(), idx2.data_ptr(), w1.data_ptr(), dlogits.data_ptr(), h.data_ptr(),
            gw1.data_ptr(), gb1.data_ptr(), gw2.data_ptr(), gb2.data_ptr(), _ptr(dz2), _ptr(per_sample),
            _ptr(stats), float(loss_scale), B, bases, int(rank), int(world), int(shard4), int(w1_off) // 4,
            err, _ptr(dpool), _stream())
        _native.check(rc, "fc1_bwd(xpush)")
        return out
    rc = lib.pto_mnist_fc1_bwd(dh.data_ptr(), a2.data_ptr(), idx2.data_ptr(), w1.data_ptr(),
                               dlogits.data_ptr(), h.data_ptr(), gw1.data_ptr(), gb1.data_ptr(),
                               gw2.data_ptr(), gb2.data_ptr(), _ptr(dz2), _ptr(per_sample),
                               _ptr(stats), float(loss_scale), int(jobs), B, _ptr(dpool), _stream())
    _native.check(rc, "fc1_bwd")
    return out


def fc1_bwd_head(h_parts, w2, b2, lab, a2, idx2, w1, *, dz2, h_out, dh_out, dlog_out, per_sample,
                 grad_scale: float, src: Optional[BatchSource] = None, stage: Optional["BatchStage"] = None,
                 stage_adv: int = 1, dpool: Optional[torch.Tensor] = None) -> None:
    """fc1 backward with the head fused in (one launch instead of head + fc1_bwd; the world-1
    step).  ``h_parts``: the split-K fc1 pre-activation partials [2, B, 500], the bias in
    ``h_parts[0]`` (``fc1_fwd_parts(..., bias)``).  Writes dz2 (or, with ``dz2=None`` and ``dpool``
    [B, 800], the pooled d(a2) -- see ``fc1_bwd``) and publishes h = relu(p0 + p1), dh, d(logits) and per-sample (loss, correct) for the
    tail (``tail_``).  With ``src`` + ``stage`` it also stages the batch of step
    ``cursor + stage_adv`` (as ``fc1_bwd``)."""
    lib = _native.load()
    B = a2.shape[0]
    if h_parts.dim() != 3 or h_parts.shape[0] != 2 or tuple(h_parts.shape[1:]) != (B, 500) or \
            h_parts.dtype != torch.float32 or not h_parts.is_contiguous():
        raise ValueError("h_parts must be contiguous fp32 [2, B, 500]")
    _req(w2, (10, 500), torch.float32, "fc2.weight")
    _req(b2, (10,), torch.float32, "fc2.bias")
    _req(lab, (B,), torch.int32, "labels")
    _req(a2, (B, 800), torch.float32, "a2")
    _req(idx2, (B, 800), torch.uint8, "idx2")
    _req(w1, (500, 800), torch.float32, "fc1.weight")
    if (dz2 is None) == (dpool is None):
        raise ValueError("exactly one of dz2 / dpool")
    if dz2 is not None:
        _req(dz2, (B, 50, 8, 8), torch.float32, "dz2")
    else:
        _req(dpool, (B, 800), torch.float32, "dpool")
    _req(h_out, (B, 500), torch.float32, "h")
    _req(dh_out, (B, 500), torch.float32, "dh")
    _req(dlog_out, (B, 10), torch.float32, "dlogits")
    _req(per_sample, (B, 2), torch.float32, "per_sample")
    st = (0, 0, 0, 0, 0, 0, 0, 0, 0)
    if stage is not None:
        if src is None or not BatchStage.supported(src) or stage.B < B or src.x.data_ptr() % 16:
            raise ValueError("staging needs a uint8 BatchSource with labels, perm, cursor and a large enough stage")
        st = (src.x.data_ptr(), src.labels.data_ptr(), src.perm.data_ptr(), src.cursor.data_ptr(), src.n_total,
              int(stage_adv), stage.x.data_ptr(), stage.lab.data_ptr(), stage.tag.data_ptr())
    rc = lib.pto_mnist_fc1_bwd_head(h_parts[0].data_ptr(), h_parts[1].data_ptr(), w2.data_ptr(),
                                    b2.data_ptr(), lab.data_ptr(), a2.data_ptr(), idx2.data_ptr(), w1.data_ptr(),
                                    _ptr(dz2), h_out.data_ptr(), dh_out.data_ptr(), dlog_out.data_ptr(),
                                    per_sample.data_ptr(), float(grad_scale), B, *st, _ptr(dpool), _stream())
    _native.check(rc, "fc1_bwd_head")


def tail_(slab: torch.Tensor, B: int, grads: torch.Tensor, params: torch.Tensor, buf: torch.Tensor, *,
          lr: float, momentum: float = 0.0, dampening: float = 0.0, weight_decay: float = 0.0,
          nesterov: bool = False, grad_scale: float = 1.0, first_step: bool = False,
          step_counter: Optional[torch.Tensor] = None, big: Optional[tuple] = None, w1: tuple, fc2: tuple) -> None:
    """The fused-head step's tail: ``slab_reduce_sgd_(..., w1=w1)`` plus fc1_bwd's job 3 --
    ``fc2=(dlogits, h, per_sample, stats, loss_scale, fc2.weight params, momentum, grads or None,
    fc2.bias params, momentum, grads or None)`` -- with SGD applied from the accumulators."""
    lib = _native.load()
    n = params.numel()
    for t, nm in ((grads, "grads"), (params, "params"), (buf, "momentum_buffer")):
        if t.dtype != torch.float32 or not t.is_cuda or not t.is_contiguous() or t.numel() != n:
            raise ValueError(f"{nm} must be contiguous fp32 CUDA with {n} elements")
    if slab.dtype != torch.float32 or not slab.is_contiguous() or slab.dim() != 2 or \
            slab.shape[1] < n or slab.shape[0] < B:
        raise ValueError("slab must be contiguous fp32 [>=B, >=n]")
    dh, a2, w1p, w1m, w1g = w1
    _req(dh, (B, 500), torch.float32, "dh")
    _req(a2, (B, 800), torch.float32, "a2")
    for t, nm in ((w1p, "fc1 params"), (w1m, "fc1 momentum")) + (((w1g, "fc1 grads"),) if w1g is not None else ()):
        if t.dtype != torch.float32 or not t.is_contiguous() or t.numel() < 400500:
            raise ValueError(f"{nm}: contiguous fp32 [fc1.weight (400000) | fc1.bias (500)] expected")
    dlog, h, per_sample, stats, loss_scale, p2, m2, g2, pb, mb, gb = fc2
    _req(dlog, (B, 10), torch.float32, "dlogits")
    _req(h, (B, 500), torch.float32, "h")
    _req(per_sample, (B, 2), torch.float32, "per_sample")
    for t, nm, k in ((p2, "fc2.weight", 5000), (m2, "fc2.weight momentum", 5000), (pb, "fc2.bias", 10),
                     (mb, "fc2.bias momentum", 10)) + (((g2, "fc2.weight grads", 5000),) if g2 is not None else ()) + \
            (((gb, "fc2.bias grads", 10),) if gb is not None else ()):
        if t.dtype != torch.float32 or not t.is_contiguous() or t.numel() < k:
            raise ValueError(f"{nm}: contiguous fp32 with >= {k} elements expected")
    rb, lo, hi = big if big is not None else (B, 0, 0)
    rc = lib.pto_mnist_tail(slab.data_ptr(), B, n, slab.shape[1], grads.data_ptr(), params.data_ptr(),
                            buf.data_ptr(), float(lr), float(momentum), float(dampening), float(weight_decay),
                            float(grad_scale), int(nesterov), int(first_step), _ptr(step_counter), int(rb), int(lo),
                            int(hi), dh.data_ptr(), a2.data_ptr(), w1p.data_ptr(), w1m.data_ptr(), _ptr(w1g),
                            dlog.data_ptr(), h.data_ptr(), per_sample.data_ptr(), stats.data_ptr(), float(loss_scale),
                            p2.data_ptr(), m2.data_ptr(), _ptr(g2), pb.data_ptr(), mb.data_ptr(), _ptr(gb), _stream())
    _native.check(rc, "tail")


def tail_grads_(slab: torch.Tensor, B: int, conv_grads: torch.Tensor, *, big: Optional[tuple], dh, a2,
                fc1_grads: torch.Tensor, dlogits, h, per_sample, stats, loss_scale: float,
                fc2w_grads: torch.Tensor, fc2b_grads: torch.Tensor) -> None:
    """The fused-head step's gradients, stored (DDP over RCCL): ``tail_``'s dW_fc1 / db_fc1 and
    dW_fc2 / db_fc2 tiles and its slab reduction into ``conv_grads``, the loss statistics -- no
    parameter or momentum touched, no cursor advance (the SGD launch after the all-reduces does
    both).  ``fc1_grads``: fc1.weight (400000) then fc1.bias (500), contiguous."""
    lib = _native.load()
    n = conv_grads.numel()
    if conv_grads.dtype != torch.float32 or not conv_grads.is_contiguous():
        raise ValueError("conv_grads must be contiguous fp32")
    if slab.dtype != torch.float32 or not slab.is_contiguous() or slab.dim() != 2 or \
            slab.shape[1] < n or slab.shape[0] < B:
        raise ValueError("slab must be contiguous fp32 [>=B, >=n]")
    _req(dh, (B, 500), torch.float32, "dh")
    _req(a2, (B, 800), torch.float32, "a2")
    _req(dlogits, (B, 10), torch.float32, "dlogits")
    _req(h, (B, 500), torch.float32, "h")
    _req(per_sample, (B, 2), torch.float32, "per_sample")
    for t, nm, k in ((fc1_grads, "fc1 grads", 400500), (fc2w_grads, "fc2.weight grads", 5000),
                     (fc2b_grads, "fc2.bias grads", 10), (stats, "stats", 2)):
        if t.dtype != torch.float32 or not t.is_contiguous() or t.numel() < k:
            raise ValueError(f"{nm}: contiguous fp32 with >= {k} elements expected")
    rb, lo, hi = big if big is not None else (B, 0, 0)
    rc = lib.pto_mnist_tail_grads(slab.data_ptr(), B, n, slab.shape[1], conv_grads.data_ptr(), int(rb), int(lo),
                                  int(hi), dh.data_ptr(), a2.data_ptr(), fc1_grads.data_ptr(), dlogits.data_ptr(),
                                  h.data_ptr(), per_sample.data_ptr(), stats.data_ptr(), float(loss_scale),
                                  fc2w_grads.data_ptr(), fc2b_grads.data_ptr(), _stream())
    _native.check(rc, "tail_grads")


def conv_bwd(dz2, w2, a1, idx1, xn, gw2, gb2, gw1, gb1, want_dz1=False,
             slab: Optional[torch.Tensor] = None):
    """conv2 weight/bias grads, dz1 (internal), conv1 weight/bias grads.

    ``xn`` is the normalised batch [B,784] (``conv1_fwd`` output).
    Without ``slab`` the conv grads are ACCUMULATED with fp32 atomics (zero them
    first).  With ``slab`` ([B, S] fp32, and gw2/gb2/gw1/gb1 being views into
    ``slab[0]``), every sample writes its partial grads into its own slab row
    (plain stores); ``slab_reduce`` then sums the rows deterministically.
    """
    lib = _native.load()
    B = dz2.shape[0]
    _req(dz2, (B, 50, 8, 8), torch.float32, "dz2")
    _req(w2, (50, 20, 5, 5), torch.float32, "conv2.weight")
    _req(a1, (B, 20, 12, 12), torch.float32, "a1")
    _req(idx1, (B, 20, 12, 12), torch.uint8, "idx1")
    _req(xn, (B, 784), torch.float32, "xn")
    _req(gw2, (50, 20, 5, 5), torch.float32, "grad conv2.weight")
    _req(gb2, (50,), torch.float32, "grad conv2.bias")
    _req(gw1, (20, 1, 5, 5), torch.float32, "grad conv1.weight")
    _req(gb1, (20,), torch.float32, "grad conv1.bias")
    stride = 0
    if slab is not None:
        if slab.dim() != 2 or slab.shape[0] < B or not slab.is_contiguous() or \
                slab.dtype != torch.float32:
            raise ValueError("slab must be contiguous fp32 [>=B, S]")
        stride = slab.shape[1]
        lo, hi = slab.data_ptr(), slab.data_ptr() + stride * 4
        for t in (gw2, gb2, gw1, gb1):
            if not (lo <= t.data_ptr() and t.data_ptr() + t.numel() * 4 <= hi):
                raise ValueError("with slab=, grad views must lie inside slab[0]")
    dz1 = torch.empty((B, 20, 24, 24), device=dz2.device) if want_dz1 else None
    rc = lib.pto_mnist_conv_bwd(dz2.data_ptr(), w2.data_ptr(), a1.data_ptr(), idx1.data_ptr(),
                                xn.data_ptr(), gw2.data_ptr(), gb2.data_ptr(), gw1.data_ptr(),
                                gb1.data_ptr(), _ptr(dz1), stride, B, _stream())
    _native.check(rc, "conv_bwd")
    return dz1


CONV2_W = (50, 20, 5, 5)


def conv_bwd4(dpool, idx2, w2, a1, idx1, xn, slab: torch.Tensor, offsets: dict, B: Optional[int] = None):
    """conv backward with dW_conv2 summed over 4-sample chunks (deterministic, no atomics).

    ``dpool`` [B, 800]: d(a2), pooled and ReLU-masked (``fc1_bwd(..., dpool=)`` /
    ``fc1_bwd_head(..., dpool=)``); ``idx2`` [B, 800] uint8: conv12_fwd's pool argmax -- the
    kernel un-pools dz2 while staging.
    ``slab``: contiguous fp32 [>= B, S]; ``offsets``: the row offsets (floats) of
    ``conv2.weight`` / ``conv2.bias`` / ``conv1.weight`` / ``conv1.bias`` inside a row (the
    flat conv-segment layout).  Rows 0..ceil(B/4)-1 receive the chunk partials of
    conv2.weight, rows 0..B-1 the per-sample partials of the other three; reduce with
    ``slab_reduce(..., big=conv_bwd4_rows(B, offsets))``.
    """
    lib = _native.load()
    B = dpool.shape[0] if B is None else B
    _req(dpool, (B, 800), torch.float32, "dpool")
    _req(idx2, (B, 800), torch.uint8, "idx2")
    _req(w2, CONV2_W, torch.float32, "conv2.weight")
    _req(a1, (B, 20, 12, 12), torch.float32, "a1")
    _req(idx1, (B, 20, 12, 12), torch.uint8, "idx1")
    _req(xn, (B, 784), torch.float32, "xn")
    if slab.dim() != 2 or slab.shape[0] < B or not slab.is_contiguous() or slab.dtype != torch.float32:
        raise ValueError("slab must be contiguous fp32 [>=B, S]")
    o = [int(offsets[k]) for k in ("conv2.weight", "conv2.bias", "conv1.weight", "conv1.bias")]
    rc = lib.pto_mnist_conv_bwd4(dpool.data_ptr(), idx2.data_ptr(), w2.data_ptr(), a1.data_ptr(),
                                 idx1.data_ptr(), xn.data_ptr(), slab.data_ptr(), slab.shape[1], *o, B, _stream())
    _native.check(rc, "conv_bwd4")


def synth_mnist(templates: torch.Tensor, n: int, seed: int, noise: float = 0.35):
    """(images uint8 [n, 784], labels int32 [n]) of the synthetic MNIST recipe drawn on the
    device by one kernel (``templates``: fp32 [10, 28, 28] on the device); see
    data/synthetic.py."""
    lib = _native.load()
    _req(templates, (10, 28, 28), torch.float32, "templates")
    img = torch.empty((n, 784), dtype=torch.uint8, device=templates.device)
    lab = torch.empty((n,), dtype=torch.int32, device=templates.device)
    rc = lib.pto_mnist_synth(templates.data_ptr(), img.data_ptr(), lab.data_ptr(), int(n),
                             int(seed) & 0xFFFFFFFF, float(noise), _stream())
    _native.check(rc, "synth_mnist")
    return img, lab


def conv_bwd4_rows(B: int, offsets: dict) -> tuple:
    """(rows, lo, hi): the slab columns conv_bwd4 writes per 4-sample chunk."""
    lo = int(offsets["conv2.weight"])
    return ((B + 3) // 4, lo, lo + 25000)


def slab_reduce(slab: torch.Tensor, B: int, out: torch.Tensor, big: Optional[tuple] = None) -> torch.Tensor:
    """out[o] = sum_{b<B} slab[b, o] for o < out.numel() (deterministic order).
    ``big = (rows, lo, hi)``: columns [lo, hi) sum only their first ``rows`` rows
    (``conv_bwd4_rows``)."""
    lib = _native.load()
    if slab.dtype != torch.float32 or not slab.is_contiguous() or slab.dim() != 2:
        raise ValueError("slab must be contiguous fp32 [rows, S]")
    if B > slab.shape[0]:
        raise ValueError("B exceeds slab rows")
    n = out.numel()
    if out.dtype != torch.float32 or not out.is_contiguous() or n > slab.shape[1]:
        raise ValueError("out must be contiguous fp32 with <= S elements")
    rb, lo, hi = big if big is not None else (B, 0, 0)
    rc = lib.pto_slab_reduce(slab.data_ptr(), B, n, slab.shape[1], out.data_ptr(), int(rb), int(lo), int(hi),
                             _stream())
    _native.check(rc, "slab_reduce")
    return out


def slab_reduce_sgd_(slab: torch.Tensor, B: int, grads: torch.Tensor, params: torch.Tensor,
                     buf: torch.Tensor, *, lr: float, momentum: float = 0.0,
                     dampening: float = 0.0, weight_decay: float = 0.0, nesterov: bool = False,
                     grad_scale: float = 1.0, first_step: bool = False,
                     step_counter: Optional[torch.Tensor] = None,
                     extra: Optional[tuple] = None, big: Optional[tuple] = None,
                     w1: Optional[tuple] = None) -> None:
    """grads = sum_b slab[b, :n]; then SGD(momentum) on params/buf[:n] (one launch).

    ``extra=(params2, grads2, buf2)``: also apply the same SGD to a second,
    already-reduced range in the same launch (e.g. the fc parameters).
    ``big=(rows, lo, hi)``: columns [lo, hi) sum only their first ``rows`` rows.
    ``w1=(dh, a2, params_w1, buf_w1, grads_w1 or None)``: also compute fc1's weight / bias
    gradient (dh^T . a2 and dh's column sums, fc1_bwd's job 1, bit-identical) in this launch and
    apply SGD to it (``params_w1`` = fc1.weight followed by fc1.bias); ``extra`` must then
    exclude those two.
    """
    lib = _native.load()
    n = params.numel()
    for t, nm in ((grads, "grads"), (params, "params"), (buf, "momentum_buffer")):
        if t.dtype != torch.float32 or not t.is_cuda or not t.is_contiguous() or t.numel() != n:
            raise ValueError(f"{nm} must be contiguous fp32 CUDA with {n} elements")
    if slab.dtype != torch.float32 or not slab.is_contiguous() or slab.dim() != 2 or \
            slab.shape[1] < n or slab.shape[0] < B:
        raise ValueError("slab must be contiguous fp32 [>=B, >=n]")
    p2 = g2 = b2 = None
    n2 = 0
    if extra is not None:
        p2, g2, b2 = extra
        n2 = p2.numel()
        for t, nm in ((p2, "params2"), (g2, "grads2"), (b2, "buf2")):
            if t.dtype != torch.float32 or not t.is_contiguous() or t.numel() != n2:
                raise ValueError(f"{nm} must be contiguous fp32 with {n2} elements")
    rb, lo, hi = big if big is not None else (B, 0, 0)
    if w1 is not None:
        dh, a2, w1p, w1m, w1g = w1
        _req(dh, (B, 500), torch.float32, "dh")
        _req(a2, (B, 800), torch.float32, "a2")
        for t, nm in ((w1p, "fc1 params"), (w1m, "fc1 momentum")) + (((w1g, "fc1 grads"),) if w1g is not None else ()):
            if t.dtype != torch.float32 or not t.is_contiguous() or t.numel() < 400500:
                raise ValueError(f"{nm}: contiguous fp32 [fc1.weight (400000) | fc1.bias (500)] expected")
        rc = lib.pto_slab_reduce_sgd_w1(slab.data_ptr(), B, n, slab.shape[1], grads.data_ptr(),
                                        params.data_ptr(), buf.data_ptr(), float(lr), float(momentum),
                                        float(dampening), float(weight_decay), float(grad_scale),
                                        int(nesterov), int(first_step), _ptr(step_counter), _ptr(p2),
                                        _ptr(g2), _ptr(b2), n2, int(rb), int(lo), int(hi), dh.data_ptr(),
                                        a2.data_ptr(), w1p.data_ptr(), w1m.data_ptr(), _ptr(w1g), _stream())
        _native.check(rc, "slab_reduce_sgd(w1)")
        return
    rc = lib.pto_slab_reduce_sgd(slab.data_ptr(), B, n, slab.shape[1], grads.data_ptr(),
                                 params.data_ptr(), buf.data_ptr(), float(lr), float(momentum),
                                 float(dampening), float(weight_decay), float(grad_scale),
                                 int(nesterov), int(first_step), _ptr(step_counter), _ptr(p2),
                                 _ptr(g2), _ptr(b2), n2, int(rb), int(lo), int(hi), _stream())
    _native.check(rc, "slab_reduce_sgd")


def set_debug_buffer(buf: Optional[torch.Tensor]) -> None:
    """Route per-phase wall_clock64 stamps of every kernel into ``buf`` (int64, or None)."""
    _native.load().pto_set_debug_buffer(_ptr(buf))


def sgd_momentum_(params: torch.Tensor, grads: torch.Tensor, buf: torch.Tensor, *, lr: float,
                  momentum: float = 0.0, dampening: float = 0.0, weight_decay: float = 0.0,
                  nesterov: bool = False, grad_scale: float = 1.0, first_step: bool = False,
                  step_counter: Optional[torch.Tensor] = None) -> None:
    """In-place fused SGD(momentum) over flat fp32 buffers (torch.optim.SGD math)."""
    lib = _native.load()
    n = params.numel()
    for t, nm in ((params, "params"), (grads, "grads"), (buf, "momentum_buffer")):
        if t.dtype != torch.float32 or not t.is_cuda or not t.is_contiguous() or t.numel() != n:
            raise ValueError(f"{nm} must be contiguous fp32 CUDA with {n} elements")
    if step_counter is not None and (step_counter.dtype != torch.int32 or not step_counter.is_cuda):
        raise ValueError("step_counter must be int32 CUDA")
    rc = lib.pto_sgd_momentum(params.data_ptr(), grads.data_ptr(), buf.data_ptr(), n, float(lr),
                              float(momentum), float(dampening), float(weight_decay),
                              float(grad_scale), int(nesterov), int(first_step),
                              _ptr(step_counter), _stream())
    _native.check(rc, "sgd_momentum")
