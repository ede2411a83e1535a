"""The reference MNIST CNN and its MI355X-native fused trainer.

``Net`` is the reference architecture verbatim in behaviour (jiaqianjing/pytorch-operator
examples/mnist/mnist.py:17-33) and is the plain-PyTorch path (``--kernels torch``) and
the numerics oracle for the HIP kernels.

``FusedMnistTrainer`` runs the same model with the hand-written gfx950 kernels of
``csrc/kernels/mnist_kernels.hip``: all parameters, gradients and momentum buffers
live in three flat fp32 buffers (so the DDP gradient all-reduce is one or two
contiguous RCCL calls and SGD is one multi-tensor launch), activations live in
pre-allocated workspaces, and a whole step can be captured into one hipGraph.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F


class Net(nn.Module):
    """conv1(1,20,5) relu pool conv2(20,50,5) relu pool fc1(800,500) relu fc2(500,10) log_softmax."""

    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(1, 20, 5, 1)
        self.conv2 = nn.Conv2d(20, 50, 5, 1)
        self.fc1 = nn.Linear(4 * 4 * 50, 500)
        self.fc2 = nn.Linear(500, 10)

    def forward(self, x):
        x = F.relu(self.conv1(x))
        x = F.max_pool2d(x, 2, 2)
        x = F.relu(self.conv2(x))
        x = F.max_pool2d(x, 2, 2)
        x = x.view(-1, 4 * 4 * 50)
        x = F.relu(self.fc1(x))
        x = self.fc2(x)
        return F.log_softmax(x, dim=1)


def _pool_at(r: torch.Tensor, code: torch.Tensor) -> torch.Tensor:
    """2x2/stride-2 pooling of ``r`` [B, C, H, W] that takes, per window, the element whose
    in-window code (dy * 2 + dx, the kernels' idx1 / idx2 convention) is ``code``."""
    B, C, H, W = r.shape
    win = r.view(B, C, H // 2, 2, W // 2, 2).permute(0, 1, 2, 4, 3, 5).reshape(B, C, H // 2, W // 2, 4)
    return win.gather(4, code.view(B, C, H // 2, W // 2, 1).long()).squeeze(4)


class DecisionAlignedNet(Net):
    """``Net`` whose discontinuous decisions -- the two max-pool argmaxes and the three ReLU
    masks -- are taken from the HIP step that ran on the same batch (its idx1 / idx2 codes and
    the signs of its a1, a2 and h); every value is torch's own fp32 arithmetic (convs, linears,
    log-softmax, and through the caller NLL, DDP averaging and SGD).

    Why: an argmax between two values within fp32 rounding of each other, or a ReLU input within
    rounding of 0, has no stable decision.  The HIP kernels sum in another order than torch, so
    such a point may go either way -- a different but equally valid gradient, and from then on a
    different trajectory (tools/dbg/grad_diag.py: one flipped conv2 pool window moved the conv
    grads of a batch by 6e-3; fc1 ReLU flips move dW_fc1 rows by O(1/B)).

    ``forward`` records in ``self.decision_gap`` how far torch's own numbers are from every
    decision it was given (relative to the layer's magnitude): torch's window maximum minus its
    value at the given argmax, and |pre-activation| wherever the given ReLU mask disagrees with
    torch's sign.  ~1e-6 means every given decision is torch's own up to rounding."""

    def forward(self, x, idx1=None, idx2=None, m1=None, m2=None, mh=None):
        if idx1 is None:
            return super().forward(x)
        B = x.shape[0]
        z1 = self.conv1(x)
        q1 = _pool_at(z1, idx1)                     # pre-activation at the chosen element
        p1 = q1 * m1.view_as(q1) if m1 is not None else F.relu(q1)
        z2 = self.conv2(p1)
        q2 = _pool_at(z2, idx2.view(B, 50, 4, 4))
        p2 = q2 * m2.view_as(q2) if m2 is not None else F.relu(q2)
        zh = self.fc1(p2.reshape(B, 800))
        h = zh * mh if mh is not None else F.relu(zh)
        with torch.no_grad():
            gap = 0.0
            for z, q, m in ((z1, q1, m1), (z2, q2, m2)):
                mx = F.max_pool2d(z, 2, 2)  # relu and max commute: the window max pre-activation
                scale = float(mx.abs().max().clamp_min(1e-30))
                g = float((F.relu(mx) - F.relu(q)).max()) / scale
                if m is not None:
                    bad = (q > 0) != m.view_as(q).bool()
                    g = max(g, float(q[bad].abs().max()) / scale if bad.any() else 0.0)
                gap = max(gap, g)
            if mh is not None:
                bad = (zh > 0) != mh.bool()
                if bad.any():
                    gap = max(gap, float(zh[bad].abs().max() / zh.abs().max().clamp_min(1e-30)))
            self.decision_gap = max(getattr(self, "decision_gap", 0.0), gap)
        return F.log_softmax(self.fc2(h), dim=1)


PARAM_SPECS: List[Tuple[str, Tuple[int, ...]]] = [
    ("conv1.weight", (20, 1, 5, 5)),
    ("conv1.bias", (20,)),
    ("conv2.weight", (50, 20, 5, 5)),
    ("conv2.bias", (50,)),
    ("fc1.weight", (500, 800)),
    ("fc1.bias", (500,)),
    ("fc2.weight", (10, 500)),
    ("fc2.bias", (10,)),
]
NUM_PARAMS = sum(int(torch.Size(s).numel()) for _, s in PARAM_SPECS)  # 431080
_CONV_NAMES = ("conv1.weight", "conv1.bias", "conv2.weight", "conv2.bias")
_FC_NAMES = ("fc1.weight", "fc1.bias", "fc2.weight", "fc2.bias")
_ALIGN = 16  # floats (64 B) per segment start


@dataclass
class FlatLayout:
    offsets: Dict[str, int]
    total: int
    conv_end: int  # [0, conv_end) = conv grads (atomically accumulated) -> bucket 2
    # [conv_end, total) = fc grads (written by fc1_bwd)        -> bucket 1


def flat_layout() -> FlatLayout:
    offs, o = {}, 0
    for name, shape in PARAM_SPECS:
        offs[name] = o
        n = int(torch.Size(shape).numel())
        o += (n + _ALIGN - 1) // _ALIGN * _ALIGN
    return FlatLayout(offs, o, offs["fc1.weight"])


def _views(flat: torch.Tensor, layout: FlatLayout) -> Dict[str, torch.Tensor]:
    out = {}
    for name, shape in PARAM_SPECS:
        o = layout.offsets[name]
        n = int(torch.Size(shape).numel())
        out[name] = flat[o:o + n].view(shape)
    return out


def K_stage(source, B: int, device):
    """A next-batch staging slot when the source supports one (uint8 + perm + cursor)."""
    from ..ops.mnist import BatchStage
    return BatchStage(B, device) if source is not None and BatchStage.supported(source) else None


def reference_init(seed: int = 1) -> Dict[str, torch.Tensor]:
    """Parameters exactly as ``torch.manual_seed(seed); Net()`` creates them."""
    g = torch.random.get_rng_state()
    torch.manual_seed(seed)
    net = Net()
    torch.random.set_rng_state(g)
    return {k: v.detach().clone() for k, v in net.state_dict().items()}


class FusedMnistTrainer:
    """One DDP rank's MNIST training state + step on the HIP kernels.

    Parameters
    ----------
    batch_size: per-rank batch (reference default 64).
    source: ``ops.mnist.BatchSource`` with labels (uint8 pixels normalised in-kernel).
    lr, momentum, dampening, weight_decay, nesterov: torch.optim.SGD hyper-parameters.
    grad_sync: optional object with ``fc_ready(t)``, ``conv_ready(t)`` and
        ``finish() -> grad_scale`` hooks (see ``parallel.ddp.FlatGradAllReduce``);
        ``None`` = single process.
    """

    def __init__(self, batch_size: int = 64, source=None, lr: float = 0.01, momentum: float = 0.5,
                 dampening: float = 0.0, weight_decay: float = 0.0, nesterov: bool = False,
                 device: Optional[torch.device] = None, seed: int = 1, grad_sync=None):
        from ..ops import mnist as K  # noqa: N812
        self.K = K
        self.device = torch.device(device or "cuda")
        self.B = int(batch_size)
        self.lr, self.momentum, self.dampening = lr, momentum, dampening
        self.weight_decay, self.nesterov = weight_decay, nesterov
        self.layout = flat_layout()
        L = self.layout.total
        dev = self.device
        self._fp = torch.zeros(L, device=dev)
        # grads are overwritten (never accumulated, so never zeroed) by the launches that
        # produce them -- but not every step form stores every gradient: the default world-1
        # step applies SGD to fc1/fc2 straight from the MFMA accumulators and the xGMI step
        # reduces conv grads in the exchange.  ``grads`` therefore raises for the segments the
        # last step did not store (``_stale``); stats = (loss, #correct) of the step
        self.flat_grads = torch.zeros(L, device=dev)
        self.stats = torch.zeros(16, device=dev)
        self._fm = torch.zeros(L, device=dev)
        self._pv = _views(self._fp, self.layout)
        self._gv = _views(self.flat_grads, self.layout)
        self._stale: Tuple[str, ...] = ()
        # device batch cursor: advanced by the SGD launch, read by conv12_fwd / fc1_bwd's staging
        self.cursor = source.cursor if (source is not None and source.cursor is not None) \
            else torch.zeros(1, device=dev, dtype=torch.int32)
        self.load_state_dict(reference_init(seed))
        self.grad_sync = grad_sync
        # torch.optim.SGD's first step sets buf = d_p; with dampening == 0 the steady-state
        # update buf = momentum * buf + d_p on the zero-initialised buffer is bit-identical
        # (momentum * 0 + d_p == d_p), so every step -- the first included -- is the same
        # graph-capturable launch sequence
        self._first_step = dampening != 0.0
        self.source = source
        self._alloc(self.B)
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        # step knobs (defaults measured on MI355X, docs/kernels.md):
        #   fuse_conv12: conv1 + conv2 forward as one launch (False: the two standalone kernels)
        #   conv_chunk 4: conv_bwd4 sums dW_conv2 over 4-sample chunks -> the slab the tail
        #                 reduces is 4x smaller (1: the per-sample conv_bwd, the fallback)
        #   stage_batches: fc1_bwd stages the next step's batch; conv12 reads it with one load
        self.fuse_conv12 = True
        self.conv_chunk = 4
        self.stage_batches = True
        #   w1_tail: the single-process step computes dW_fc1 / db_fc1 in the tail launch and
        #            applies SGD from the accumulators (fc1_bwd runs only dz2 + fc2 + staging);
        #            materialize_fc1_grad: the tail also stores that gradient into flat_grads
        self.w1_tail = os.environ.get("PTO_W1_TAIL", "1") != "0"
        self.materialize_fc1_grad = False
        #   fuse_head (with w1_tail): fc1_bwd recomputes the head of its sample tile on MFMA (no
        #             head launch); dW_fc2 / db_fc2 / statistics move to the tail with their SGD
        self.fuse_head = os.environ.get("PTO_FUSE_HEAD", "1") != "0"
        #   ddp_fused (world > 1, round 6): the DDP step on the same four forward/backward launches
        #             plus a gradient tail (forward_backward_fused) -- over RCCL one all-reduce of
        #             the whole flat gradient and one SGD launch; over xGMI the exchange computes the
        #             fc gradients itself (five launches).  0: the round-5 forms (head + fc1_bwd)
        self.ddp_fused = os.environ.get("PTO_DDP_FUSED", "1") != "0"

    # ---------------------------------------------------------------- state
    @property
    def flat_params(self) -> torch.Tensor:
        return self._fp

    @property
    def flat_momentum(self) -> torch.Tensor:
        return self._fm

    @property
    def params(self) -> Dict[str, torch.Tensor]:
        return self._pv

    @property
    def grads(self) -> Dict[str, torch.Tensor]:
        """Per-parameter gradient views of ``flat_grads`` as the last step stored them.

        Raises if that step did not store some of them (their buffer then holds an older
        step's values): the default single-process step keeps the fc gradients in registers
        (set ``materialize_fc1_grad = True`` to also store them), the xGMI step the conv and
        dW_fc1 gradients.  ``forward_backward()`` stores all of them."""
        if self._stale:
            raise RuntimeError(f"gradients {list(self._stale)} were not stored by the last step "
                               "(materialize_fc1_grad=True, or forward_backward(), stores them)")
        return self._gv

    def _alloc(self, B: int):
        dev = self.device
        self.a1 = torch.empty((B, 20, 12, 12), device=dev)
        self.idx1 = torch.empty((B, 20, 12, 12), device=dev, dtype=torch.uint8)
        self.a2 = torch.empty((B, 800), device=dev)
        self.idx2 = torch.empty((B, 800), device=dev, dtype=torch.uint8)
        self.h1 = torch.empty((B, 500), device=dev)
        self.dlogits = torch.empty((B, 10), device=dev)
        self.dh = torch.empty((B, 500), device=dev)
        self.dz2 = torch.empty((B, 50, 8, 8), device=dev)
        self.dpool = torch.empty((B, 800), device=dev)
        self.xn = torch.empty((B, 784), device=dev)
        self.lab = torch.empty((B,), device=dev, dtype=torch.int32)
        self.per_sample = torch.empty((B, 2), device=dev)
        self.fc1_ks = self.K.fc1_split()
        self.h_parts = torch.empty(self.fc1_ks * B * 500, device=dev)  # split-K fc1 pre-activations
        self.stage = K_stage(self.source, B, dev)
        # conv-grad slabs in the flat conv-segment layout (pads stay 0): per-sample rows, or
        # (conv_bwd4) per-4-sample-chunk rows for conv2.weight
        self.conv_slab = torch.zeros((B, self.layout.conv_end), device=dev)
        self.slab_views = {
            k: self.conv_slab[0][self.layout.offsets[k]:self.layout.offsets[k] +
                                 int(torch.Size(shape).numel())].view(shape)
            for k, shape in PARAM_SPECS if self.layout.offsets[k] < self.layout.conv_end}

    def state_dict(self) -> Dict[str, torch.Tensor]:
        return {k: v.detach().clone() for k, v in self.params.items()}

    def load_state_dict(self, sd: Dict[str, torch.Tensor]) -> None:
        for k, v in self.params.items():
            v.copy_(sd[k].to(v.device, torch.float32).view(v.shape))

    def momentum_state(self) -> Dict[str, torch.Tensor]:
        return {k: v.detach().clone() for k, v in _views(self.flat_momentum, self.layout).items()}

    def fc_bucket(self) -> torch.Tensor:
        return self.flat_grads[self.layout.conv_end:]

    def conv_bucket(self) -> torch.Tensor:
        return self.flat_grads[:self.layout.conv_end]

    # ---------------------------------------------------------------- step
    #
    # One single-process step is five launches (round 5; one hipGraph, or the captured kernel
    # list launched from C++ -- parallel/graphed_step.py):
    #
    #   conv12_fwd -> fc1_fwd<2> -> fc1_bwd_head (head recomputed per tile + d(a2) pooled +
    #   next-batch staging) -> conv_bwd4 -> tail (dW_fc1 / dW_fc2 tiles with SGD, conv slab
    #   reduction + SGD, cursor advance)
    #
    # (fuse_head / w1_tail off, or world > 1: the six-launch form with head + fc1_bwd.)
    #
    # Fusing a pair across an in-launch hand-off (last-arriving workgroups continue, write-through
    # stores + an arrival counter) measured slower than the launch boundary it removes: fc1 + head
    # +5.3 us, conv_bwd4 + tail +7.3 to +10.8 us per step (profiles/r4_inlaunch_handoff_ab.txt).
    #
    # DDP: with the xGMI kernel the tail launch is the cross-GPU exchange + SGD
    # (parallel/xgmi.py); with RCCL the fc / conv buckets are all-reduced between the pieces.
    def invalidate_stage(self) -> None:
        """Drop the staged next batch (call after changing the source's perm in place)."""
        if self.stage is not None:
            self.stage.invalidate()

    def _stage_for(self, source) -> object:
        return self.stage if (self.stage_batches and self.stage is not None and
                              (source is None or source is self.source)) else None

    def forward(self, source=None, B: Optional[int] = None) -> None:
        """conv12_fwd (or conv1_fwd + conv2_fwd) + split-K fc1 (the head finishes h)."""
        K, p = self.K, self._pv
        src = source or self.source
        B = self.B if B is None else B
        if self.fuse_conv12:
            K.conv12_fwd(src, p["conv1.weight"], p["conv1.bias"], p["conv2.weight"],
                         p["conv2.bias"], B, a1=self.a1[:B], idx1=self.idx1[:B], xn=self.xn[:B],
                         lab=self.lab[:B], a2=self.a2[:B], idx2=self.idx2[:B],
                         stage=self._stage_for(source))
        else:
            K.conv1_fwd(src, p["conv1.weight"], p["conv1.bias"], B, out=self.a1[:B],
                        idx=self.idx1[:B], xn=self.xn[:B], lab=self.lab[:B])
            K.conv2_fwd(self.a1[:B], p["conv2.weight"], p["conv2.bias"], out=self.a2[:B],
                        idx=self.idx2[:B])
        ks = self.fc1_ks
        K.fc1_fwd_parts(self.a2[:B], p["fc1.weight"], p["fc1.bias"],
                        out=self.h_parts[:ks * B * 500].view(ks, B, 500))

    def _head(self, B: int) -> None:
        """h = relu(part0 + part1) (part0 holds the bias), fc2, log-softmax, NLL, d(logits), dh (one launch)."""
        K, p = self.K, self._pv
        hp = self.h_parts[:self.fc1_ks * B * 500].view(self.fc1_ks, B, 500)
        K.head(hp[0], p["fc2.weight"], p["fc2.bias"], self.lab[:B], grad_scale=1.0 / B,
               per_sample=self.per_sample[:B], dlogits=self.dlogits[:B], dh=self.dh[:B],
               h_second=hp[1], h_out=self.h1[:B])

    def _dz2_out(self, B: int) -> dict:
        """Where the input-gradient job writes: d(a2) still pooled ([B, 800], 3.2 KB per sample; conv_bwd4
        un-pools it through idx2 -- round 5: -0.5 us per step, profiles/r5_dpool/ab.txt) or, for the
        per-sample conv_bwd, the dense dz2."""
        if self.conv_chunk == 4:
            return {"dz2": None, "dpool": self.dpool[:B]}
        return {"dz2": self.dz2[:B], "dpool": None}

    def _fc1_bwd(self, B: int, stage_adv: Optional[int] = None, xpush: Optional[tuple] = None,
                 jobs: Optional[int] = None) -> None:
        """fc1_bwd; with ``stage_adv`` (and staging on), also stage the batch of cursor + stage_adv;
        with ``xpush``, also push dW_fc1 to its xGMI owners (ops.mnist.fc1_bwd)."""
        K, p, g = self.K, self._pv, self._gv
        st = self._stage_for(None) if stage_adv is not None and xpush is None else None
        K.fc1_bwd(self.dh[:B], self.a2[:B], self.idx2[:B], p["fc1.weight"], self.dlogits[:B],
                  self.h1[:B], g["fc1.weight"], g["fc1.bias"], g["fc2.weight"], g["fc2.bias"],
                  **self._dz2_out(B), per_sample=self.per_sample[:B], stats=self.stats,
                  loss_scale=1.0 / B, jobs=K.FC1_BWD_ALL if jobs is None else jobs,
                  src=self.source if st is not None else None,
                  stage=st, stage_adv=stage_adv or 0, xpush=xpush)

    def _fc1_bwd_head(self, B: int, stage_adv: int) -> None:
        """fc1_bwd with the head fused in (ops.mnist.fc1_bwd_head)."""
        K, p = self.K, self._pv
        st = self._stage_for(None)
        K.fc1_bwd_head(self.h_parts[:2 * B * 500].view(2, B, 500), p["fc2.weight"], p["fc2.bias"],
                       self.lab[:B], self.a2[:B], self.idx2[:B], p["fc1.weight"], **self._dz2_out(B),
                       h_out=self.h1[:B], dh_out=self.dh[:B], dlog_out=self.dlogits[:B],
                       per_sample=self.per_sample[:B], grad_scale=1.0 / B,
                       src=self.source if st is not None else None, stage=st, stage_adv=stage_adv)

    def _conv_bwd(self, B: int) -> None:
        K, p = self.K, self._pv
        if self.conv_chunk == 4:
            K.conv_bwd4(self.dpool[:B], self.idx2[:B], p["conv2.weight"], self.a1[:B], self.idx1[:B],
                        self.xn[:B], self.conv_slab, self.layout.offsets, B)
            self._last_big = K.conv_bwd4_rows(B, self.layout.offsets)
            return
        self._last_big = None
        sv = self.slab_views
        K.conv_bwd(self.dz2[:B], p["conv2.weight"], self.a1[:B], self.idx1[:B], self.xn[:B],
                   sv["conv2.weight"], sv["conv2.bias"], sv["conv1.weight"], sv["conv1.bias"],
                   slab=self.conv_slab)

    def _slab_big(self, B: int):
        """Chunk-row geometry of the slab the last conv backward wrote (None: per-sample rows)."""
        return getattr(self, "_last_big", None)

    def _sgd(self, lo: int, hi: int, grad_scale: float, advance_cursor: bool) -> None:
        self.K.sgd_momentum_(self._fp[lo:hi], self.flat_grads[lo:hi],
                             self._fm[lo:hi], lr=self.lr, momentum=self.momentum,
                             dampening=self.dampening, weight_decay=self.weight_decay,
                             nesterov=self.nesterov, grad_scale=grad_scale,
                             first_step=self._first_step,
                             step_counter=self.cursor if advance_cursor else None)

    def forward_backward_fc(self, source=None, B: Optional[int] = None) -> None:
        """Forward + loss + fc backward (the fc bucket and dz2 are complete after this)."""
        B = self.B if B is None else B
        self.forward(source, B)
        self._head(B)
        self._fc1_bwd(B)

    def backward_conv(self, source=None, B: Optional[int] = None) -> None:
        """conv backward + deterministic slab reduction into the conv bucket."""
        B = self.B if B is None else B
        self._conv_bwd(B)
        self.K.slab_reduce(self.conv_slab, B, self.conv_bucket(), big=self._slab_big(B))

    def fused_ok(self) -> bool:
        """The fused-head DDP forms apply (fc1 split-K 2: fc1_bwd_head's partial layout)."""
        return self.ddp_fused and self.fc1_ks == 2

    def forward_backward_fused(self, source=None, B: Optional[int] = None, stage_adv: int = 1) -> None:
        """The DDP step's forward and backward on the world-1 step's kernels, every gradient stored
        (five launches): conv12_fwd -> fc1_fwd<2> -> fc1_bwd_head (+ staging of the batch of cursor +
        ``stage_adv``) -> conv_bwd4 -> tail_grads (dW_fc1 / db_fc1 / dW_fc2 / db_fc2 tiles, the conv
        slab reduction, the loss statistics).  Both buckets are complete when it returns."""
        B = self.B if B is None else B
        K, ce = self.K, self.layout.conv_end
        o2w, o2b = self.layout.offsets["fc2.weight"], self.layout.offsets["fc2.bias"]
        self.forward(source, B)
        self._fc1_bwd_head(B, stage_adv=stage_adv)
        self._conv_bwd(B)
        K.tail_grads_(self.conv_slab, B, self.conv_bucket(), big=self._slab_big(B), dh=self.dh[:B], a2=self.a2[:B],
                      fc1_grads=self.flat_grads[ce:o2w], dlogits=self.dlogits[:B], h=self.h1[:B],
                      per_sample=self.per_sample[:B], stats=self.stats, loss_scale=1.0 / B,
                      fc2w_grads=self.flat_grads[o2w:o2b], fc2b_grads=self.flat_grads[o2b:])
        self._stale = ()

    def forward_backward(self, source=None, B: Optional[int] = None) -> None:
        """All fwd/bwd launches for one batch; grads land in flat_grads (DDP hooks fire)."""
        self.forward_backward_fc(source, B)
        if self.grad_sync is not None:
            self.grad_sync.fc_ready(self.fc_bucket())
        self.backward_conv(source, B)
        if self.grad_sync is not None:
            self.grad_sync.conv_ready(self.conv_bucket())
        self._stale = ()

    def optimizer_step(self, advance_cursor: bool = True, grad_scale: Optional[float] = None) -> None:
        if grad_scale is None:
            grad_scale = self.grad_sync.finish() if self.grad_sync is not None else 1.0
        self._sgd(0, self.layout.total, grad_scale, advance_cursor)
        self._first_step = False

    def train_step(self, source=None, B: Optional[int] = None, advance_cursor: bool = True):
        """One full training step (forward, backward, [all-reduce], SGD)."""
        B = self.B if B is None else B
        if getattr(self.grad_sync, "fused_sgd", False) and self.fused_ok():
            # xGMI, fused (five launches): conv12_fwd -> fc1_fwd<2> -> fc1_bwd_head -> conv_bwd4 ->
            # the exchange, which computes dW_fc1 / db_fc1 / dW_fc2 / db_fc2 (and the loss
            # statistics) itself, deposits them and the slab-reduced conv gradient with their
            # owners, applies SGD to this rank's shard and all-gathers the parameters.  flat_grads
            # is not written.
            xar = self.grad_sync.xar
            o = self.layout.offsets
            self.forward(source, B)
            self._fc1_bwd_head(B, stage_adv=1 if advance_cursor else 0)
            self._conv_bwd(B)
            xar.allreduce_sgd_fc_(
                self.flat_grads, self._fp, self._fm, lr=self.lr, momentum=self.momentum,
                dampening=self.dampening, weight_decay=self.weight_decay, nesterov=self.nesterov,
                first_step=self._first_step, step_counter=self.cursor if advance_cursor else None,
                slab=self.conv_slab, slab_rows=B, conv_n=self.layout.conv_end, slab_big=self._slab_big(B),
                fc=(self.dh[:B], self.a2[:B], self.dlogits[:B], self.h1[:B], self.per_sample[:B], self.stats,
                    1.0 / B, (o["fc1.weight"], o["fc1.bias"], o["fc2.weight"], o["fc2.bias"])))
            self._first_step = False
            self._stale = _CONV_NAMES + _FC_NAMES
            return
        if getattr(self.grad_sync, "fused_sgd", False):
            # xGMI path: one kernel reduces the per-sample conv-grad slabs, does the
            # cross-GPU reduce-scatter, SGD on this rank's shard and the all-gather of the
            # updated parameters (parallel/xgmi.py).  flat_grads[:conv_end] is not written.
            # fc1_bwd pushes dW_fc1 (93.9 % of the gradient) into its owners' receive buffers
            # itself; the exchange produces and pushes only the rest
            xar = self.grad_sync.xar
            w1o = self.layout.offsets["fc1.weight"]
            push = getattr(self.grad_sync, "push_fc1", True)
            self.forward(source, B)
            self._head(B)
            self._fc1_bwd(B, xpush=(*xar.push_info(), w1o, xar.err_ptr()) if push else None)
            self._conv_bwd(B)
            self.grad_sync.xar.allreduce_sgd_(
                self.flat_grads, self._fp, self._fm, lr=self.lr,
                momentum=self.momentum, dampening=self.dampening, weight_decay=self.weight_decay,
                nesterov=self.nesterov, first_step=self._first_step,
                step_counter=self.cursor if advance_cursor else None,
                slab=self.conv_slab, slab_rows=B, conv_n=self.layout.conv_end,
                slab_big=self._slab_big(B), skip=(w1o, w1o + 400000) if push else None)
            self._first_step = False
            self._stale = _CONV_NAMES + (("fc1.weight",) if push else ())
            return
        if self.grad_sync is not None:
            if self.fused_ok():
                # six launches + ONE all-reduce of the whole flat gradient (both buckets are complete
                # at the same time, so one collective instead of two)
                self.forward_backward_fused(source, B, stage_adv=1 if advance_cursor else 0)
                self.grad_sync.all_ready(self.flat_grads)
                self.optimizer_step(advance_cursor)
                return
            self.forward_backward(source, B)
            self.optimizer_step(advance_cursor)
            return
        K = self.K
        ce = self.layout.conv_end
        if self.w1_tail and self.fuse_head and self.fc1_ks == 2:
            # 5 launches: conv12_fwd -> fc1_fwd<2> -> fc1_bwd_head -> conv_bwd4 -> tail
            self.forward(source, B)
            self._fc1_bwd_head(B, stage_adv=1 if advance_cursor else 0)
            self._conv_bwd(B)
            o2w, o2b = self.layout.offsets["fc2.weight"], self.layout.offsets["fc2.bias"]
            mat = self.materialize_fc1_grad
            K.tail_(self.conv_slab, B, self.conv_bucket(), self._fp[:ce], self._fm[:ce], lr=self.lr,
                    momentum=self.momentum, dampening=self.dampening, weight_decay=self.weight_decay,
                    nesterov=self.nesterov, first_step=self._first_step,
                    step_counter=self.cursor if advance_cursor else None, big=self._slab_big(B),
                    w1=(self.dh[:B], self.a2[:B], self._fp[ce:o2w], self._fm[ce:o2w],
                        self.flat_grads[ce:o2w] if mat else None),
                    fc2=(self.dlogits[:B], self.h1[:B], self.per_sample[:B], self.stats, 1.0 / B,
                         self._fp[o2w:o2b], self._fm[o2w:o2b], self.flat_grads[o2w:o2b] if mat else None,
                         self._fp[o2b:], self._fm[o2b:], self.flat_grads[o2b:] if mat else None))
            self._first_step = False
            self._stale = () if mat else _FC_NAMES
            return
        # 6 launches: conv12_fwd -> fc1_fwd<2> -> head -> fc1_bwd -> conv_bwd4 -> tail
        self.forward(source, B)
        self._head(B)
        w1t = self.w1_tail
        self._fc1_bwd(B, stage_adv=1 if advance_cursor else 0,
                      jobs=(K.FC1_BWD_DGRAD | K.FC1_BWD_FC2) if w1t else None)
        self._conv_bwd(B)
        e0 = self.layout.offsets["fc2.weight"] if w1t else ce  # the plain-SGD range
        w1 = (self.dh[:B], self.a2[:B], self._fp[ce:e0], self._fm[ce:e0],
              self.flat_grads[ce:e0] if self.materialize_fc1_grad else None) if w1t else None
        K.slab_reduce_sgd_(self.conv_slab, B, self.conv_bucket(), self._fp[:ce],
                           self._fm[:ce], lr=self.lr, momentum=self.momentum,
                           dampening=self.dampening, weight_decay=self.weight_decay,
                           nesterov=self.nesterov, first_step=self._first_step,
                           step_counter=self.cursor if advance_cursor else None,
                           extra=(self._fp[e0:], self.flat_grads[e0:], self._fm[e0:]),
                           big=self._slab_big(B), w1=w1)
        self._first_step = False
        self._stale = ("fc1.weight", "fc1.bias") if w1t and not self.materialize_fc1_grad else ()

    def loss(self) -> float:
        return float(self.stats[0].item())

    # ---------------------------------------------------------------- graphs
    def capture(self, steps_per_graph: int = 1, warmup: int = 0) -> torch.cuda.CUDAGraph:
        """Capture ``steps_per_graph`` whole training steps into one hipGraph.

        Requires a ``source`` with a device ``cursor`` (so replays read successive
        batches).  The first (momentum-initialising) step runs eagerly before the
        capture so the graph only contains steady-state steps.
        """
        if self.source is None or self.source.cursor is None:
            raise ValueError("graph capture needs a BatchSource with a device cursor")
        if self._first_step:
            self.train_step()
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self.train_step()
        torch.cuda.current_stream(self.device).wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(steps_per_graph):
                self.train_step()
        self.graph = g
        return g

    # ---------------------------------------------------------------- eval
    @torch.no_grad()
    def evaluate(self, source, n: Optional[int] = None, batch_size: int = 1000) -> Tuple[float, float]:
        """Average NLL and accuracy over the first ``n`` samples of ``source`` (B=1000 batches)."""
        K, p = self.K, self.params
        n = source.n_total if n is None else n
        dev = self.device
        a1 = torch.empty((batch_size, 20, 12, 12), device=dev)
        idx1 = torch.empty((batch_size, 20, 12, 12), device=dev, dtype=torch.uint8)
        a2 = torch.empty((batch_size, 800), device=dev)
        idx2 = torch.empty((batch_size, 800), device=dev, dtype=torch.uint8)
        h1 = torch.empty((batch_size, 500), device=dev)
        xn = torch.empty((batch_size, 784), device=dev)
        lab = torch.empty((batch_size,), device=dev, dtype=torch.int32)
        stats = torch.zeros(16, device=dev)
        from ..ops.mnist import BatchSource
        ident = torch.arange(source.n_total, device=dev, dtype=torch.int32) \
            if source.perm is None else source.perm
        for off in range(0, n, batch_size):
            B = min(batch_size, n - off)
            sub = BatchSource(source.x, source.labels, perm=ident, host_offset=off,
                              normalize=None)
            sub.scale, sub.shift = source.scale, source.shift
            K.conv12_fwd(sub, p["conv1.weight"], p["conv1.bias"], p["conv2.weight"],
                         p["conv2.bias"], B, a1=a1[:B], idx1=idx1[:B], xn=xn[:B], lab=lab[:B],
                         a2=a2[:B], idx2=idx2[:B])
            K.fc1_fwd(a2[:B], p["fc1.weight"], p["fc1.bias"], out=h1[:B])
            K.head(h1[:B], p["fc2.weight"], p["fc2.bias"], lab[:B], loss_scale=1.0,
                   want_grad=False, stats=stats)
        s = stats.cpu()
        return float(s[0]) / n, float(s[1]) / n
