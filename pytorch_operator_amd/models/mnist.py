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
        self.flat_params = torch.zeros(L, device=dev)
        # grads are fully overwritten every step (no zeroing): fc grads by fc1_bwd, conv
        # grads by the deterministic slab reduction; stats = (loss, #correct) of the step
        self.flat_grads = torch.zeros(L, device=dev)
        self.stats = torch.zeros(16, device=dev)
        self.flat_momentum = torch.zeros(L, device=dev)
        self.params = _views(self.flat_params, self.layout)
        self.grads = _views(self.flat_grads, self.layout)
        # device batch cursor: advanced by the SGD launch, read by conv1_fwd/head/conv_bwd
        self.cursor = source.cursor if (source is not None and source.cursor is not None) \
            else torch.zeros(1, device=dev, dtype=torch.int32)
        self.load_state_dict(reference_init(seed))
        self.grad_sync = grad_sync
        self._first_step = True
        self.source = source
        self._alloc(self.B)
        self.graph: Optional[torch.cuda.CUDAGraph] = None

    # ---------------------------------------------------------------- state
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
        self.xn = torch.empty((B, 784), device=dev)
        self.lab = torch.empty((B,), device=dev, dtype=torch.int32)
        self.per_sample = torch.empty((B, 2), device=dev)
        # per-sample conv-grad slabs in the flat conv-segment layout (pads stay 0)
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
    def forward_backward_fc(self, source=None, B: Optional[int] = None) -> None:
        """Launches A-E: forward, loss, fc1/fc2 grads (the fc bucket is complete after this)."""
        K, p, g = self.K, self.params, self.grads
        src = source or self.source
        B = self.B if B is None else B
        a1, idx1, xn, lab = self.a1[:B], self.idx1[:B], self.xn[:B], self.lab[:B]
        a2, idx2, h1 = self.a2[:B], self.idx2[:B], self.h1[:B]
        dlog, dh, dz2, ps = self.dlogits[:B], self.dh[:B], self.dz2[:B], self.per_sample[:B]
        K.conv1_fwd(src, p["conv1.weight"], p["conv1.bias"], B, out=a1, idx=idx1, xn=xn, lab=lab)
        K.conv2_fwd(a1, p["conv2.weight"], p["conv2.bias"], out=a2, idx=idx2)
        K.fc1_fwd(a2, p["fc1.weight"], p["fc1.bias"], out=h1)
        K.head(h1, p["fc2.weight"], p["fc2.bias"], lab, grad_scale=1.0 / B, per_sample=ps,
               dlogits=dlog, dh=dh)
        K.fc1_bwd(dh, a2, idx2, p["fc1.weight"], dlog, h1, g["fc1.weight"], g["fc1.bias"],
                  g["fc2.weight"], g["fc2.bias"], dz2=dz2, per_sample=ps, stats=self.stats,
                  loss_scale=1.0 / B)

    def backward_conv(self, source=None, B: Optional[int] = None) -> None:
        """Launch F: conv2/conv1 grads (the conv bucket is complete after this)."""
        K, p, g = self.K, self.params, self.grads
        B = self.B if B is None else B
        sv = self.slab_views
        K.conv_bwd(self.dz2[:B], p["conv2.weight"], self.a1[:B], self.idx1[:B], self.xn[:B],
                   sv["conv2.weight"], sv["conv2.bias"], sv["conv1.weight"], sv["conv1.bias"],
                   slab=self.conv_slab)
        K.slab_reduce(self.conv_slab, B, self.conv_bucket())

    def forward_backward(self, source=None, B: Optional[int] = None) -> None:
        """Launch the 6 fused fwd/bwd kernels for one batch (grads land in flat_grads)."""
        self.forward_backward_fc(source, B)
        if self.grad_sync is not None:
            self.grad_sync.fc_ready(self.fc_bucket())
        self.backward_conv(source, B)
        if self.grad_sync is not None:
            self.grad_sync.conv_ready(self.conv_bucket())

    def optimizer_step(self, advance_cursor: bool = True, grad_scale: Optional[float] = None) -> None:
        if grad_scale is None:
            grad_scale = self.grad_sync.finish() if self.grad_sync is not None else 1.0
        self.K.sgd_momentum_(self.flat_params, self.flat_grads, self.flat_momentum, lr=self.lr,
                             momentum=self.momentum, dampening=self.dampening,
                             weight_decay=self.weight_decay, nesterov=self.nesterov,
                             grad_scale=grad_scale, first_step=self._first_step,
                             step_counter=self.cursor if advance_cursor else None)
        self._first_step = False

    def train_step(self, source=None, B: Optional[int] = None, advance_cursor: bool = True):
        self.forward_backward(source, B)
        self.optimizer_step(advance_cursor)

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
            K.conv1_fwd(sub, p["conv1.weight"], p["conv1.bias"], B, out=a1[:B], idx=idx1[:B],
                        xn=xn[:B], lab=lab[:B])
            K.conv2_fwd(a1[:B], p["conv2.weight"], p["conv2.bias"], out=a2[:B], idx=idx2[:B])
            K.fc1_fwd(a2[:B], p["fc1.weight"], p["fc1.bias"], out=h1[:B])
            K.head(h1[:B], p["fc2.weight"], p["fc2.bias"], lab[:B], loss_scale=1.0,
                   want_grad=False, stats=stats)
        s = stats.cpu()
        return float(s[0]) / n, float(s[1]) / n
