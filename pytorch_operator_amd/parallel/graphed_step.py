"""hipGraph execution of the fused MNIST DDP step.

At B=64 one training step is ~0.84 GFLOP spread over six kernel launches, so
per-launch host cost (3-4 us each from Python) would dominate the device time.
Every mode below replays pre-captured hipGraphs; the device batch cursor advances
inside the SGD launch, so replays walk the dataset without host involvement.

Modes
-----
``eager``       plain launches (debugging / first step).
``graph``       world == 1: one graph holding ``steps_per_graph`` whole steps.
                world  > 1: three graphs per step -- G1 (forward + fc backward),
                G2 (conv backward), G3 (SGD) -- with the two bucket all-reduces
                issued eagerly between them (the fc bucket's RCCL all-reduce
                overlaps G2 on RCCL's own stream; G3 waits for both).
``graph-comm``  the all-reduces are captured too: one graph per step (RCCL
                collectives support stream capture).  Fewest host calls.

With the xGMI peer-memory all-reduce (``parallel.xgmi``, ``grad_sync.fused_sgd``) the
exchange is an ordinary kernel, so ``graph`` captures ``steps_per_graph`` whole DDP
steps exactly like the single-GPU case.
"""
from __future__ import annotations

from typing import Optional

import torch

from ..models.mnist import FusedMnistTrainer


def _capture(fn, device) -> torch.cuda.CUDAGraph:
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    return g


class GraphedStep:
    def __init__(self, trainer: FusedMnistTrainer, mode: str = "graph", steps_per_graph: int = 1):
        if mode not in ("eager", "graph", "graph-comm"):
            raise ValueError(f"unknown mode {mode}")
        self.tr = trainer
        self.sync = trainer.grad_sync  # the gradient path these graphs were built for
        self.mode = mode
        self.steps_per_graph = steps_per_graph if mode != "eager" else 1
        self.world = trainer.grad_sync.world if trainer.grad_sync is not None else 1
        self._graphs = []
        self.internal_steps = 0  # untimed steps taken while preparing the graphs
        if mode == "eager":
            return
        tr = trainer
        if tr._first_step:
            tr.train_step()  # momentum initialisation happens outside any graph
            self.internal_steps += 1
        torch.cuda.synchronize(tr.device)
        # warm the allocator / RCCL on a side stream before capture (torch recommendation)
        s = torch.cuda.Stream(device=tr.device)
        s.wait_stream(torch.cuda.current_stream(tr.device))
        with torch.cuda.stream(s):
            tr.train_step()
        self.internal_steps += 1
        torch.cuda.current_stream(tr.device).wait_stream(s)
        torch.cuda.synchronize(tr.device)
        if self.world == 1 or mode == "graph-comm" or getattr(tr.grad_sync, "fused_sgd", False):
            def whole():
                for _ in range(self.steps_per_graph):
                    tr.train_step()
            self._graphs = [_capture(whole, tr.device)]
        else:
            inv = 1.0 / self.world
            self._g1 = _capture(lambda: tr.forward_backward_fc(), tr.device)
            self._g2 = _capture(lambda: tr.backward_conv(), tr.device)
            self._g3 = _capture(lambda: tr.optimizer_step(grad_scale=inv), tr.device)
        torch.cuda.synchronize(tr.device)

    def run(self, n_steps: int) -> None:
        """Execute ``n_steps`` training steps (must be a multiple of steps_per_graph in graph modes)."""
        tr = self.tr
        tr.grad_sync = self.sync
        if self.mode == "eager":
            for _ in range(n_steps):
                tr.train_step()
            return
        if self._graphs:
            if n_steps % self.steps_per_graph:
                raise ValueError("n_steps must be a multiple of steps_per_graph")
            g = self._graphs[0]
            for _ in range(n_steps // self.steps_per_graph):
                g.replay()
            return
        sync = tr.grad_sync
        for _ in range(n_steps):
            self._g1.replay()
            sync.fc_ready(tr.fc_bucket())
            self._g2.replay()
            sync.conv_ready(tr.conv_bucket())
            sync.finish()
            self._g3.replay()
