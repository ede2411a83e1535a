"""hipGraph execution of the fused MNIST DDP step.

At B=64 one training step is ~0.84 GFLOP spread over six kernel launches, so
per-launch host cost (3-4 us each from Python) would dominate the device time.
Every mode below replays pre-captured hipGraphs; the device batch cursor advances
inside the SGD launch, so replays walk the dataset without host involvement.

Modes
-----
``eager``       plain launches (debugging / first step).
``graph``       no collectives (world 1): one graph holding ``steps_per_graph`` whole steps.
                RCCL collectives (world > 1, or forced at world 1), the round-6 fused form
                (``trainer.fused_ok()``): two pieces per step -- the five launches up to the
                complete flat gradient (``forward_backward_fused``), then the SGD launch -- with
                ONE all-reduce of the whole gradient issued eagerly between them.  The round-5
                form (``ddp_fused`` off): three pieces -- G1 (forward + fc backward), G2 (conv
                backward), G3 (SGD) -- with the two bucket all-reduces between them (the fc
                bucket's overlaps G2 on RCCL's own stream; G3 waits for both).  With
                ``launch="stream"`` the pieces are native recordings whose kernel lists are
                launched directly on the stream.
``graph-comm``  the all-reduces are captured too: one graph per step (RCCL
                collectives support stream capture).  Fewest host calls.

With the xGMI peer-memory all-reduce (``parallel.xgmi``, ``grad_sync.fused_sgd``) the
exchange is an ordinary kernel, so ``graph`` captures ``steps_per_graph`` whole DDP
steps exactly like the single-GPU case.

Whole-step graphs are captured natively (``csrc/kernels/graph_exec.hip``): the step
launches only this library's kernels, so the HIP runtime can record it directly, and the
executable graph is staged with ``hipGraphUpload`` right after capture.  Measured on
MI355X (profiles/r2_launch_overhead.json): a graph's FIRST launch still costs ~0.75 us per
node more than later ones, while back-to-back launches of a warm graph cost no more than
one big graph -- so ``warm()`` replays the timed graph itself before falling back to a
one-step graph for the remainder, and a caller sizes ``steps_per_graph`` to fit its warm-up.

``launch="stream"`` (the bench / worker default since round 2) avoids both costs: the
one-step graph's kernel nodes are launched straight onto the stream from C++
(``pto_graph_launch_stream``), because each hipGraphLaunch leaves the GPU idle ~8.6 us
before its first kernel (profiles/r2_k20_timeline.json, r2_launch_ab.json).  A graph with
any non-kernel node keeps graph replay.
"""
from __future__ import annotations

import ctypes
from typing import Callable, Optional

import torch

from ..models.mnist import FusedMnistTrainer
from ..ops import _native


def _capture(fn, device) -> torch.cuda.CUDAGraph:
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    return g


class NativeGraph:
    """A hipGraph recorded from ``fn`` (which must only launch this library's kernels on
    the current stream), instantiated and uploaded; ``replay(n)`` launches it n times."""

    def __init__(self, fn: Callable[[], None], device: torch.device):
        lib = _native.load()
        self._lib = lib
        self.device = device
        s = torch.cuda.Stream(device=device)
        s.wait_stream(torch.cuda.current_stream(device))
        h = ctypes.c_void_p()
        with torch.cuda.stream(s):
            _native.check(lib.pto_graph_begin(s.cuda_stream), "hipStreamBeginCapture")
            try:
                fn()
            finally:
                rc = lib.pto_graph_end(s.cuda_stream, ctypes.byref(h))
        _native.check(rc, "hipStreamEndCapture/hipGraphInstantiate")
        self._h = h
        self.nodes = int(lib.pto_graph_nodes(h))
        # a zero-count stream replay reports whether every node is a kernel (-2 otherwise)
        self.stream_ok = lib.pto_graph_launch_stream(h, s.cuda_stream, 0) == 0
        _native.check(lib.pto_graph_upload(h, s.cuda_stream), "hipGraphUpload")
        s.synchronize()
        torch.cuda.current_stream(device).wait_stream(s)

    def replay(self, n: int = 1) -> None:
        _native.check(self._lib.pto_graph_launch(
            self._h, _native.current_stream_ptr(self.device), int(n)), "hipGraphLaunch")

    def replay_stream(self, n: int = 1) -> None:
        """The captured kernels launched directly on the current stream, ``n`` times over
        (same kernels and arguments as ``replay``; no per-replay graph-launch cost)."""
        _native.check(self._lib.pto_graph_launch_stream(
            self._h, _native.current_stream_ptr(self.device), int(n)), "graph stream replay")

    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.pto_graph_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class GraphedStep:
    """Replays whole training steps.  ``run(n)`` needs ``n % steps_per_graph == 0`` (the
    timed graph); ``warm(n)`` takes any ``n`` (one-step graph)."""

    def __init__(self, trainer: FusedMnistTrainer, mode: str = "graph", steps_per_graph: int = 1,
                 native: bool = True, launch: str = "graph"):
        """``launch`` (whole-step native graphs only): "graph" replays the hipGraph,
        "stream" launches the one-step graph's recorded kernels directly on the stream
        (``NativeGraph.replay_stream``) -- any step count, no graph-launch gaps."""
        if mode not in ("eager", "graph", "graph-comm"):
            raise ValueError(f"unknown mode {mode}")
        if launch not in ("graph", "stream"):
            raise ValueError(f"unknown launch {launch}")
        self.tr = trainer
        self.sync = trainer.grad_sync  # the gradient path these graphs were built for
        self.mode = mode
        self.steps_per_graph = max(1, int(steps_per_graph)) if mode != "eager" else 1
        self.world = trainer.grad_sync.world if trainer.grad_sync is not None else 1
        # collectives issued per step: world > 1, or forced at world 1 (FlatGradAllReduce.active)
        gs = trainer.grad_sync
        self.collectives = gs is not None and bool(getattr(gs, "active", self.world > 1))
        self._graph = None   # timed graph: steps_per_graph whole steps
        self._warm = None    # one whole step (warm-up of any length)
        self._split = False  # RCCL step in pieces with the collectives issued between them
        self._fused = False  # the fused form's two pieces (trainer.fused_ok()) instead of three
        self.internal_steps = 0  # untimed steps taken while preparing the graphs
        self.launch = "graph"
        if mode == "eager":
            return
        try:
            self._prepare(native, launch)
        except Exception as e:
            e.internal_steps = self.internal_steps  # steps taken before the failure (autotune counts them)
            raise

    def _prepare(self, native: bool, launch: str) -> None:
        tr, mode = self.tr, self.mode
        if tr._first_step:
            tr.train_step()  # momentum initialisation happens outside any graph
            self.internal_steps += 1
        torch.cuda.synchronize(tr.device)
        whole_step = not self.collectives or getattr(tr.grad_sync, "fused_sgd", False)
        if not whole_step or mode == "graph-comm":
            # torch capture: RCCL collectives need torch's capture bookkeeping.  Warm the
            # allocator / RCCL on a side stream before capture (torch recommendation).
            s = torch.cuda.Stream(device=tr.device)
            s.wait_stream(torch.cuda.current_stream(tr.device))
            with torch.cuda.stream(s):
                tr.train_step()
            self.internal_steps += 1
            torch.cuda.current_stream(tr.device).wait_stream(s)
            torch.cuda.synchronize(tr.device)
        if whole_step:
            def steps(n):
                def fn():
                    for _ in range(n):
                        tr.train_step()
                return fn
            if native and launch == "stream" and mode == "graph":
                one = NativeGraph(steps(1), tr.device)
                if one.stream_ok:
                    self.launch, self.steps_per_graph = "stream", 1
                    self._graph = self._warm = one
                else:  # a captured node that is not a kernel: graph replay
                    self._warm = one
            if native and self._graph is None:
                self._graph = NativeGraph(steps(self.steps_per_graph), tr.device)
                self._warm = self._warm or (self._graph if self.steps_per_graph == 1 else
                                            NativeGraph(steps(1), tr.device))
            elif not native:
                g = _capture(steps(self.steps_per_graph), tr.device)
                self._graph = _TorchGraph(g)
                self._warm = self._graph if self.steps_per_graph == 1 else \
                    _TorchGraph(_capture(steps(1), tr.device))
        elif mode == "graph-comm":
            self._graph = self._warm = _TorchGraph(_capture(lambda: tr.train_step(), tr.device))
            self.steps_per_graph = 1
        else:
            inv = 1.0 / self.world
            self._split = True
            self.steps_per_graph = 1
            if tr.fused_ok():
                # fused form: one piece up to the complete gradient (five launches), ONE all-reduce
                # of the whole flat gradient, the SGD launch
                self._fused = True
                pieces = (lambda: tr.forward_backward_fused(stage_adv=1),
                          lambda: tr.optimizer_step(grad_scale=inv))
            else:
                pieces = (lambda: tr.forward_backward_fc(), lambda: tr.backward_conv(),
                          lambda: tr.optimizer_step(grad_scale=inv))
            if native and launch == "stream":
                # the three pieces launch only this library's kernels: record them natively
                # and launch their kernel lists straight onto the stream (no ~8.6 us
                # hipGraphLaunch gap per piece, three per step); profiles/r3_split_launch_ab.md
                gs = [NativeGraph(f, tr.device) for f in pieces]
                if all(g.stream_ok for g in gs):
                    self.launch = "stream"
                    self._gs = gs
            if self.launch != "stream":
                self._gs = [_TorchGraph(_capture(f, tr.device)) for f in pieces]
        torch.cuda.synchronize(tr.device)

    def _split_steps(self, n: int) -> None:
        tr = self.tr
        sync = tr.grad_sync
        go = (lambda g: g.replay_stream(1)) if self.launch == "stream" else (lambda g: g.replay(1))
        if self._fused:
            g1, g3 = self._gs
            for _ in range(n):
                go(g1)
                sync.all_ready(tr.flat_grads)
                sync.finish()
                go(g3)
            return
        g1, g2, g3 = self._gs
        for _ in range(n):
            go(g1)
            sync.fc_ready(tr.fc_bucket())
            go(g2)
            sync.conv_ready(tr.conv_bucket())
            sync.finish()
            go(g3)

    def warm(self, n_steps: int) -> None:
        """``n_steps`` untimed steps of any count: whole replays of the timed graph first (a
        hipGraph's first launch costs ~0.75 us per node more than later ones, even after
        hipGraphUpload -- profiles/r2_launch_overhead.json), then one-step replays."""
        tr = self.tr
        tr.grad_sync = self.sync
        if n_steps <= 0:
            return
        if self.mode == "eager":
            for _ in range(n_steps):
                tr.train_step()
        elif self._split:
            self._split_steps(n_steps)
        else:
            if self.launch == "stream":
                self._graph.replay_stream(n_steps)
                return
            full = n_steps // self.steps_per_graph
            if full:
                self._graph.replay(full)
            if n_steps - full * self.steps_per_graph:
                self._warm.replay(n_steps - full * self.steps_per_graph)

    def run(self, n_steps: int) -> None:
        """Execute ``n_steps`` training steps (a multiple of steps_per_graph in graph modes)."""
        tr = self.tr
        tr.grad_sync = self.sync
        if self.mode == "eager":
            for _ in range(n_steps):
                tr.train_step()
            return
        if self._split:
            self._split_steps(n_steps)
            return
        if self.launch == "stream":
            self._graph.replay_stream(n_steps)
            return
        if n_steps % self.steps_per_graph:
            raise ValueError("n_steps must be a multiple of steps_per_graph")
        self._graph.replay(n_steps // self.steps_per_graph)


class _TorchGraph:
    def __init__(self, g: torch.cuda.CUDAGraph):
        self.g = g

    def replay(self, n: int = 1) -> None:
        for _ in range(n):
            self.g.replay()
