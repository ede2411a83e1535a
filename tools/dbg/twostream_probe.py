#!/usr/bin/env python3
"""Price of a two-stream step structure (pto_graph_launch_stream_probe), no work moved.

The world-1 step's five kernels replay on the main stream; variants add, per step, an event record
after kernel ``rec`` (0 conv12_fwd, 1 fc1_fwd, 2 fc1_bwd_head, 3 conv_bwd4, 4 tail), a side stream
that waits for it, runs a no-op kernel and records a second event, and a wait of the main stream
for that second event before kernel ``wait`` of the next step.  Interleaved, K steps each, MAX of
nothing (one process): us per step.  Decides whether moving the tail's fc work onto a side stream
can pay for its synchronisation.

    python tools/dbg/twostream_probe.py [--steps 2000] [--reps 5]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

VARIANTS = {  # name: (rec_after, wait_before, side_blocks)
    "plain": (-1, -1, 0),
    "rec3_only": (3, -1, 0),
    "rec3_side_wait1": (3, 1, 256),
    "rec2_side_wait1": (2, 1, 256),
    "rec3_noside_wait1": (3, 1, 0),
}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch
    from bench import prewarm
    from pytorch_operator_amd.data.synthetic import make_synthetic_mnist
    from pytorch_operator_amd.models.mnist import FusedMnistTrainer
    from pytorch_operator_amd.ops import _native
    from pytorch_operator_amd.ops import mnist as K
    from pytorch_operator_amd.parallel.graphed_step import GraphedStep

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    ds = make_synthetic_mnist(60000, seed=1, device=dev)
    cursor = torch.zeros(1, dtype=torch.int32, device=dev)
    src = K.BatchSource(ds.images, ds.labels, perm=ds.perm, cursor=cursor)
    tr = FusedMnistTrainer(batch_size=64, source=src, lr=0.01, momentum=0.5, device=dev, seed=1)
    runner = GraphedStep(tr, mode="graph", steps_per_graph=1, launch="stream")
    g = runner._graph
    lib = _native.load()
    side = torch.cuda.Stream(device=dev)
    main_s = torch.cuda.current_stream(dev)
    prewarm(40, dev)

    def run(name, n):
        rec, wait, blocks = VARIANTS[name]
        _native.check(lib.pto_graph_launch_stream_probe(g._h, main_s.cuda_stream, side.cuda_stream, n, rec, wait,
                                                        blocks), "probe")

    for name in VARIANTS:
        run(name, 50)
    torch.cuda.synchronize(dev)
    res = {k: [] for k in VARIANTS}
    for _ in range(a.reps):
        for name in VARIANTS:
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            run(name, a.steps)
            torch.cuda.synchronize(dev)
            res[name].append((time.perf_counter() - t0) / a.steps * 1e6)
    out = {k: {"median_us": round(statistics.median(v), 3), "min_us": round(min(v), 3)} for k, v in res.items()}
    print(json.dumps({"steps": a.steps, "reps": a.reps, "us_per_step": out}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
