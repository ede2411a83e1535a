#!/usr/bin/env python3
"""Latency anatomy of the xGMI push all-reduce, emulated on one GPU (grid.y = rank).

For each buffer allocation kind and world size: us per fused launch (graph of 50
back-to-back launches) and, for one stamped launch, the mean/max per-block phase times
(produce+push | wait flags1 + reduce/SGD + push | wait flags2 + gather) and the span.
XAR_SLAB=chunk (default): the conv2.weight slab columns hold conv_bwd4's ceil(B/4) chunk rows
(the round-3 step); XAR_SLAB=sample: B per-sample rows everywhere (round 1-2).
Prints one JSON line per configuration.
"""
from __future__ import annotations

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    import torch
    from pytorch_operator_amd.models.mnist import flat_layout
    from pytorch_operator_amd.parallel.xgmi import XgmiEmulation

    dev = torch.device("cuda", 0)
    L, ce, B = flat_layout().total, flat_layout().conv_end, 64
    kinds = [int(k) for k in os.environ.get("XAR_KINDS", "0,1,2").split(",")]
    worlds = [int(w) for w in os.environ.get("XAR_WORLDS", "2,8").split(",")]
    nblks = [int(b) for b in os.environ.get("XAR_NBLK", "128").split(",")]
    fences = [int(f) for f in os.environ.get("XAR_FENCE", "-1").split(",")]
    slab_modes = os.environ.get("XAR_SLAB", "chunk").split(",")
    # XAR_PUSH=1: fc1_bwd pushes dW_fc1 itself (round 4; emulated by a prepush launch, timed apart)
    pushes = [int(x) for x in os.environ.get("XAR_PUSH", "0,1").split(",")]
    w1o = flat_layout().offsets["fc1.weight"]
    lo = flat_layout().offsets["conv2.weight"]
    for kind, fence, sm, push in [(k, f, m, q) for k in kinds for f in fences for m in slab_modes for q in pushes]:
        for world in worlds:
            for nblk in nblks:
                emu = XgmiEmulation(world, L, nblk=nblk, alloc_kind=kind, fence=fence)
                ps = [torch.zeros(L, device=dev) for _ in range(world)]
                ms = [torch.zeros(L, device=dev) for _ in range(world)]
                grads = [torch.randn(L, device=dev) for _ in range(world)]
                slabs = [torch.randn(B, ce, device=dev) for _ in range(world)]
                cfg = dict(slab=slabs, slab_rows=B, conv_n=ce, lr=0.0, momentum=0.5,
                           slab_big=((B + 3) // 4, lo, lo + 25000) if sm == "chunk" else None,
                           skip=(w1o, w1o + 400000) if push else None)
                emu.configure(1, grads, ps, ms, **cfg)
                if push:
                    emu.prepush()
                emu.launch()
                torch.cuda.synchronize()

                def timed(fn):
                    graph = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(graph):
                        for _ in range(50):
                            fn()
                    best = float("inf")
                    for _ in range(5):
                        torch.cuda.synchronize()
                        t0 = time.perf_counter()
                        graph.replay()
                        torch.cuda.synchronize()
                        best = min(best, time.perf_counter() - t0)
                    return best
                # the exchange alone (with push: after a prepush, which is what fc1_bwd did)
                best = timed((lambda: (emu.prepush(), emu.launch())) if push else emu.launch)
                pre = timed(emu.prepush) if push else 0.0
                best -= pre
                st = emu.enable_stamps()
                emu.configure(1, grads, ps, ms, **cfg)
                for _ in range(3):
                    if push:
                        emu.prepush()
                    emu.launch()
                torch.cuda.synchronize()
                s = st.view(world, nblk, 4).double().cpu() / 100.0  # us (100 MHz)
                t0 = s[..., 0].min()
                ph = s[..., 1:] - s[..., :-1]
                res = {"alloc_kind": kind, "fence": fence, "slab": sm, "push_fc1": push, "world": world,
                       "nblk": nblk, "threads": emu.threads,
                       "us_per_launch": round(best / 50 * 1e6, 2),
                       "prepush_us_per_launch": round(pre / 50 * 1e6, 2),
                       "span_us": round(float(s[..., 3].max() - t0), 2),
                       "start_skew_us": round(float(s[..., 0].max() - t0), 2),
                       "phase_mean_us": [round(float(x), 2) for x in ph.mean((0, 1))],
                       "phase_max_us": [round(float(x), 2) for x in ph.amax((0, 1))],
                       "error": emu.error()}
                print(json.dumps(res), flush=True)
                emu.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
