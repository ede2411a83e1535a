#!/usr/bin/env python3
"""Does a K=20 / W=5 timed region pay a cold-GPU penalty?  After an idle gap, replay the
warm-up (5 steps) and time 20 steps; compare with the same after ``prewarm_ms`` of
unrelated GPU work (clock ramp) and with a steady-state run."""
from __future__ import annotations

import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    import torch
    from pytorch_operator_amd.data.synthetic import make_synthetic_mnist
    from pytorch_operator_amd.models.mnist import FusedMnistTrainer
    from pytorch_operator_amd.ops import mnist as K
    from pytorch_operator_amd.parallel.graphed_step import GraphedStep

    dev = torch.device("cuda", 0)
    ds = make_synthetic_mnist(60000, seed=1, device=dev)
    cursor = torch.zeros(1, dtype=torch.int32, device=dev)
    src = K.BatchSource(ds.images, ds.labels, perm=ds.perm, cursor=cursor)
    tr = FusedMnistTrainer(batch_size=64, source=src, device=dev, seed=1)
    r = GraphedStep(tr, mode="graph", steps_per_graph=5)
    a = torch.randn(4096, 4096, device=dev)

    def timed():
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        r.run(20)
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) * 1e6

    out = {}
    for idle_s in (0.0, 0.05, 0.3, 1.0):
        for pre_ms in (0, 5, 30):
            ts = []
            for _ in range(5):
                time.sleep(idle_s)
                if pre_ms:
                    t0 = time.perf_counter()
                    while (time.perf_counter() - t0) * 1e3 < pre_ms:
                        a = a @ a
                        a = a / a.norm()
                        torch.cuda.synchronize(dev)
                r.warm(5)
                ts.append(timed())
            out[f"idle{idle_s}_pre{pre_ms}"] = round(statistics.median(ts), 1)
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
