#!/usr/bin/env python3
"""Tail of the bench's K=20 timed region: N back-to-back regions (synchronize, 20 stream-launched
steps, synchronize) in one process, as a distribution -- to find where a rare 250-300 us stall
of the region comes from (the driver records ONE K=20 run).  One JSON line: median / p90 / p99 /
max in us per step and how many regions ran over 1.1 x the median.

    python tools/dbg/k20_tail.py [--regions 300] [--steps 20]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--regions", type=int, default=300)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    import torch
    from bench import prewarm
    from pytorch_operator_amd.data.synthetic import make_synthetic_mnist
    from pytorch_operator_amd.models.mnist import FusedMnistTrainer
    from pytorch_operator_amd.ops import mnist as K
    from pytorch_operator_amd.parallel.graphed_step import GraphedStep

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    ds = make_synthetic_mnist(60000, seed=1, device=dev)
    cursor = torch.zeros(1, dtype=torch.int32, device=dev)
    src = K.BatchSource(ds.images, ds.labels, perm=ds.perm, cursor=cursor)
    tr = FusedMnistTrainer(batch_size=64, source=src, lr=0.01, momentum=0.5, device=dev, seed=1)
    runner = GraphedStep(tr, mode="graph", steps_per_graph=1, launch="stream")
    prewarm(40, dev)
    runner.warm(50)
    ts = []
    for _ in range(a.regions):
        runner.warm(5)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        runner.run(a.steps)
        torch.cuda.synchronize(dev)
        ts.append((time.perf_counter() - t0) / a.steps * 1e6)
    s = sorted(ts)
    med = statistics.median(s)
    q = lambda p: round(s[min(len(s) - 1, int(p * len(s)))], 3)  # noqa: E731
    env = {k: os.environ[k] for k in ("HSA_KERNARG_POOL_SIZE", "HIP_FORCE_DEV_KERNARG", "ROC_USE_FGS_KERNARG")
           if k in os.environ}
    print(json.dumps({"regions": a.regions, "steps": a.steps, "median": round(med, 3), "p90": q(0.9), "p99": q(0.99),
                      "max": round(s[-1], 3), "over_1.1x": sum(1 for t in s if t > 1.1 * med), "env": env}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
