#!/usr/bin/env python3
"""Fixed cost around a timed region of K graph-replayed MNIST steps on one MI355X.

For K in (1, 5, 20, 100, 200) it times ``launch(K-step graph) + synchronize`` (median of
reps) and reports the per-step slope and the fixed intercept, plus the round trip of an
idle ``torch.cuda.synchronize()``.  Run it under different runtime wait settings (e.g.
``ROC_ACTIVE_WAIT_TIMEOUT``) to see what the host-side completion wait costs.
"""
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
    out = {"env": {k: v for k, v in os.environ.items() if k.startswith(("ROC_", "HIP_", "GPU_"))}}
    idle = []
    for _ in range(50):
        t0 = time.perf_counter()
        torch.cuda.synchronize(dev)
        idle.append((time.perf_counter() - t0) * 1e6)
    out["idle_sync_us"] = round(statistics.median(idle), 2)
    res = {}
    for k in (1, 5, 20, 100, 200):
        r = GraphedStep(tr, mode="graph", steps_per_graph=k, native=os.environ.get("PTO_PROBE_TORCH_GRAPH") != "1")
        r.warm(5)
        ts = []
        for _ in range(15):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            r.run(k)
            torch.cuda.synchronize(dev)
            ts.append((time.perf_counter() - t0) * 1e6)
        first = ts[0]
        res[k] = {"median_us": round(statistics.median(ts[1:]), 1), "first_us": round(first, 1),
                  "per_step_us": round(statistics.median(ts[1:]) / k, 2)}
    out["graphs"] = res
    # K=20 timed as back-to-back launches of smaller, already replayed graphs
    multi = {}
    for k in (1, 2, 4, 5, 10):
        r = GraphedStep(tr, mode="graph", steps_per_graph=k, native=os.environ.get("PTO_PROBE_TORCH_GRAPH") != "1")
        r.run(k)
        ts = []
        for _ in range(15):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            r.run(20)
            torch.cuda.synchronize(dev)
            ts.append((time.perf_counter() - t0) * 1e6)
        multi[f"{20 // k}x{k}"] = round(statistics.median(ts), 1)
    out["k20_as_launches"] = multi
    slope = (res[200]["median_us"] - res[20]["median_us"]) / 180
    out["slope_us_per_step"] = round(slope, 3)
    out["intercept_us"] = round(res[20]["median_us"] - 20 * slope, 1)
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
