#!/usr/bin/env python3
"""Fixed vs per-step cost of bench.py's timed region: t(K) = a + b K.

Builds the bench's world-1 runner (stream-launched one-step kernel list) and times K steps
bracketed by ``torch.cuda.synchronize()`` exactly as bench.py does, for several K, several
repeats each, interleaved.  Also times the floor of the bracket itself: an idle synchronize, and
one empty kernel launch + synchronize.  Prints one JSON line.

    python tools/dbg/k_sweep.py [--ks 1,2,5,10,20,50,200,2000] [--reps 7]
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
    ap.add_argument("--ks", default="1,2,5,10,20,50,200,2000")
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--prewarm-ms", type=int, default=40)
    ap.add_argument("--brackets", default="double,single,event",
                    help="end-of-region waits compared at K=20: double (bench.py at world 1), single, event")
    ap.add_argument("--spin", action="store_true", help="hipSetDeviceFlags(hipDeviceScheduleSpin) first")
    a = ap.parse_args()
    import torch
    if a.spin:
        import ctypes
        hip = [ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln][0]
        rc = ctypes.CDLL(hip).hipSetDeviceFlags(1)
        print(f"hipSetDeviceFlags(spin) rc={rc} ({hip})", file=sys.stderr)
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
    prewarm(a.prewarm_ms, dev)
    runner.warm(50)
    torch.cuda.synchronize(dev)

    ev = torch.cuda.Event()

    def bracket_end(kind):
        if kind == "event":  # wait on the stream's last kernel, then the device
            ev.record()
            ev.synchronize()
        torch.cuda.synchronize(dev)
        if kind == "double":
            torch.cuda.synchronize(dev)

    def timed(fn, kind="double"):
        torch.cuda.synchronize(dev)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        fn()
        bracket_end(kind)
        return time.perf_counter() - t0

    ks = [int(x) for x in a.ks.split(",")]
    res = {k: [] for k in ks}
    sink = torch.zeros(1, device=dev)
    floor_idle, floor_one = [], []
    kinds = a.brackets.split(",")
    by_kind = {kd: [] for kd in kinds}
    for _ in range(a.reps):
        for k in ks:
            runner.warm(5)
            res[k].append(timed(lambda: runner.run(k)))
        kinds = kinds[1:] + kinds[:1]  # rotated each rep: no wait kind always follows the K=2000 run
        for kd in kinds:  # K = 20 under each end-of-region wait
            runner.warm(5)
            by_kind[kd].append(timed(lambda: runner.run(20), kd))
        floor_idle.append(timed(lambda: None))
        floor_one.append(timed(lambda: sink.add_(1.0)))
    med = {k: statistics.median(v) for k, v in res.items()}
    mn = {k: min(v) for k, v in res.items()}
    # least squares on the medians
    xs, ys = ks, [med[k] for k in ks]
    xb, yb = sum(xs) / len(xs), sum(ys) / len(ys)
    b = sum((x - xb) * (y - yb) for x, y in zip(xs, ys)) / sum((x - xb) ** 2 for x in xs)
    out = {
        "us_per_step_median": {k: round(med[k] / k * 1e6, 3) for k in ks},
        "us_per_step_min": {k: round(mn[k] / k * 1e6, 3) for k in ks},
        "fit_us": {"fixed": round((yb - b * xb) * 1e6, 2), "per_step": round(b * 1e6, 3)},
        "floor_idle_sync_us": round(statistics.median(floor_idle) * 1e6, 2),
        "floor_one_kernel_us": round(statistics.median(floor_one) * 1e6, 2),
        "k20_us_per_step_by_bracket": {kd: round(statistics.median(v) / 20 * 1e6, 3) for kd, v in by_kind.items()},
        "reps": a.reps, "spin": a.spin,
        "env": {k: os.environ[k] for k in ("ROC_ACTIVE_WAIT_TIMEOUT", "ROC_CPU_WAIT_FOR_SIGNAL") if k in os.environ},
    }
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
