#!/usr/bin/env python3
"""Per-shape bandwidth of the fused NHWC batch-norm kernels (csrc/kernels/batchnorm.hip) at the
ResNet-50 B=256 layer shapes: forward (statistics + normalise[+add][+ReLU]) and backward
(reductions + dx[+dz]) timed with HIP events, effective TB/s from the minimum bytes each pass
must move (bf16 elements: fwd 3E [+E residual], bwd 5E [+2E saved y, +E dz]).

    python tools/bn_bench.py [--batch 256] [--iters 20] [--json out.json]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_operator_amd.ops.batchnorm import batch_norm_act  # noqa: E402

# (H, C, relu, residual, count per ResNet-50 forward) -- torchvision v1.5 bottlenecks
SHAPES = [
    (112, 64, True, False, 1),                          # stem
    (56, 64, True, False, 6), (56, 256, True, True, 3), (56, 256, False, False, 1),
    (56, 128, True, False, 1), (28, 128, True, False, 7), (28, 512, True, True, 4), (28, 512, False, False, 1),
    (28, 256, True, False, 1), (14, 256, True, False, 11), (14, 1024, True, True, 6), (14, 1024, False, False, 1),
    (14, 512, True, False, 1), (7, 512, True, False, 5), (7, 2048, True, True, 3), (7, 2048, False, False, 1),
]


def timed(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    rows, tot_f, tot_b = [], 0.0, 0.0
    for H, C, relu, res, cnt in SHAPES:
        shp = (a.batch, C, H, H)
        x = torch.randn(shp, device=dev, dtype=torch.bfloat16).to(memory_format=torch.channels_last)
        x.requires_grad_(True)
        z = torch.randn_like(x).requires_grad_(True) if res else None
        w = torch.rand(C, device=dev) + 0.5
        b = torch.randn(C, device=dev)
        w.requires_grad_(True)
        b.requires_grad_(True)
        dy = torch.randn_like(x)

        def fwd():
            with torch.no_grad():
                batch_norm_act(x, w, b, relu=relu, residual=z)

        def fwdbwd():
            for t in (x, z, w, b):
                if t is not None:
                    t.grad = None
            y = batch_norm_act(x, w, b, relu=relu, residual=z)
            y.backward(dy)

        tf = timed(fwd, a.iters)
        tfb = timed(fwdbwd, a.iters)
        tb = max(tfb - tf, 1e-3)
        E = x.numel() * 2
        bf = E * (3 + (1 if res else 0))
        bb = E * (5 + (2 if (relu and res) else 0) + (1 if res else 0))
        r = {"H": H, "C": C, "relu": relu, "res": res, "count": cnt, "MB": round(E / 2 ** 20, 1),
             "fwd_us": round(tf, 1), "bwd_us": round(tb, 1),
             "fwd_TBps": round(bf / tf / 1e6, 2), "bwd_TBps": round(bb / tb / 1e6, 2)}
        rows.append(r)
        tot_f += tf * cnt
        tot_b += tb * cnt
        print(json.dumps(r), flush=True)
        del x, z, dy
    summ = {"batch": a.batch, "fwd_ms_per_step": round(tot_f / 1e3, 2), "bwd_ms_per_step": round(tot_b / 1e3, 2)}
    print(json.dumps(summ), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"rows": rows, "summary": summ}, f, indent=1)


if __name__ == "__main__":
    main()
