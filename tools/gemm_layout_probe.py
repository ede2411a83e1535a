#!/usr/bin/env python3
"""Which GEMM operand layouts run fastest on MI355X hipBLASLt for the Llama-3 8B step shapes?

For every linear of a block (T = 8192 tokens) times the forward GEMM (x.W^T, both operands
K-contiguous), the input-gradient GEMM as autograd issues it (dy.W, W K-strided) and in the
K-contiguous form (dy.(W^T)^T with a transposed weight copy), the weight-gradient GEMM as
autograd issues it (dy^T.x, both K-strided) and in the K-contiguous form (dy^T and x^T
materialised), plus the transpose copies themselves.  TunableOp tunes every shape first so
each layout is compared at its best hipBLASLt solution.  Prints one JSON line per linear.
"""
import json
import sys
import time

import torch
import torch.nn.functional as F


def bench(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / it * 1e3


def main():
    import torch.cuda.tunable as tunable
    tune = "--no-tune" not in sys.argv
    if tune:
        tunable.enable(True)
        tunable.tuning_enable(True)
        tunable.set_max_tuning_duration(10)
        tunable.set_max_tuning_iterations(10)
    T = 8192
    shapes = {"qkv": (4096, 6144), "wo": (4096, 4096), "w13": (4096, 28672), "w2": (14336, 4096)}
    dev = torch.device("cuda")
    for name, (fin, fout) in shapes.items():
        x = torch.randn(T, fin, device=dev, dtype=torch.bfloat16)
        w = torch.randn(fout, fin, device=dev, dtype=torch.bfloat16) * 0.02
        dy = torch.randn(T, fout, device=dev, dtype=torch.bfloat16)
        wt, dyt, xt = w.t().contiguous(), dy.t().contiguous(), x.t().contiguous()
        r = {"linear": name, "in": fin, "out": fout,
             "fwd_tn_ms": bench(lambda: F.linear(x, w)),
             "dgrad_autograd_ms": bench(lambda: dy @ w),
             "dgrad_tn_ms": bench(lambda: F.linear(dy, wt)),
             "wgrad_autograd_ms": bench(lambda: dy.t() @ x),
             "wgrad_tn_ms": bench(lambda: F.linear(dyt, xt)),
             "transpose_w_ms": bench(lambda: w.t().contiguous()),
             "transpose_dy_ms": bench(lambda: dy.t().contiguous()),
             "transpose_x_ms": bench(lambda: x.t().contiguous())}
        fl = 2 * T * fin * fout / 1e12
        for k in list(r):
            if k.endswith("_ms") and not k.startswith("transpose"):
                r[k.replace("_ms", "_pflops")] = round(fl / r[k], 2)
        r = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()}
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
