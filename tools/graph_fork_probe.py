#!/usr/bin/env python3
"""Cost of a fork/join (two-stream) hipGraph vs the same kernels on one stream.

Kernel A (~13 us, stands in for conv_bwd) and kernel B (~5 us, stands in for a side-stream
exchange) are captured (1) back to back on one stream, (2) B on a side stream forked
after a short kernel P and joined before a short kernel Q.  Prints us per replay of 20
repetitions for both graphs.
"""
import time

import torch


def busy(t: torch.Tensor, n: int):
    for _ in range(n):
        t.mul_(1.0000001).add_(1e-7)


def main():
    dev = torch.device("cuda")
    a = torch.randn(1 << 22, device=dev)
    b = torch.randn(1 << 20, device=dev)
    p = torch.randn(1 << 10, device=dev)
    side = torch.cuda.Stream()
    reps = 20

    def serial():
        for _ in range(reps):
            p.add_(1)
            busy(a, 4)
            busy(b, 4)
            p.add_(1)

    def forked():
        for _ in range(reps):
            p.add_(1)
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                busy(b, 4)
            busy(a, 4)
            torch.cuda.current_stream().wait_stream(side)
            p.add_(1)

    res = {}
    for name, fn in (("serial", serial), ("forked", forked)):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            fn()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        with torch.cuda.graph(g):
            fn()
        best = 1e9
        for _ in range(10):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            g.replay()
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        res[name] = round(best / reps * 1e6, 2)
    # components alone
    for name, fn in (("a_only", lambda: busy(a, 4)), ("b_only", lambda: busy(b, 4))):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(reps):
                fn()
        best = 1e9
        for _ in range(10):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            g.replay()
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        res[name] = round(best / reps * 1e6, 2)
    print(res)


if __name__ == "__main__":
    main()
