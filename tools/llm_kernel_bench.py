#!/usr/bin/env python3
"""Per-op timing of the Llama fused HIP kernels at the 8B B=4 S=2048 shapes (one MI355X).

Prints one JSON line per op: us per call and the achieved HBM bandwidth of its minimum
traffic (bytes every element must move once).  ``--rpb`` sweeps the RMSNorm backward's
rows-per-workgroup.
"""
import argparse
import json

import torch


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rpb", default="4,8,16,32")
    a = ap.parse_args()
    from pytorch_operator_amd.models.llama import rope_tables
    from pytorch_operator_amd.ops import llm, norm
    from pytorch_operator_amd.ops import _native
    lib = _native.load()
    dev = torch.device("cuda")
    T, D, F, H, HD = 4 * 2048, 4096, 14336, 32, 128
    x = torch.randn(T, D, device=dev)
    w = torch.ones(D, device=dev)
    y = torch.empty(T, D, device=dev, dtype=torch.bfloat16)
    rstd = torch.empty(T, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    us = timeit(lambda: lib.pto_rmsnorm_fwd(x.data_ptr(), w.data_ptr(), y.data_ptr(), rstd.data_ptr(), T, D,
                                            1e-5, 2, st))
    print(json.dumps({"op": "rmsnorm_fwd fp32->bf16", "shape": [T, D], "us": round(us, 1),
                      "GBps": round(T * D * 6 / us / 1e3, 1)}))
    dy = torch.randn(T, D, device=dev).bfloat16()
    dx = torch.empty_like(x)
    dw = torch.empty(D, device=dev)
    for rpb in [int(v) for v in a.rpb.split(",")]:
        parts = torch.empty((T + rpb - 1) // rpb, D, device=dev)
        us = timeit(lambda: lib.pto_rmsnorm_bwd(dy.data_ptr(), x.data_ptr(), w.data_ptr(), rstd.data_ptr(),
                                                dx.data_ptr(), dw.data_ptr(), parts.data_ptr(), T, D, rpb, 2, st))
        print(json.dumps({"op": "rmsnorm_bwd bf16 dy, fp32 x/dx (+colsum)", "rows_per_block": rpb, "us": round(us, 1),
                          "GBps": round(T * D * 10 / us / 1e3, 1)}))
    q = torch.randn(4, 2048, H, HD, device=dev).bfloat16()
    cos, sin = rope_tables(HD, 2048, 500000.0, dev)
    us = timeit(lambda: llm._rope_launch(q, cos, sin, 1.0))
    print(json.dumps({"op": "rope bf16 (q)", "shape": list(q.shape), "us": round(us, 1),
                      "GBps": round(q.numel() * 4 / us / 1e3, 1)}))
    a1 = torch.randn(T, F, device=dev).bfloat16()
    b1 = torch.randn(T, F, device=dev).bfloat16()
    o = torch.empty_like(a1)
    o2 = torch.empty_like(a1)
    n = a1.numel()
    us = timeit(lambda: lib.pto_swiglu_fwd(a1.data_ptr(), b1.data_ptr(), o.data_ptr(), n, 1, st))
    print(json.dumps({"op": "swiglu_fwd bf16", "n": n, "us": round(us, 1), "GBps": round(n * 6 / us / 1e3, 1)}))
    us = timeit(lambda: lib.pto_swiglu_bwd(o.data_ptr(), a1.data_ptr(), b1.data_ptr(), o2.data_ptr(), o.data_ptr(),
                                           n, 1, st))
    print(json.dumps({"op": "swiglu_bwd bf16", "n": n, "us": round(us, 1), "GBps": round(n * 10 / us / 1e3, 1)}))
    big = torch.empty(1 << 28, device=dev)  # 1 GiB copy: the achievable-bandwidth yardstick
    big2 = torch.empty_like(big)
    us = timeit(lambda: big2.copy_(big))
    print(json.dumps({"op": "torch copy_ fp32 1 GiB (yardstick)", "us": round(us, 1),
                      "GBps": round(big.numel() * 8 / us / 1e3, 1)}))


if __name__ == "__main__":
    main()
