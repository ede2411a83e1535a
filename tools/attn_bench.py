#!/usr/bin/env python3
"""Attention kernel timing at Llama-3 8B shapes: HIP flash attention vs the library SDPA.

usage: python tools/attn_bench.py [--batch 4] [--seq 2048] [--hq 32] [--hkv 8] [--reps 20] [--json-out F]

Times forward alone and forward+backward (CUDA events, median of reps); FLOPs count the
causal half: fwd 2 products, bwd 5 products (the HIP backward does 7: see attention.hip).
"""
import argparse
import json
import math
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import torch  # noqa: E402


def timed(fn, reps):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return statistics.median(ts)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=4)
    p.add_argument("--seq", type=int, default=2048)
    p.add_argument("--hq", type=int, default=32)
    p.add_argument("--hkv", type=int, default=8)
    p.add_argument("--reps", type=int, default=20)
    p.add_argument("--causal", type=int, default=1)
    p.add_argument("--impl", default="hip,sdpa")
    p.add_argument("--json-out", default=None)
    a = p.parse_args()
    from pytorch_operator_amd.ops.attention import flash_attention, sdpa_bshd
    B, S, Hq, Hkv, D = a.batch, a.seq, a.hq, a.hkv, 128
    g = torch.Generator(device="cuda").manual_seed(0)
    q = torch.randn(B, S, Hq, D, device="cuda", generator=g).to(torch.bfloat16).requires_grad_(True)
    k = torch.randn(B, S, Hkv, D, device="cuda", generator=g).to(torch.bfloat16).requires_grad_(True)
    v = torch.randn(B, S, Hkv, D, device="cuda", generator=g).to(torch.bfloat16).requires_grad_(True)
    do = torch.randn(B, S, Hq, D, device="cuda", generator=g).to(torch.bfloat16)
    frac = 0.5 if a.causal else 1.0
    fwd_flop = 4 * B * Hq * S * S * D * frac
    res = {"shape": {"B": B, "S": S, "Hq": Hq, "Hkv": Hkv, "D": D, "causal": bool(a.causal)}}
    for name, fn in (("hip", flash_attention), ("sdpa", sdpa_bshd)):
        if name not in a.impl.split(","):
            continue
        with torch.no_grad():
            fn(q, k, v, bool(a.causal))
            t_f = timed(lambda: fn(q, k, v, bool(a.causal)), a.reps)

        def fb():
            o = fn(q, k, v, bool(a.causal))
            o.backward(do)
        fb()
        t_fb = timed(fb, a.reps)
        t_b = t_fb - t_f
        res[name] = {"fwd_us": round(t_f, 1), "fwd_bwd_us": round(t_fb, 1), "bwd_us": round(t_b, 1),
                     "fwd_tflops": round(fwd_flop / t_f / 1e6, 1),
                     "bwd_tflops": round(2.5 * fwd_flop / t_b / 1e6, 1)}
        print(name, res[name], flush=True)
        q.grad = k.grad = v.grad = None
    if "hip" in res and "sdpa" in res:
        res["speedup_fwd_bwd"] = round(res["sdpa"]["fwd_bwd_us"] / res["hip"]["fwd_bwd_us"], 2)
    print(json.dumps(res))
    if a.json_out:
        Path(a.json_out).write_text(json.dumps(res, indent=1) + "\n")


if __name__ == "__main__":
    main()
