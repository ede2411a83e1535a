#!/usr/bin/env python3
"""Stress the xGMI exchange against dist.all_reduce: W ranks (torchrun, gloo) run
``XgmiAllReduce.self_test`` for --steps steps (each: one mean all-reduce and one fused SGD
exchange, checked to 1e-5).  One JSON line per rank: failing steps, the error word, the buffer's
allocation kind and the fence flavour (PTO_XAR_FENCE).

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 tools/dbg/xar_stress.py --steps 200
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--n", type=int, default=431080)
    ap.add_argument("--discriminate", action="store_true",
                    help="check the exchange and gloo's GPU-tensor all_reduce separately against a host float64 mean")
    a = ap.parse_args()
    import torch
    import torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", 0)) % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pytorch_operator_amd.parallel.xgmi import XgmiAllReduce
    n = a.n - a.n % 4
    xar = XgmiAllReduce(n, device=dev, timeout_s=float(os.environ.get("PTO_XGMI_TIMEOUT_S", "20")))
    t0 = time.perf_counter()
    if a.discriminate:
        # per step: the exchange's mean and gloo's all_reduce of the GPU tensor, each against the
        # float64 mean of every rank's input gathered on the host (CPU tensors through gloo)
        g = torch.Generator(device="cpu").manual_seed(1234 + rank)
        rep = []
        for i in range(a.steps):
            xc = torch.randn(n, generator=g)
            x = xc.to(dev)
            xs = [torch.empty(n) for _ in range(world)]
            dist.all_gather(xs, xc)
            truth = torch.stack(xs).double().mean(0).float()
            ref = x.clone()
            dist.all_reduce(ref)
            ref /= world
            out = torch.empty_like(x)
            xar.allreduce_mean(x, out)
            torch.cuda.synchronize(dev)
            e_x = float((out.cpu() - truth).abs().max())
            e_ref = float((ref.cpu() - truth).abs().max())
            if e_x > 1e-5 or e_ref > 1e-5:
                rep.append({"step": i, "xgmi_err": e_x, "gloo_err": e_ref})
        ok = not rep
    else:
        ok = xar.self_test(steps=a.steps)
        rep = xar.last_report
    print(json.dumps({"rank": rank, "world": world, "ok": ok, "failed_steps": [r.get("step") for r in rep][:40],
                      "first": rep[:2], "error": xar.error(), "alloc_kind": xar.alloc_kind,
                      "fence": os.environ.get("PTO_XAR_FENCE", "default"), "prebarrier": xar.prebarrier,
                      "nblk": xar.nblk, "seconds": round(time.perf_counter() - t0, 2)}), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
