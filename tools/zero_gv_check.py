#!/usr/bin/env python3
"""ZeRO-1 gradient-as-bucket-view (``grad_view``) at world > 1 against the copy path.

Run under ``torch.distributed.run`` (any world size; ranks may share one GPU with gloo):
every rank builds the same Llama (tiny config), steps it with ``ZeroAdamW(reduce_dtype=bf16,
grad_view=True)`` and, from the same initial state, with ``grad_view=False``, on rank-dependent
batches.  With grad_view the bf16 buckets hold the unscaled gradient sum and AdamW applies 1/W;
the copy path scales each deposit by 1/W before the sum.  For a power-of-two W both are exact,
so the gathered fp32 masters must be bit-identical.  Each rank writes its result to
``<out>/rank<r>.json`` (concurrent ranks share one stdout pipe, where their lines can interleave, so
callers must read the files, not stdout); the process exits 0 when every rank agrees.

    python -m torch.distributed.run --nproc-per-node 2 tools/zero_gv_check.py --backend gloo --out DIR
"""
import argparse
import copy
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default="gloo")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--out", default=None, help="directory for rank<r>.json result files")
    a = ap.parse_args(argv)
    from pytorch_operator_amd.models.llama import CONFIGS, Llama
    from pytorch_operator_amd.ops.optim import to_bf16_matmul_weights
    from pytorch_operator_amd.parallel.zero import ZeroAdamW
    dist.init_process_group(a.backend)
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    torch.manual_seed(0)
    with torch.device(dev):
        base = Llama(CONFIGS["llama-tiny"])
    models, opts = [], []
    for gv in (True, False):
        m = copy.deepcopy(base)
        to_bf16_matmul_weights(m)
        o = ZeroAdamW(m, lr=1e-3, betas=(0.9, 0.95), weight_decay=0.1, bucket_mb=0.05,
                      reduce_dtype=torch.bfloat16, grad_view=gv)
        models.append(m)
        opts.append(o)
    g = torch.Generator().manual_seed(100 + rank)
    for _ in range(a.steps):
        x = torch.randint(0, 256, (2, 65), generator=g).to(dev)
        for m, o in zip(models, opts):
            o.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = m(x[:, :-1], x[:, 1:])
            loss.backward()
            o.step()
    for o in opts:
        o.synchronize()
    torch.cuda.synchronize(dev)
    d_view, d_copy = opts[0].full_masters_digest(), opts[1].full_masters_digest()
    weights_equal = all(torch.equal(p, q) for p, q in zip(models[0].parameters(), models[1].parameters()))
    res = {"rank": rank, "world": world, "sinks": opts[0].sinks,
           "unscaled_buckets": sum(b.unscaled for b in opts[0].buckets),
           "masters_equal": d_view == d_copy, "weights_equal": weights_equal, "digest": d_view}
    if a.out:
        os.makedirs(a.out, exist_ok=True)
        with open(os.path.join(a.out, f"rank{rank}.json"), "w") as f:
            json.dump(res, f)
    if rank == 0:
        print(json.dumps(res), flush=True)
    ok = torch.tensor([1 if (res["masters_equal"] and weights_equal and res["sinks"] > 0) else 0], dtype=torch.int32)
    if a.backend == "nccl":
        ok = ok.to(dev)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    dist.destroy_process_group()
    return 0 if int(ok.item()) == 1 else 1


if __name__ == "__main__":
    sys.exit(main())
