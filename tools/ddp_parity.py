#!/usr/bin/env python3
"""Multi-rank HIP trainer against torch's own DistributedDataParallel, step for step.

    torchrun --nproc-per-node 2 --master-addr 127.0.0.1 tools/ddp_parity.py [--steps 12]

Every rank builds three replicas of the reference MNIST job on the same per-rank batches:

* ``torch``: ``DistributedDataParallel(Net())`` + ``torch.optim.SGD(lr=0.01, momentum=0.5)`` in
  fp32 on the CPU -- the reference's wrapper and optimiser (examples/mnist/mnist.py:135-140),
  whose constructor broadcasts rank 0's parameters.  The net is ``DecisionAlignedNet``: its two
  max-pool argmaxes and three ReLU masks are the ones the HIP step took on that batch (a window
  whose top two values, or a ReLU input within fp32 rounding of 0, has no stable decision, and a
  flipped one sends a different trajectory); ``decision_gap`` proves every given decision is
  torch's own up to rounding, and ``param_rel_torch_own_decisions`` reports the unaligned
  comparison as well;
* ``rccl``: ``FusedMnistTrainer`` + ``FlatGradAllReduce`` (two bucket all-reduces), run by the
  bench's runner (``GraphedStep(launch="stream")``);
* ``xgmi``: ``FusedMnistTrainer`` + ``XgmiGradSync`` (the peer-memory exchange fused with SGD).

Each rank initialises its own weights from a different seed, so only the start-up broadcast
makes the replicas agree.  On a 1-GPU box the ranks share GPU 0 (gloo process group).  Rank 0
prints one JSON line: the worst relative parameter / momentum error of each HIP replica against
torch over all ranks (max |a - b| / max |b|).  Exit 0 iff all are within ``--tol``.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _rel(a, b) -> float:
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def _run_path(entry, upto: int, B: int, dev) -> None:
    """Step one replica to ``upto`` steps, one ``run(1)`` at a time (the same recorded kernels as the
    bench's run(n)), keeping each step's decisions (pool argmax codes, ReLU masks) for the torch side."""
    import torch
    tr, runner, codes = entry

    def keep():
        torch.cuda.synchronize(dev)
        codes.append((tr.idx1[:B].cpu(), tr.idx2[:B].cpu(), (tr.a1[:B] > 0).cpu(), (tr.a2[:B] > 0).cpu(),
                      (tr.h1[:B] > 0).cpu()))
    if not codes and runner.internal_steps:
        keep()
    while len(codes) < upto:
        runner.run(1)
        keep()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default="gloo")
    ap.add_argument("--steps", type=int, default=12, help="HIP steps before the comparison (>= 10)")
    ap.add_argument("--dataset", type=int, default=2048)
    ap.add_argument("--tol", type=float, default=1e-4)
    ap.add_argument("--paths", default="rccl,xgmi")
    ap.add_argument("--eager", action="store_true", help="eager train_step() calls instead of the bench's runner")
    ap.add_argument("--interleave", action="store_true", help="(with --eager) step the paths' trainers in turn")
    ap.add_argument("--gap-tol", type=float, default=1e-5,
                    help="largest distance of torch's own numbers from a HIP decision (relative)")
    a = ap.parse_args(argv)
    import torch
    import torch.distributed as dist
    import torch.nn.functional as F
    from pytorch_operator_amd.data.synthetic import make_synthetic_mnist
    from pytorch_operator_amd.models.mnist import DecisionAlignedNet, FusedMnistTrainer, _views, flat_layout
    from pytorch_operator_amd.ops import mnist as K
    from pytorch_operator_amd.parallel.ddp import FlatGradAllReduce
    from pytorch_operator_amd.parallel.dist import init_from_env
    from pytorch_operator_amd.parallel.graphed_step import GraphedStep
    from pytorch_operator_amd.parallel.xgmi import try_xgmi

    env = init_from_env(a.backend, use_gpu=True)
    rank, world, dev = env.rank, env.world_size, env.device
    B = 64
    ds = make_synthetic_mnist(a.dataset, seed=21 + rank, device=dev)
    res = {"rank": rank, "world": world, "backend": env.backend, "tol": a.tol}

    def hip_replica(sync):
        cursor = torch.zeros(1, dtype=torch.int32, device=dev)
        src = K.BatchSource(ds.images, ds.labels, perm=ds.perm, cursor=cursor)
        tr = FusedMnistTrainer(batch_size=B, source=src, lr=0.01, momentum=0.5, device=dev,
                               seed=1 + rank, grad_sync=sync)
        dist.broadcast(tr.flat_params, 0)  # DDP constructor semantics, as bench.py
        return tr

    trained, runners = {}, {}
    for path in [p for p in a.paths.split(",") if p]:
        if path == "rccl":
            tr = hip_replica(FlatGradAllReduce())
        elif path == "xgmi":
            xg = try_xgmi(flat_layout().total, dev, required=True,
                          log=lambda m: print(m, file=sys.stderr) if rank == 0 else None)
            tr = hip_replica(xg)
        else:
            raise SystemExit(f"unknown path {path}")
        runner = GraphedStep(tr, mode="eager" if a.eager else "graph", launch="stream")
        if runner.internal_steps > 1:
            raise SystemExit("more than one untimed preparation step: its decisions are lost")
        runners[path] = (tr, runner, [])
        if not a.interleave:
            _run_path(runners[path], a.steps, B, dev)
    if a.interleave:
        for _ in range(a.steps):
            for v in runners.values():
                _run_path(v, len(v[2]) + 1, B, dev)
    for path, (tr, runner, codes) in runners.items():
        steps = int(tr.cursor.item())
        if steps != len(codes):
            raise SystemExit(f"cursor {steps} != steps taken {len(codes)}")
        trained[path] = (tr, steps, runner.launch, getattr(tr.grad_sync, "xar", None), codes)

    # torch's DDP on the same per-rank batches (cursor t -> perm[t*B : (t+1)*B], wrapping):
    # decision-aligned (DecisionAlignedNet: HIP's pool argmaxes and ReLU masks, each checked to be
    # torch's own up to rounding), and torch's own decisions for reference
    xf, lab, perm = ds.float_images().cpu(), ds.labels.long().cpu(), ds.perm.long().cpu()
    n = perm.numel()

    def torch_ddp(codes, steps):
        torch.manual_seed(1 + rank)  # this rank's own init: only DDP's broadcast aligns the ranks
        net = DecisionAlignedNet()
        ddp = torch.nn.parallel.DistributedDataParallel(net)
        opt = torch.optim.SGD(ddp.parameters(), lr=0.01, momentum=0.5)
        for t in range(steps):
            idx = perm[(torch.arange(B) + t * B) % n]
            opt.zero_grad(set_to_none=True)
            args = (xf[idx],) + (codes[t] if codes is not None else ())
            F.nll_loss(ddp(*args), lab[idx]).backward()
            opt.step()
        return (dict(net.named_parameters()), {k: opt.state[q]["momentum_buffer"] for k, q in net.named_parameters()},
                getattr(net, "decision_gap", 0.0))

    worst = {}
    for path, (tr, steps, launch, xar, codes) in trained.items():
        ref_p, ref_m, gap = torch_ddp(codes, steps)
        own_p, _, _ = torch_ddp(None, steps)
        row = {"steps": steps, "launch": launch, "decisions_aligned": True,
               "param_rel": max(_rel(tr.params[k], ref_p[k]) for k in ref_p),
               "decision_gap": gap,
               "param_rel_torch_own_decisions": max(_rel(tr.params[k], own_p[k]) for k in own_p)}
        if path == "rccl":  # the xGMI step keeps momentum only for the rank's own shard
            mv = _views(tr.flat_momentum, tr.layout)
            row["momentum_rel"] = max(_rel(mv[k], ref_m[k]) for k in ref_m)
        if xar is not None:
            row["kernel_error"] = int(xar.error())
        res[path] = row
        for key in ("param_rel", "momentum_rel", "decision_gap"):
            if key in row:
                worst[f"{path}_{key}"] = row[key]
    # worst over ranks
    keys = sorted(worst)
    v = torch.tensor([worst[k] for k in keys], dtype=torch.float64)
    dist.all_reduce(v, op=dist.ReduceOp.MAX)
    res["worst_over_ranks"] = dict(zip(keys, [float(x) for x in v]))
    errs = torch.tensor([res[p].get("kernel_error", 0) for p in trained], dtype=torch.int64)
    dist.all_reduce(errs, op=dist.ReduceOp.MAX)
    ok = all(x <= (a.gap_tol if k.endswith("decision_gap") else a.tol) for k, x in zip(keys, v.tolist())) and \
        int(errs.max()) == 0 and all(t[1] >= 10 for t in trained.values())
    res["all_ok"] = bool(ok)
    if rank == 0:
        print(json.dumps(res), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
