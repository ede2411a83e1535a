#!/usr/bin/env python3
"""Rehearse the xGMI peer-memory all-reduce with W ranks on the GPUs this box has.

    torchrun --nproc-per-node 2 tools/xgmi_check.py [--backend gloo]

On a 1-GPU box the ranks share GPU 0 (gloo for the reference collectives), which still
exercises the whole protocol -- IPC export/import, counters, parity buffers, bounded
waits, fused SGD, graph capture -- everything except the cross-GPU fabric itself.
Prints one JSON line per rank; exit 0 iff every check passed on every rank.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _bench_exchange(xar, tr, dev, launches: int = 50, reps: int = 5) -> dict:
    """us per fused exchange launch (slab reduce + push + reduce-scatter/SGD + all-gather),
    back-to-back in one graph, MAX over ranks; on a shared GPU this bounds the protocol's
    latency floor, not the xGMI fabric's."""
    import time
    import torch
    import torch.distributed as dist
    p, m, g = tr.flat_params.clone(), tr.flat_momentum.clone(), tr.flat_grads.clone()
    slab, B, ce = tr.conv_slab, tr.B, tr.layout.conv_end

    def body():
        for _ in range(launches):
            xar.allreduce_sgd_(g, p, m, lr=0.0, momentum=0.5, slab=slab, slab_rows=B, conv_n=ce)
    body()
    torch.cuda.synchronize(dev)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        body()
    best = float("inf")
    for _ in range(reps):
        torch.cuda.synchronize(dev)
        dist.barrier()
        t0 = time.perf_counter()
        graph.replay()
        torch.cuda.synchronize(dev)
        t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        best = min(best, float(t.item()))
    return {"per_launch_us": round(best / launches * 1e6, 2), "launches": launches}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default="gloo")
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--out", default=None, help="also write <out>/rank<r>.json")
    ap.add_argument("--nblk", type=int, default=0,
                    help="workgroups per rank (0 = auto: 256 when every rank owns its GPU, 128 "
                         "when ranks share one; 256 on a shared GPU runs the cross-device geometry)")
    ap.add_argument("--handover-nblk", type=int, default=0,
                    help="workgroups of the hand-over stage's exchange (0 = the main exchange's)")
    ap.add_argument("--stamps", action="store_true",
                    help="record the hand-over exchange's per-workgroup phase stamps (XgmiAllReduce."
                         "enable_stamps) and write <out>/rank<r>_stamps.json (tools/xgmi_stamps.py reads them)")
    ap.add_argument("--fuse-conv12", type=int, default=-1,
                    help="1/0: force the fused conv12 forward on/off (default: on, off only under "
                         "--prebarrier 0 at two exchange waves per SIMD, see below)")
    ap.add_argument("--prebarrier", type=int, default=-1,
                    help="1/0: rank barrier before each exchange (default: on when crowded)")
    ap.add_argument("--conv-chunk", type=int, default=0,
                    help="conv backward samples per chunk (0 = auto: 1 where conv12 is split, else 4)")
    ap.add_argument("--ddp-form", default="auto", choices=["auto", "fused", "r5"],
                    help="DDP step form (auto: fused, round-5 only under --prebarrier 0 when crowded)")
    ap.add_argument("--bench", action="store_true",
                    help="time the fused exchange alone (graph of back-to-back launches)")
    a = ap.parse_args(argv)
    import torch
    import torch.distributed as dist
    from pytorch_operator_amd.data.synthetic import make_synthetic_mnist
    from pytorch_operator_amd.models.mnist import FusedMnistTrainer, flat_layout
    from pytorch_operator_amd.ops import mnist as K
    from pytorch_operator_amd.parallel.ddp import FlatGradAllReduce
    from pytorch_operator_amd.parallel.dist import init_from_env
    from pytorch_operator_amd.parallel.graphed_step import GraphedStep
    from pytorch_operator_amd.parallel.xgmi import XgmiAllReduce, XgmiGradSync

    env = init_from_env(a.backend, use_gpu=True)
    rank, world, dev = env.rank, env.world_size, env.device
    res = {"rank": rank, "world": world}
    L = flat_layout().total
    xar = XgmiAllReduce(L, device=dev, nblk=a.nblk)
    res["nblk"] = xar.nblk
    res["alloc_kind"] = xar.alloc_kind
    stamps_main = xar.enable_stamps(64) if a.stamps else None
    res["self_test"] = xar.self_test()
    res["self_test_report"] = xar.last_report[:4]

    ds = make_synthetic_mnist(4096, seed=11 + rank, device=dev)
    # Ranks sharing one GPU: a rank's exchange workgroups spin on the CUs until its peers reach the
    # same step.  A peer still running its step kernels must then find room beside them: its waves
    # per SIMD x VGPR allocation + the spinning exchange waves' <= 512, and its LDS in ONE free
    # range.  Round 5 found the fused conv12 forward waiting out the peer's deadline beside the
    # 112-VGPR exchange (profiles/r5_xgmi_handover.md); round 6 brought the exchange to 96 VGPRs, so
    # every production kernel fits the budget beside one exchange wave per SIMD
    # (tests/test_kernel_resources.py) -- and still saw the same starvation now and then: LDS / VGPR
    # fragmentation around a spinning workgroup (an exchange workgroup's 4.3 KB placed mid-LDS leaves
    # no 152 KB range for conv_bwd4).  The fix is the ordering, not the budget: when crowded, a
    # one-wave rank barrier runs before every exchange (XgmiAllReduce.set_prebarrier), so no rank's
    # exchange starts before every rank has finished its step kernels, and the rehearsal runs the
    # production step in the fused DDP form (profiles/r6_xgmi_geometry.md).  --prebarrier 0 keeps the
    # budget-only policy: the round-5 form, split conv kernels at two exchange waves per SIMD.  The
    # job topology never shares CUs: one rank per GPU runs its own kernels in stream order.
    peers = [None] * world
    dist.all_gather_object(peers, dev.index)
    on_gpu = sum(1 for p in peers if p == dev.index)
    exch_waves = -(-(on_gpu - 1) * xar.nblk // 256) if on_gpu > 1 else 0
    crowded = on_gpu > 1 and (on_gpu - 1) * xar.nblk >= 256  # every CU can hold a spinning exchange
    res["crowded"] = crowded
    res["exchange_waves_per_simd"] = exch_waves
    res["prebarrier"] = crowded if a.prebarrier < 0 else bool(a.prebarrier)
    budget_only = crowded and not res["prebarrier"]
    split = budget_only and exch_waves >= 2
    res["conv_chunk"] = a.conv_chunk if a.conv_chunk > 0 else (1 if split else 4)
    res["fuse_conv12"] = bool(a.fuse_conv12) if a.fuse_conv12 >= 0 else not split
    res["ddp_form"] = "r5" if (budget_only if a.ddp_form == "auto" else a.ddp_form == "r5") else "fused"
    xar.set_prebarrier(res["prebarrier"])  # XgmiAllReduce turns it on by itself when crowded

    def trainer(sync):
        cursor = torch.zeros(1, dtype=torch.int32, device=dev)
        src = K.BatchSource(ds.images, ds.labels, perm=ds.perm, cursor=cursor)
        tr = FusedMnistTrainer(batch_size=64, source=src, lr=0.01, momentum=0.5, device=dev, seed=1,
                               grad_sync=sync)
        tr.conv_chunk = res["conv_chunk"]
        tr.fuse_conv12 = res["fuse_conv12"]
        tr.ddp_fused = res["ddp_form"] == "fused"
        dist.broadcast(tr.flat_params, 0)
        return tr

    ta = trainer(XgmiGradSync(xar))
    tb = trainer(FlatGradAllReduce())
    # the exchange pushing dW_fc1 itself (fc1_bwd's producer push off): must be bit-identical
    nopush = XgmiGradSync(xar)
    nopush.push_fc1 = False
    tc = trainer(nopush)
    res["push_fc1"] = bool(getattr(ta.grad_sync, "push_fc1", False))
    for _ in range(a.steps):
        ta.train_step()
        tb.train_step()
        tc.train_step()
    torch.cuda.synchronize(dev)
    res["max_diff_vs_rccl_path"] = float((ta.flat_params - tb.flat_params).abs().max())
    res["eager_match"] = res["max_diff_vs_rccl_path"] < 1e-4
    res["push_bit_identical"] = bool(torch.equal(ta.flat_params, tc.flat_params)) and bool(
        torch.equal(ta.flat_momentum, tc.flat_momentum))
    res["error_after"] = {"eager": xar.error()}

    runner = GraphedStep(ta, mode="graph", steps_per_graph=4)
    torch.cuda.synchronize(dev)
    dist.barrier()
    runner.run(8)
    torch.cuda.synchronize(dev)
    ref = ta.flat_params.clone()
    dist.broadcast(ref, 0)
    res["graph_in_sync"] = bool(torch.equal(ref, ta.flat_params))
    res["error_after"]["graph"] = xar.error()
    res["finite"] = bool(torch.isfinite(ta.flat_params).all())
    # autotune hand-over in both directions keeps the replicas identical (on the main exchange's
    # geometry; round 4 ran it at 128 workgroups when ranks shared a GPU at 256 -- the timeouts
    # that prompted it were the co-residency starvation above, not the hand-over)
    from pytorch_operator_amd.parallel.autotune import choose_grad_sync
    hnb = a.handover_nblk or xar.nblk
    hx = XgmiAllReduce(L, device=dev, nblk=hnb) if hnb != xar.nblk else xar
    if hx is not xar:
        hx.set_prebarrier(res["prebarrier"])
    stamps_hx = hx.enable_stamps(64) if a.stamps and hx is not xar else None
    if hx is not xar:
        res["handover_self_test"] = hx.self_test()
    res["handover_nblk"] = hx.nblk
    launch = "stream"
    res["handover_launch"] = launch
    for force in ("rccl", "xgmi"):
        try:
            runner, path, times = choose_grad_sync(ta, FlatGradAllReduce(), XgmiGradSync(hx), spg=4,
                                                   trial_steps=8, force=force, launch=launch)
        except ValueError as e:  # the forced candidate was dropped (its step cross-check failed)
            res[f"handover_{force}_in_sync"] = False
            res[f"handover_{force}_error"] = str(e)[:300]
            res["error_after"][f"handover_{force}"] = hx.error()
            continue
        runner.run(8)
        torch.cuda.synchronize(dev)
        ref = ta.flat_params.clone()
        dist.broadcast(ref, 0)
        mref = ta.flat_momentum.clone()
        dist.broadcast(mref, 0)
        res[f"handover_{force}_in_sync"] = bool(torch.equal(ref, ta.flat_params)) and (
            force == "xgmi" or bool(torch.equal(mref, ta.flat_momentum)))
        res[f"handover_{force}_times"] = times
        res["error_after"][f"handover_{force}"] = hx.error()
    if a.bench:
        res["exchange_us"] = _bench_exchange(xar, ta, dev)
    res["kernel_error"] = xar.error() | (hx.error() if hx is not xar else 0)
    if a.stamps and a.out:
        torch.cuda.synchronize(dev)
        res["stamp_rows"] = {}
        for tag, xx, st in (("main", xar, stamps_main), ("handover", hx, stamps_hx)):
            if st is None:
                continue
            rows = [[i % xx.nblk] + r[:7] for i, r in enumerate(st.view(-1, 8).cpu().tolist()) if r[0] > 0]
            os.makedirs(os.path.join(a.out, f"stamps_{tag}"), exist_ok=True)
            with open(os.path.join(a.out, f"stamps_{tag}", f"rank{rank}_stamps.json"), "w") as f:
                json.dump({"rank": rank, "world": world, "nblk": xx.nblk, "error": xx.error(), "timeout_s": 5.0,
                           "fields": ["block", "step", "start", "flag1", "flag2", "end", "err", "missing"],
                           "rows": rows}, f)
            res["stamp_rows"][tag] = len(rows)
    ok = res.get("handover_self_test", True) and res["self_test"] and res["eager_match"] and res["push_bit_identical"] and res["graph_in_sync"] and res["finite"] \
        and res["kernel_error"] == 0 and res["handover_rccl_in_sync"] and res["handover_xgmi_in_sync"]
    flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    res["all_ok"] = bool(flag.item())
    print(json.dumps(res), flush=True)
    if a.out:
        os.makedirs(a.out, exist_ok=True)
        with open(os.path.join(a.out, f"rank{rank}.json"), "w") as f:
            json.dump(res, f)
    dist.barrier()
    if hx is not xar:
        hx.close()
    xar.close()
    dist.destroy_process_group()
    return 0 if res["all_ok"] else 1


if __name__ == "__main__":
    sys.exit(main())
