#!/usr/bin/env python3
"""The RCCL gradient-path step forms under a real (single-rank) RCCL communicator.

At world 1 ``FlatGradAllReduce`` normally skips its collectives; with ``force=True`` (a
single-rank ``nccl`` process group, ``init_from_env(force_pg=True)``) both bucket all-reduces
are issued every step.  This runs, on one GPU, the forms the start-up race
(``parallel/autotune.py``) would otherwise execute for the first time on a multi-GPU node:

* ``rccl``        stream-launched pieces with eager RCCL all-reduces between them;
* ``rccl-graph``  ``GraphedStep(mode="graph-comm")``: the step with its collectives in one graph;
* eager steps with the collectives.

Each trainer takes N steps from the same initial state; at world 1 the all-reduce is an exact
identity, so params and momentum must equal (``torch.equal``) the split step without collectives,
and that must equal the single-GPU step it is built from: the default (round 6) DDP form is the
five-launch step's kernels plus a gradient tail and one SGD launch, bit-identical to the
five-launch single-GPU step; the round-5 form (``ddp_fused`` off: head launch + fc1_bwd) is
bit-identical to the six-kernel single-GPU step (head launch).  Then the RCCL race runs (``choose_grad_sync`` without an xGMI
candidate) beside a timed six-kernel run of the same length: RCCL's single-rank floor.

    python tools/rccl_w1_check.py --out DIR      (writes DIR/rank0.json, exit 0 iff all equal)
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--trial-steps", type=int, default=200)
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    import torch
    import torch.distributed as dist
    from pytorch_operator_amd.data.synthetic import make_synthetic_mnist
    from pytorch_operator_amd.models.mnist import FusedMnistTrainer
    from pytorch_operator_amd.ops import mnist as K
    from pytorch_operator_amd.parallel.autotune import _timed, choose_grad_sync
    from pytorch_operator_amd.parallel.ddp import FlatGradAllReduce
    from pytorch_operator_amd.parallel.dist import init_from_env
    from pytorch_operator_amd.parallel.graphed_step import GraphedStep

    env = init_from_env("nccl", use_gpu=True, force_pg=True)
    dev = env.device
    assert dist.get_world_size() == 1 and dist.get_backend() == "nccl"
    res = {"rank": env.rank, "world": 1, "backend": "rccl",
           "rccl_version": ".".join(map(str, torch.cuda.nccl.version()))}
    ds = make_synthetic_mnist(8192, seed=11, device=dev)

    def trainer(sync):
        cursor = torch.zeros(1, dtype=torch.int32, device=dev)
        src = K.BatchSource(ds.images, ds.labels, perm=ds.perm, cursor=cursor)
        return FusedMnistTrainer(batch_size=64, source=src, lr=0.01, momentum=0.5, device=dev, seed=1,
                                 grad_sync=sync)

    N = a.steps
    six = trainer(None)                              # the single-GPU six-kernel step (head launch)
    six.fuse_head = False
    fused = trainer(None)                            # the five-launch step (head fused into fc1_bwd)
    split = trainer(FlatGradAllReduce(force=False))  # the DDP step's kernels, collectives skipped
    split_r5 = trainer(FlatGradAllReduce(force=False))
    split_r5.ddp_fused = False                       # the round-5 DDP form: head + fc1_bwd, 7 launches
    eager = trainer(FlatGradAllReduce(force=True))
    for tr in (six, fused, split, split_r5, eager):
        for _ in range(N):
            tr.train_step()
    forms = {"eager": eager}
    for name, mode in (("rccl", "graph"), ("rccl_graph", "graph-comm")):
        tr = trainer(FlatGradAllReduce(force=True))
        r = GraphedStep(tr, mode=mode, launch="stream")
        res[f"{name}_exec"] = {"split": r._split, "launch": r.launch, "internal_steps": r.internal_steps}
        r.run(N - r.internal_steps)
        forms[name] = tr
    torch.cuda.synchronize(dev)
    res["steps"] = N
    res["cursors"] = {k: int(t.cursor.item()) for k, t in [("six", six), ("fused", fused), ("split", split),
                                                           ("split_r5", split_r5), *forms.items()]}
    res["ddp_form"] = "fused" if split.fused_ok() else "r5"
    res["issued"] = {k: t.grad_sync.issued for k, t in forms.items()}

    def same(x, y):
        return bool(torch.equal(x.flat_params, y.flat_params) and torch.equal(x.flat_momentum, y.flat_momentum))
    res["split_vs_fused_equal"] = same(split, fused)
    res["split_r5_vs_six_equal"] = same(split_r5, six)
    res["split_vs_six_equal"] = same(split, six)
    res["fused_head_max_rel_diff_vs_six"] = float((fused.flat_params - six.flat_params).abs().max() /
                                                 six.flat_params.abs().max())
    for k, t in forms.items():
        res[f"{k}_vs_split_equal"] = same(t, split)
        res[f"{k}_vs_six_equal"] = same(t, six)
        res[f"{k}_max_diff_vs_six"] = float((t.flat_params - six.flat_params).abs().max())

    # the race (no xGMI candidate at world 1) beside the no-collective six-kernel step
    rt = trainer(FlatGradAllReduce(force=True))
    rt.train_step()
    runner, pick, rec = choose_grad_sync(rt, rt.grad_sync, None, trial_steps=a.trial_steps, launch="stream")
    base = trainer(None)
    rb = GraphedStep(base, mode="graph", launch="stream")
    rb.warm(20)
    t_six = _timed(rb, a.trial_steps, dev, "six")
    rec["six_kernel_ms_per_step"] = round(t_six / a.trial_steps * 1e3, 4)
    res["race"] = rec
    res["picked"] = pick
    ok = all(res["cursors"][k] == N for k in res["cursors"]) and res["split_vs_fused_equal"] and \
        res["split_r5_vs_six_equal"] and all(
        res[f"{k}_vs_split_equal"] for k in forms) and all(v > 0 for v in res["issued"].values()) and (
        rec.get("rccl_ms_per_step") is not None and rec.get("rccl_graph_ms_per_step") is not None)
    res["all_ok"] = bool(ok)
    print(json.dumps(res), flush=True)
    if a.out:
        os.makedirs(a.out, exist_ok=True)
        with open(os.path.join(a.out, "rank0.json"), "w") as f:
            json.dump(res, f)
    dist.destroy_process_group()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
