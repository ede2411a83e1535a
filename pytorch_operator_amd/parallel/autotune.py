"""Pick the faster DDP gradient path on the actual hardware, at start-up.

The xGMI peer-memory kernel (``parallel.xgmi``) is expected to beat RCCL for this 1.7 MB
gradient on a fully connected 8x MI355X node, but that is a property of the fabric the
job lands on, so it is measured rather than assumed: both paths run a short graph-replayed
trial inside the warm-up, every rank reports its time, and all ranks adopt the path with
the lower MAX-over-ranks time.  Both trials are real DDP steps (replicas stay identical);
when RCCL wins after the xGMI trial, the sharded momentum is reassembled first.
"""
from __future__ import annotations

import time
from typing import Optional, Tuple

import torch
import torch.distributed as dist

from .graphed_step import GraphedStep


def _timed(runner: GraphedStep, steps: int, device) -> float:
    torch.cuda.synchronize(device)
    dist.barrier()
    t0 = time.perf_counter()
    runner.warm(steps)
    torch.cuda.synchronize(device)
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def choose_grad_sync(tr, rccl_sync, xgmi_sync, mode: str = "graph", spg: int = 10,
                     trial_steps: int = 60, force: Optional[str] = None,
                     launch: str = "graph") -> Tuple[GraphedStep, str, dict]:
    """Returns (runner, "xgmi" | "rccl", per-step times of both trials + ``steps``: the
    training steps taken here).  ``force`` overrides the measured decision (tests use it to
    cover both hand-overs).  ``spg``: whole steps per replay of the returned xGMI runner's
    timed graph; the trials replay one-step graphs, so any ``trial_steps`` works."""
    trial = max(1, int(trial_steps))
    # the RCCL step keeps momentum for every parameter: make it whole if fused xGMI steps
    # ran before (a no-op when it already is)
    xgmi_sync.xar.gather_sharded_(tr.flat_momentum)
    tr.grad_sync = rccl_sync
    r_rccl = GraphedStep(tr, mode=mode, steps_per_graph=1 if mode == "graph" else spg)
    t_rccl = _timed(r_rccl, trial, tr.device)
    tr.grad_sync = xgmi_sync
    r_xgmi = GraphedStep(tr, mode="graph", steps_per_graph=spg, launch=launch)
    t_xgmi = _timed(r_xgmi, trial, tr.device)
    if xgmi_sync.xar.error():
        t_xgmi = float("inf")
    want = (t_xgmi < t_rccl) if force is None else (force == "xgmi")
    flag = torch.tensor([1 if want else 0], dtype=torch.int32, device=tr.device)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)  # unanimous or RCCL
    times = {"rccl_ms_per_step": round(t_rccl / trial * 1e3, 4), "xgmi_ms_per_step": round(t_xgmi / trial * 1e3, 4),
             "steps": r_rccl.internal_steps + r_xgmi.internal_steps + 2 * trial}
    if flag.item():
        return r_xgmi, "xgmi", times
    xgmi_sync.xar.gather_sharded_(tr.flat_momentum)
    tr.grad_sync = rccl_sync
    return r_rccl, "rccl", times
