"""Checkpoint / resume for the large-model DDP worker (``harness/ddp_train.py --ckpt-dir``).

BASELINE's "Llama-3 8B DDP ... OnFailure restart" only pays off if a restarted replica set
continues where it stopped: the operator restarts the pods (retryable exit codes,
``pkg/controller.v1/pytorch/controller.go`` + tf-operator ``train_util.go:18-53``), the worker
reloads the last checkpoint.  The MNIST worker has the reference's own ``--save-model`` plus
epoch checkpoints (``harness/mnist.py``); this is the same contract for the bigger workers.

Layout of ``<dir>``:
  step_<N>/model.pt          weights as the model holds them (bf16 matmul weights, fp32 rest), rank 0
  step_<N>/optim.pt          replicated optimizer state (DDP paths), rank 0
  step_<N>/optim_rank<r>.pt  this rank's shard (ZeRO-1: fp32 master + moments of its 1/W of each bucket)
  meta.json                  {"step", "world", "sharded", "subdir"}: the pointer to the newest COMPLETE
                             checkpoint, replaced atomically by rank 0 after every rank finished
                             writing step_<N>/ (a barrier); older step_* directories are pruned
                             after the pointer moved (``keep`` newest are kept)

A crash at any point of ``save`` leaves meta.json pointing at the previous complete checkpoint:
files of the interrupted save live only in their own step_<N>/ directory, which no pointer
names, so ``load`` never mixes shards of different steps.  All files are written to a
temporary name and renamed; tensors are loaded with ``torch.load(weights_only=True)``.  A
sharded checkpoint needs the same world size to resume.  (Checkpoints written before this
layout -- files directly in ``<dir>``, meta.json without "subdir" -- still load.)
"""
from __future__ import annotations

import json
import os
import shutil
from typing import Optional

import torch
import torch.distributed as dist


def _atomic_save(obj, path: str) -> None:
    tmp = path + ".tmp"
    torch.save(obj, tmp)
    os.replace(tmp, path)


def _barrier(world: int) -> None:
    if world > 1:
        dist.barrier()


def _cpu(x):
    if isinstance(x, torch.Tensor):
        return x.detach().cpu()
    if isinstance(x, dict):
        return {k: _cpu(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(_cpu(v) for v in x)
    return x


def optimizer_state(opt) -> dict:
    """Replicated optimizer state in a form that reloads without dtype casts: MasterAdamW keeps
    fp32 masters/moments for bf16 parameters, which ``Optimizer.load_state_dict`` would cast
    to the parameter dtype, so its per-parameter state is stored by parameter index."""
    from ..ops.optim import MasterAdamW
    if isinstance(opt, MasterAdamW):
        params = [p for g in opt.param_groups for p in g["params"]]
        return {"kind": "master_adamw",
                "state": [{k: v for k, v in opt.state[p].items()} if p in opt.state else None for p in params]}
    return {"kind": "torch", "state_dict": opt.state_dict()}


def load_optimizer_state(opt, blob: dict) -> None:
    if blob["kind"] == "master_adamw":
        params = [p for g in opt.param_groups for p in g["params"]]
        if len(params) != len(blob["state"]):
            raise ValueError("checkpoint optimizer state does not match the parameters")
        for p, st in zip(params, blob["state"]):
            if st is None:
                continue
            opt.state[p] = {k: (v.to(p.device) if isinstance(v, torch.Tensor) else v) for k, v in st.items()}
            if hasattr(p, "_pto_master"):
                del p._pto_master  # the checkpoint's master replaces the init copy
    else:
        opt.load_state_dict(blob["state_dict"])


def _step_dirs(dirpath: str):
    out = []
    for name in os.listdir(dirpath):
        if name.startswith("step_") and name[5:].isdigit() and os.path.isdir(os.path.join(dirpath, name)):
            out.append((int(name[5:]), name))
    return sorted(out)


def save(dirpath: str, step: int, model, opt, rank: int, world: int, keep: int = 2) -> None:
    sub = f"step_{int(step)}"
    path = os.path.join(dirpath, sub)
    os.makedirs(path, exist_ok=True)
    sharded = hasattr(opt, "shard_state_dict")
    if hasattr(opt, "synchronize"):
        opt.synchronize()  # ZeRO: weights all-gathered before they are written
    if rank == 0:
        _atomic_save(_cpu(model.state_dict()), os.path.join(path, "model.pt"))
        if not sharded:
            _atomic_save(_cpu(optimizer_state(opt)), os.path.join(path, "optim.pt"))
    if sharded:
        _atomic_save(_cpu(opt.shard_state_dict()), os.path.join(path, f"optim_rank{rank}.pt"))
    _barrier(world)  # every rank's files of step_<N> are complete
    if rank == 0:
        # the pointer file lists the last `keep` COMPLETE checkpoints (newest last); everything
        # else under step_* is pruned -- including a higher-numbered directory a crashed save left
        # behind, which must never displace the fallback checkpoint
        prev = []
        meta_path = os.path.join(dirpath, "meta.json")
        if os.path.exists(meta_path):
            try:
                with open(meta_path) as f:
                    old = json.load(f)
                prev = old.get("complete") or ([old["subdir"]] if old.get("subdir") else [])
            except (OSError, ValueError):
                prev = []
        older = [d for d in prev if d != sub and os.path.isdir(os.path.join(dirpath, d))]
        complete = (older[-(keep - 1):] if keep > 1 else []) + [sub]
        tmp = os.path.join(dirpath, "meta.json.tmp")
        with open(tmp, "w") as f:
            json.dump({"step": int(step), "world": int(world), "sharded": sharded, "subdir": sub,
                       "complete": complete}, f)
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, meta_path)
        for _, name in _step_dirs(dirpath):
            if name not in complete:
                shutil.rmtree(os.path.join(dirpath, name), ignore_errors=True)
    _barrier(world)


def load(dirpath: Optional[str], model, opt, rank: int, world: int, device) -> int:
    """Restore the last checkpoint in ``dirpath`` (if any); returns the step it was taken at (0: none)."""
    if not dirpath or not os.path.exists(os.path.join(dirpath, "meta.json")):
        return 0
    with open(os.path.join(dirpath, "meta.json")) as f:
        meta = json.load(f)
    sharded = hasattr(opt, "shard_state_dict")
    if meta["sharded"] != sharded or (sharded and meta["world"] != world):
        raise ValueError(f"checkpoint {dirpath} (world {meta['world']}, sharded {meta['sharded']}) cannot "
                         f"resume a world-{world} {'sharded' if sharded else 'replicated'} optimizer")
    path = os.path.join(dirpath, meta["subdir"]) if meta.get("subdir") else dirpath
    sd = torch.load(os.path.join(path, "model.pt"), map_location=device, weights_only=True)
    with torch.no_grad():
        model.load_state_dict(sd)  # copies into the existing (bucket-view) parameters
    if sharded:
        opt.load_shard_state_dict(torch.load(os.path.join(path, f"optim_rank{rank}.pt"), map_location=device,
                                             weights_only=True))
    else:
        load_optimizer_state(opt, torch.load(os.path.join(path, "optim.pt"), map_location=device,
                                             weights_only=True))
    return int(meta["step"])
