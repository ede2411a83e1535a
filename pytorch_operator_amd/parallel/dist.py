"""Process-group bring-up from the operator's rendezvous contract.

The operator injects ``MASTER_ADDR``, ``MASTER_PORT``, ``WORLD_SIZE`` and ``RANK``
into every replica (reference: pkg/controller.v1/pytorch/pod.go:234-281); the
worker initialises ``torch.distributed`` with ``env://`` exactly like
examples/mnist/mnist.py:114-116 and examples/smoke-dist/dist_sendrecv.py:36-39.

MI355X specifics:
* ``--backend rccl`` is accepted as an alias of ``nccl`` (ROCm's nccl backend *is*
  RCCL; collectives ride the point-to-point xGMI links).
* one process per GPU: the device is ``LOCAL_RANK`` (set by torchrun or by the
  operator's optional ``LOCAL_RANK`` injection), falling back to ``RANK % ngpus``.
* MPI is not available in this image (``torch.distributed.is_mpi_available()`` is
  False); requesting it raises a clear error.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist

_ALIASES = {"rccl": "nccl", "nccl": "nccl", "gloo": "gloo", "mpi": "mpi"}


@dataclass
class DistEnv:
    rank: int
    world_size: int
    local_rank: int
    master_addr: str
    master_port: int
    backend: str
    device: torch.device

    @property
    def is_master(self) -> bool:
        return self.rank == 0


def backend_for(name: Optional[str], use_gpu: bool) -> str:
    if not name:
        return "nccl" if use_gpu else "gloo"
    key = name.lower()
    if key not in _ALIASES:
        raise ValueError(f"unknown backend {name!r} (choices: gloo, nccl, rccl, mpi)")
    b = _ALIASES[key]
    if b == "mpi" and not dist.is_mpi_available():
        raise RuntimeError("MPI backend is not available in this PyTorch-ROCm build; use rccl")
    return b


def is_distributed() -> bool:
    return dist.is_available() and dist.is_initialized()


def env_world_size() -> int:
    return int(os.environ.get("WORLD_SIZE", "1"))


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def init_from_env(backend: Optional[str] = None, use_gpu: Optional[bool] = None,
                  timeout_s: float = 600.0, force_pg: bool = False) -> DistEnv:
    """Initialise the default process group from the env contract (if WORLD_SIZE>1, or with
    ``force_pg`` also at world 1: a single-rank group, e.g. to run RCCL collectives on one GPU;
    a missing MASTER_ADDR/MASTER_PORT then defaults to 127.0.0.1 and a free port)."""
    if use_gpu is None:
        use_gpu = torch.cuda.is_available()
    world = env_world_size()
    rank = int(os.environ.get("RANK", "0"))
    ngpu = torch.cuda.device_count() if use_gpu else 0
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank % ngpu if ngpu else 0)))
    b = backend_for(backend, use_gpu)
    if use_gpu:
        dev_index = local_rank
        if ngpu and local_rank >= ngpu:
            if b == "nccl":
                raise RuntimeError(f"LOCAL_RANK {local_rank} but only {ngpu} visible GPU(s); RCCL needs one GPU per rank")
            # gloo rehearsal of a multi-rank job on fewer GPUs (ranks share a device)
            dev_index = local_rank % ngpu
        torch.cuda.set_device(dev_index)
        device = torch.device("cuda", dev_index)
    else:
        device = torch.device("cpu")
    if force_pg and world == 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
    port = int(os.environ.get("MASTER_PORT", "23456"))
    if (world > 1 or force_pg) and not dist.is_initialized():
        kw = {}
        if b == "nccl" and use_gpu:
            kw["device_id"] = device
        dist.init_process_group(b, timeout=datetime.timedelta(seconds=timeout_s), **kw)
    return DistEnv(rank, world, local_rank, addr, port, b, device)
