"""Master <-> worker smoke test (the ``smoke-dist`` job entrypoint).

Parity with the reference examples/smoke-dist/dist_sendrecv.py: log the rendezvous env
(MASTER_PORT, MASTER_ADDR, WORLD_SIZE, RANK), initialise the default process group,
then rank 0 sends a random 2x2 tensor to every worker and receives back its elementwise
square.  Additions: the master *checks* each reply (the reference only logs it), an
all-reduce of the ranks is verified on every rank, the backend may be ``rccl``, and with
``--device cuda`` the tensors live in HBM so the RCCL path over xGMI is exercised.
Exit code 0 = every check passed.
"""
from __future__ import annotations

import argparse
import logging
import os
import sys


def run(device: str) -> bool:
    import torch
    import torch.distributed as dist
    rank, size = dist.get_rank(), dist.get_world_size()
    ok = True
    g = torch.Generator().manual_seed(1234)
    inp = torch.randn(2, 2, generator=g).to(device)
    result = torch.zeros(2, 2, device=device)
    if rank == 0:
        for i in range(1, size):
            dist.send(tensor=inp, dst=i)
            dist.recv(tensor=result, src=i)
            logging.info("Result from worker %d : %s", i, result.cpu())
            if not torch.allclose(result, inp * inp):
                logging.error("worker %d returned a wrong result", i)
                ok = False
    else:
        dist.recv(tensor=inp, src=0)
        result = torch.mul(inp, inp)
        dist.send(tensor=result, dst=0)
    t = torch.tensor([float(rank + 1)], device=device)
    dist.all_reduce(t)
    want = size * (size + 1) / 2
    if abs(float(t.item()) - want) > 1e-6:
        logging.error("all_reduce gave %s, want %s", t.item(), want)
        ok = False
    else:
        logging.info("all_reduce ok (%s)", t.item())
    return ok


def main(argv=None) -> int:
    p = argparse.ArgumentParser(description="PyTorchJob distributed smoke test")
    p.add_argument("--backend", default=None, help="gloo | nccl | rccl (default: gloo on CPU, rccl on GPU)")
    p.add_argument("--device", default="cpu", choices=["cpu", "cuda"])
    args = p.parse_args(argv)
    logging.getLogger().setLevel(logging.INFO)
    logging.basicConfig(format="%(levelname)s:%(name)s:%(message)s", stream=sys.stdout)
    import torch
    from ..parallel.dist import init_from_env
    logging.info("Torch version: %s", torch.__version__)
    for k in ("MASTER_PORT", "MASTER_ADDR", "WORLD_SIZE", "RANK"):
        logging.info("%s: %s", k, os.environ.get(k, "{}"))
    use_gpu = args.device == "cuda"
    env = init_from_env(args.backend, use_gpu=use_gpu)
    import torch.distributed as dist
    if not dist.is_initialized():
        # WORLD_SIZE=1: still exercise the path with a single-rank group
        dist.init_process_group(env.backend, init_method=f"tcp://{env.master_addr}:{env.master_port}",
                                rank=0, world_size=1)
    device = str(env.device) if use_gpu else "cpu"
    ok = run(device)
    dist.barrier()
    dist.destroy_process_group()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
