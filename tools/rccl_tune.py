#!/usr/bin/env python3
"""Race RCCL tuning environments on the MNIST step's two gradient buckets.

RCCL reads NCCL_PROTO / NCCL_ALGO / NCCL_*CHANNELS when a communicator is created, so every
candidate runs in processes of its own: one ``torch.distributed.run`` job per candidate, each
rank timing ``all_reduce`` of the fc bucket (fc1 + fc2, 1.61 MB fp32) and of the conv bucket
(0.10 MB) back to back -- what the RCCL arm of the gradient path issues per step
(``parallel/ddp.py``) -- and rank 0 writing the per-step cost (MAX over ranks, median over
timed repetitions).  The winner comes out as the operator's ``--rccl-env`` flags (they replace
the injected set, so ``HSA_ENABLE_IPC_MODE_LEGACY=0`` is kept in them).

    python tools/rccl_tune.py --nproc 8 --out rccl_tune.json --env-out rccl.env   # the 8-GPU node
    pytorch-operator --inject-rccl-env --rccl-env-file rccl.env ...
    python tools/rccl_tune.py --nproc 2 --backend gloo --device cpu ...  # plumbing (CPU test)

At one rank RCCL's all-reduce is a local copy: the race then only checks that every candidate
initialises and runs under a real RCCL communicator; the protocol choice needs >= 2 GPUs.
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# name -> env.  Protocols x the two algorithms RCCL offers for all-reduce on one node; the
# default (RCCL's own tuning model) first.
CANDIDATES = {
    "default": {},
    "proto-LL": {"NCCL_PROTO": "LL"},
    "proto-LL128": {"NCCL_PROTO": "LL128"},
    "proto-Simple": {"NCCL_PROTO": "Simple"},
    "algo-Ring": {"NCCL_ALGO": "Ring"},
    "algo-Tree": {"NCCL_ALGO": "Tree"},
    "ring-LL": {"NCCL_ALGO": "Ring", "NCCL_PROTO": "LL"},
    "ring-LL128": {"NCCL_ALGO": "Ring", "NCCL_PROTO": "LL128"},
}
BASE_ENV = {"HSA_ENABLE_IPC_MODE_LEGACY": "0"}


def bucket_sizes() -> dict:
    """fp32 element counts of the two buckets the MNIST gradient path all-reduces."""
    from pytorch_operator_amd.models.mnist import flat_layout
    lay = flat_layout()
    return {"fc": lay.total - lay.conv_end, "conv": lay.conv_end}


def worker(args) -> int:
    import time

    import torch
    import torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    if args.device == "cuda":
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        dev = torch.device("cuda")
    else:
        dev = torch.device("cpu")
    dist.init_process_group(args.backend)
    sizes = bucket_sizes()
    bufs = {k: torch.ones(n, dtype=torch.float32, device=dev) for k, n in sizes.items()}

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()

    def one_step():
        for k in ("fc", "conv"):
            dist.all_reduce(bufs[k])

    for _ in range(args.warmup):
        one_step()
    sync()
    # correctness on a fresh pair of buffers: every element sums the ranks' rank + 1
    chk = {k: torch.full((n,), float(rank + 1), device=dev) for k, n in sizes.items()}
    for k in chk:
        dist.all_reduce(chk[k])
    want = world * (world + 1) / 2.0
    ok = all(bool(torch.all(chk[k] == want)) for k in chk)
    reps = []
    per = {"fc": [], "conv": []}
    for _ in range(args.reps):
        dist.barrier()
        sync()
        t0 = time.perf_counter()
        for _ in range(args.iters):
            one_step()
        sync()
        t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        reps.append(float(t.item()) / args.iters * 1e6)
        for k in ("fc", "conv"):  # each bucket alone, same protocol
            dist.barrier()
            sync()
            t0 = time.perf_counter()
            for _ in range(args.iters):
                dist.all_reduce(bufs[k])
            sync()
            t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            per[k].append(float(t.item()) / args.iters * 1e6)
    med = lambda v: sorted(v)[len(v) // 2]  # noqa: E731
    if rank == 0:
        rec = {"world": world, "backend": args.backend, "device": dev.type, "sizes": sizes,
               "step_us": round(med(reps), 2), "fc_us": round(med(per["fc"]), 2),
               "conv_us": round(med(per["conv"]), 2), "reps_us": [round(x, 2) for x in reps],
               "correct": ok, "nccl_env": {k: os.environ[k] for k in sorted(os.environ) if k.startswith("NCCL_")}}
        with open(args.out, "w") as f:
            json.dump(rec, f)
    dist.destroy_process_group()
    return 0 if ok else 1


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def race(names, nproc: int, backend: str, device: str, iters: int, reps: int, warmup: int,
         timeout: float) -> dict:
    """One torchrun job per candidate; returns the table and the winner (least step_us among
    the candidates that ran and all-reduced correctly)."""
    rows = []
    with tempfile.TemporaryDirectory(prefix="rccl_tune_") as td:
        for name in names:
            out = os.path.join(td, f"{name}.json")
            env = dict(os.environ)
            for k in [k for k in env if k.startswith("NCCL_PROTO") or k.startswith("NCCL_ALGO")]:
                del env[k]
            env.update(BASE_ENV)
            env.update(CANDIDATES[name])
            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
                   "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__),
                   "--worker", "--out", out, "--backend", backend, "--device", device, "--iters", str(iters),
                   "--reps", str(reps), "--warmup", str(warmup)]
            row = {"name": name, "env": CANDIDATES[name]}
            # own process group: a candidate that hangs is killed with its torchrun workers
            p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                                 start_new_session=True)
            try:
                so, se = p.communicate(timeout=timeout)
                if p.returncode == 0 and os.path.exists(out):
                    row.update(json.load(open(out)))
                else:
                    row["error"] = f"rc={p.returncode}: {(se or so)[-400:]}"
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
                p.communicate()
                row["error"] = f"timeout after {timeout} s"
            rows.append(row)
            print(json.dumps({k: row.get(k) for k in ("name", "step_us", "fc_us", "conv_us", "correct", "error")}),
                  flush=True)
    good = [r for r in rows if r.get("correct") and "step_us" in r]
    res = {"nproc": nproc, "backend": backend, "device": device, "iters": iters, "reps": reps,
           "sizes": bucket_sizes(), "candidates": rows}
    if good:
        best = min(good, key=lambda r: r["step_us"])
        flags = []
        for k, v in sorted({**BASE_ENV, **best["env"]}.items()):
            flags += ["--rccl-env", f"{k}={v}"]
        res["winner"] = {"name": best["name"], "step_us": best["step_us"], "env": best["env"],
                         "operator_flags": flags}
        dflt = next((r for r in good if r["name"] == "default"), None)
        if dflt is not None:
            res["winner"]["vs_default"] = round(dflt["step_us"] / best["step_us"], 3) if best["step_us"] else None
    if nproc == 1:
        res["note"] = "one rank: RCCL's all-reduce is a local copy; the protocol choice needs >= 2 GPUs"
    return res


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--worker", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--nproc", type=int, default=1)
    ap.add_argument("--backend", default="nccl")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"])
    ap.add_argument("--candidates", default=",".join(CANDIDATES),
                    help="comma-separated names from: " + ", ".join(CANDIDATES))
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--timeout", type=float, default=180.0, help="seconds per candidate job")
    ap.add_argument("--out", default=None)
    ap.add_argument("--env-out", default=None,
                    help="also write the winner's env as KEY=VALUE lines (pytorch-operator --rccl-env-file)")
    args = ap.parse_args(argv)
    if args.worker:
        return worker(args)
    names = [n for n in args.candidates.split(",") if n]
    unknown = [n for n in names if n not in CANDIDATES]
    if unknown:
        ap.error(f"unknown candidates {unknown}")
    res = race(names, args.nproc, args.backend, args.device, args.iters, args.reps, args.warmup, args.timeout)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)
    if args.env_out and "winner" in res:
        w = res["winner"]
        with open(args.env_out, "w") as f:
            if args.nproc < 2:
                # one rank: the all-reduce is a local copy, so the ranking is noise -- such a file
                # must not pin NCCL_PROTO/NCCL_ALGO for multi-GPU jobs; only the base set is written
                print("rccl_tune: --nproc < 2, the winner is not a measurement; --env-out gets the "
                      "base environment only", file=sys.stderr)
                f.write(f"# tools/rccl_tune.py at {res['nproc']} rank: no protocol measured, base environment only\n")
                env = dict(BASE_ENV)
            else:
                f.write(f"# tools/rccl_tune.py winner {w['name']} ({w['step_us']} us per step, {res['nproc']} ranks)\n")
                env = {**BASE_ENV, **w["env"]}
            for k, v in sorted(env.items()):
                f.write(f"{k}={v}\n")
    print(json.dumps(res.get("winner", {"error": "no candidate ran"})))
    return 0 if "winner" in res else 1


if __name__ == "__main__":
    sys.exit(main())
