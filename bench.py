#!/usr/bin/env python3
"""Headline benchmark: MNIST DDP training samples/sec on MI355X.

Metric/config from BASELINE.json: the reference's MNIST DDP workload
(jiaqianjing/pytorch-operator examples/mnist/mnist.py -- Net, batch 64 per rank,
SGD(lr=0.01, momentum=0.5), fp32, every rank iterating its own data, gradients
averaged by DDP all-reduce) on 1/2/4/8 MI355X, one process per GPU over RCCL.

Each timed step is a complete training step: batch gather + normalisation,
forward, NLL loss, backward, gradient all-reduce (world > 1) and the SGD update.
Data is synthetic (a learnable MNIST-shaped dataset resident in HBM), weights are
random-init (torch.manual_seed + the reference's default init).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--kernels hip|torch]
    torchrun --nproc-per-node N bench.py --gpus N ...   (N > 1)

``python bench.py --gpus N`` with N > 1 and no launcher (no ``WORLD_SIZE`` in the env) starts
the N ranks itself: before importing torch or touching HIP it runs ``torch.distributed.run
--nproc-per-node N`` as a CHILD process (never an exec), relays rank 0's line and exits with
the child's code.  A realised world size that differs from ``--gpus`` is an error (exit 2),
never a warning.

Rank 0 prints ONE JSON line.  ``value`` is the whole-job samples/s (sum over
ranks), timed as the MAX over ranks of K steps bracketed by barrier+synchronize.
``world_size`` is the process group's size and ``rccl_nranks`` the rank count RCCL's own
communicator reports (``ncclCommCount``; null unless the group runs on RCCL).
``vs_baseline`` divides by 210 samples/s/rank x N: the reference's derived
per-rank throughput (>= 210 samples/s/rank, 420 aggregate at 2 ranks).
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import signal
import subprocess
import sys
import time

BASELINE_PER_RANK = 210.0

# Kernel arguments in device memory -- this image's default; with them in host memory every
# dependent launch of the step waits on the host read: 43.61-43.83 instead of 35.30-35.37 us/step
# at K=2000 (profiles/r5_env/ab.txt).  Set before HIP initialises, unless the caller chose.
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")


def pick_steps_per_graph(steps: int, warmup: int = 0, cap: int = 250) -> int:
    """Whole training steps per hipGraph replay of the timed region: a divisor of ``steps``
    (so exactly ``steps`` steps are timed), at most ``cap``.  Preferred: the largest one not
    above ``warmup``, so the warm-up replays the timed graph itself -- a hipGraph's first
    launch is ~0.75 us per node slower than later ones (profiles/r2_launch_overhead.json),
    while back-to-back launches of a warm graph cost no more than one big graph."""
    divs = [d for d in range(1, min(steps, cap) + 1) if steps % d == 0]
    warm = [d for d in divs if d <= warmup]
    return max(warm) if warm else max(divs)


def parse_args(argv=None):
    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=2000)
    p.add_argument("--warmup", type=int, default=50)
    p.add_argument("--batch-size", type=int, default=64)
    p.add_argument("--kernels", choices=["hip", "torch"], default="hip")
    p.add_argument("--mode", choices=["eager", "graph", "graph-comm"], default="graph")
    p.add_argument("--launch", choices=["graph", "stream"], default="stream",
                   help="whole-step execution: replay the hipGraph, or launch the captured one-step "
                        "kernel list straight onto the stream from C++ (no per-replay graph-launch "
                        "gap, no first-launch cost; profiles/r2_k20_timeline.json)")
    p.add_argument("--steps-per-graph", type=int, default=0,
                   help="whole steps per hipGraph replay (world 1 only; 0 = auto)")
    p.add_argument("--dataset-size", type=int, default=60000)
    p.add_argument("--fuse-conv12", type=int, default=1)
    p.add_argument("--conv-chunk", type=int, default=4, choices=[1, 4],
                   help="conv backward: dW_conv2 per 4-sample chunk (slab 4x smaller) or per sample")
    p.add_argument("--stage", type=int, default=1, help="stage the next batch during fc1_bwd (1/0)")
    p.add_argument("--backend", default="nccl", choices=["nccl", "rccl", "gloo"],
                   help="collective backend (gloo only to rehearse the multi-rank path on one GPU)")
    p.add_argument("--allreduce", default="auto", choices=["auto", "xgmi", "rccl"],
                   help="DDP gradient path for world>1: xGMI peer-memory kernel fused with SGD "
                        "(self-tested at start-up, RCCL fallback) or RCCL all-reduce")
    p.add_argument("--force-collectives", type=int,
                   default=int(os.environ.get("PTO_FORCE_COLLECTIVES", "0") not in ("", "0")),
                   help="world 1: still build a (single-rank) process group and issue the two bucket "
                        "all-reduces every step, racing the RCCL step forms (their single-rank floor; "
                        "not the headline configuration)")
    p.add_argument("--json-out", default=None)
    p.add_argument("--job-latency", type=int, default=1,
                   help="after the timed region, run one PyTorchJob with one pod per GPU through "
                        "the native operator + local cluster and report create->first-step (1/0)")
    p.add_argument("--job-timeout", type=float, default=150.0)
    p.add_argument("--job-gpus", default="",
                   help="node GPU ids of the job's pods, comma-separated (default 0..N-1); repeated ids "
                        "let pods share a GPU (e.g. 0,0 on a 1-GPU box) and switch the job to gloo")
    p.add_argument("--job-backend", default="",
                   help="the job's torch.distributed backend (default rccl; gloo with shared GPUs)")
    p.add_argument("--prewarm-ms", type=int, default=40,
                   help="keep the GPU busy (FMA spin, no training state touched) this long before "
                        "the warm-up steps so the timed steps run at steady-state clocks "
                        "(profiles/r2_cold_start.json); 0 = off")
    return p.parse_args(argv)


SELF_LAUNCH_ENV = "PTO_BENCH_LAUNCHER"


def needs_self_launch(gpus: int, environ=None) -> bool:
    """True when this process must start the ``gpus`` ranks itself: more than one GPU asked
    for and no launcher (torchrun or the operator's pods) has set up a rank environment."""
    environ = os.environ if environ is None else environ
    return gpus > 1 and "WORLD_SIZE" not in environ


def launch_command(argv, gpus: int, port: int, script: str = None):
    """The ``torch.distributed.run`` command line of a self-launched N-rank bench: one process
    per GPU on this node, rendezvous on 127.0.0.1, the same bench arguments."""
    script = script or os.path.abspath(__file__)
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), script, *argv]


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def visible_gpu_count(timeout: float = 300.0) -> int:
    """GPUs this node exposes, counted in a child interpreter so that the launching process
    itself never loads HIP (``torch.cuda.device_count()`` does not initialise the device)."""
    r = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                       capture_output=True, text=True, timeout=timeout)
    try:
        return int(r.stdout.strip().splitlines()[-1])
    except (ValueError, IndexError):
        return 0


def check_line(line: dict, gpus: int):
    """None if rank 0's line describes a ``gpus``-rank run, else the reason it does not."""
    if line.get("n_gpus") != gpus or line.get("world_size") != gpus:
        return (f"asked for {gpus} ranks, the run reports n_gpus={line.get('n_gpus')} "
                f"world_size={line.get('world_size')}")
    if line.get("rccl_nranks") not in (None, gpus):
        return f"RCCL communicator has {line.get('rccl_nranks')} ranks, expected {gpus}"
    return None


def self_launch(args, argv, script: str = None) -> int:
    """Run the N-rank bench as a child ``torch.distributed.run`` job and relay its output.

    The parent never imports torch (the GPU count comes from a child interpreter), so no HIP
    state exists here when the ranks start.  Exit code: the job's, or 2 when RCCL is asked
    for more ranks than visible GPUs / the realised world differs from ``--gpus`` / rank 0
    printed no line."""
    if args.backend in ("nccl", "rccl"):
        n = visible_gpu_count()
        if n < args.gpus:
            print(f"error: --gpus {args.gpus} with --backend {args.backend} needs one GPU per rank; "
                  f"{n} visible (use --backend gloo to rehearse ranks sharing a GPU)", file=sys.stderr)
            return 2
    env = dict(os.environ, **{SELF_LAUNCH_ENV: "bench.py->torch.distributed.run"})
    env.setdefault("OMP_NUM_THREADS", "1")
    cmd = launch_command(argv, args.gpus, _free_port(), script)
    print("launching: " + " ".join(cmd[1:]), file=sys.stderr, flush=True)
    child = subprocess.Popen(cmd, stdout=subprocess.PIPE, env=env, text=True, bufsize=1)

    def _forward(signum, _frame):  # a timeout on the parent ends the ranks too
        child.send_signal(signum)
    prev = {s: signal.signal(s, _forward) for s in (signal.SIGTERM, signal.SIGINT)}
    line = None
    try:
        for raw in child.stdout:
            sys.stdout.write(raw)
            sys.stdout.flush()
            if raw.startswith('{"metric"'):
                line = json.loads(raw)
        rc = child.wait()
    finally:
        for s, h in prev.items():
            signal.signal(s, h)
    if rc != 0:
        return rc
    if line is None:
        print("error: rank 0 printed no result line", file=sys.stderr)
        return 2
    why = check_line(line, args.gpus)
    if why:
        print(f"error: {why}", file=sys.stderr)
        return 2
    return 0


def rccl_nranks():
    """Rank count of the default group's RCCL communicator (``ncclCommCount`` on the comm
    torch's ProcessGroupNCCL holds), from the librccl this process has loaded; None when the
    group is not on RCCL or the communicator is not exposed."""
    import ctypes
    import torch
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_backend() != "nccl":
        return None
    try:
        ptr = int(dist.group.WORLD._get_backend(torch.device("cuda"))._comm_ptr())
        path = None
        with open("/proc/self/maps") as f:
            for ln in f:
                if "librccl.so" in ln:
                    path = ln.split()[-1]
                    break
        if not ptr or path is None:
            return None
        lib = ctypes.CDLL(path)
        n = ctypes.c_int(-1)
        return int(n.value) if lib.ncclCommCount(ctypes.c_void_p(ptr), ctypes.byref(n)) == 0 else None
    except Exception:  # noqa: BLE001 -- a missing accessor leaves the field null
        return None


def job_gpu_plan(world: int, job_gpus: str, job_backend: str):
    """(node GPU ids, backend) of the bench's PyTorchJob: one pod per GPU over RCCL unless
    ``job_gpus`` repeats an id (pods sharing a device need gloo: RCCL wants one GPU per rank)."""
    gpus = [int(g) for g in job_gpus.split(",") if g.strip()] if job_gpus else list(range(world))
    if len(gpus) != world:
        raise ValueError(f"--job-gpus lists {len(gpus)} ids for {world} replicas")
    backend = job_backend or ("gloo" if len(set(gpus)) < len(gpus) else "rccl")
    return gpus, backend


def job_latency(world: int, rank: int, timeout: float, gpus=None, backend: str = "rccl",
                extra_args=()) -> dict:
    """create->first-step / create->Succeeded of a real job (BASELINE's second metric):
    fake API server -> pytorch-operator binary -> kubelet emulator -> ``world`` worker pods,
    each pinned to one GPU (HIP_VISIBLE_DEVICES narrowed like the amd.com/gpu plugin).
    Rank 0 drives it; other ranks wait on the rendezvous store (no GPU work meanwhile)."""
    import torch.distributed as dist
    store = dist.distributed_c10d._get_default_store() if world > 1 else None
    out = {}
    if rank == 0:
        try:
            sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "benchmarks"))
            from job_latency import measure
            r = measure(world, gpus=list(gpus) if gpus else list(range(world)), backend=backend,
                        timeout=timeout, extra_args=tuple(extra_args))
            out = {"create_to_first_step_s": r["create_to_first_step_s"],
                   "create_to_running_s": r["create_to_running_s"],
                   "create_to_succeeded_s": r["create_to_succeeded_s"],
                   "job": {"replicas": r["replicas"], "result": r["result"],
                           "gpus_per_pod": 1, "node_gpus": list(gpus) if gpus else list(range(world)),
                           "backend": backend, "grad_allreduce": r["grad_allreduce"],
                           "worker_samples_per_sec": r["worker_samples_per_sec"],
                           "worker_step_ms": r.get("worker_step_ms"),
                           "worker_train_seconds": r.get("worker_train_seconds"),
                           "worker_capture_seconds": r.get("worker_capture_seconds"),
                           "pod_topology": r.get("pod_topology"),
                           "startup_breakdown": r.get("startup_breakdown"),
                           "allreduce_trial": r.get("allreduce_trial"),
                           "reference_create_to_running_s": 121.0}}
        except Exception as e:  # noqa: BLE001 -- never lose the throughput line over this
            out = {"create_to_first_step_s": None, "create_to_succeeded_s": None,
                   "job": {"error": repr(e)[:300]}}
        if store is not None:
            store.set("pto_bench_job_latency", "done")
    elif store is not None:
        from datetime import timedelta
        store.wait(["pto_bench_job_latency"], timedelta(seconds=timeout + 120))
    return out


def prewarm(ms: int, dev) -> None:
    """Sustained GPU activity before the warm-up: a short timed region right after idle pays
    the power-management clock ramp (~4 % at K=20 on MI355X, profiles/r2_cold_start.json)."""
    if ms <= 0:
        return
    import torch
    from pytorch_operator_amd.ops import _native
    sink = torch.empty(256, device=dev)
    _native.check(_native.load().pto_device_prewarm(int(ms * 1000), sink.data_ptr(),
                                                    torch.cuda.current_stream(dev).cuda_stream),
                  "device_prewarm")
    torch.cuda.synchronize(dev)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    args = parse_args(argv)
    if needs_self_launch(args.gpus):
        return self_launch(args, argv)
    launcher_world = int(os.environ.get("WORLD_SIZE", "1"))
    if launcher_world != args.gpus:  # decided before any process group or GPU work
        print(f"error: --gpus {args.gpus} but the launcher's WORLD_SIZE is {launcher_world}",
              file=sys.stderr)
        return 2
    import torch
    import torch.distributed as dist

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from pytorch_operator_amd.parallel.dist import init_from_env

    force = bool(args.force_collectives) and args.kernels == "hip"
    env = init_from_env(args.backend, use_gpu=True, force_pg=force)
    world, rank, dev = env.world_size, env.rank, env.device
    pg = dist.is_initialized()  # world > 1, or a forced single-rank group
    pg_world = dist.get_world_size() if pg else 1
    if pg_world != args.gpus:
        print(f"error: --gpus {args.gpus} but the process group has {pg_world} ranks", file=sys.stderr)
        return 2
    B = args.batch_size
    job_plan = job_gpu_plan(world, args.job_gpus, args.job_backend)  # validated before any work

    from pytorch_operator_amd.data.synthetic import make_synthetic_mnist
    ds = make_synthetic_mnist(args.dataset_size, seed=1 + rank, device=dev)

    xgmi_note = []  # why the xGMI gradient path is not used (try_xgmi's log), for the JSON line
    if args.kernels == "hip":
        from pytorch_operator_amd.models.mnist import FusedMnistTrainer
        from pytorch_operator_amd.ops import mnist as K
        from pytorch_operator_amd.parallel.graphed_step import GraphedStep
        cursor = torch.zeros(1, dtype=torch.int32, device=dev)
        src = K.BatchSource(ds.images, ds.labels, perm=ds.perm, cursor=cursor)
        sync, xg, ar_path = None, None, "none"
        if world > 1 or force:
            from pytorch_operator_amd.models.mnist import flat_layout
            from pytorch_operator_amd.parallel.ddp import FlatGradAllReduce
            from pytorch_operator_amd.parallel.xgmi import try_xgmi
            sync, ar_path = FlatGradAllReduce(force=force), "rccl"
            if args.allreduce != "rccl" and world > 1:
                def xgmi_log(m):  # why the xGMI path is not used, kept for the JSON line too
                    xgmi_note.append(str(m)[:1200])
                    if rank == 0:
                        print(m, file=sys.stderr)
                xg = try_xgmi(flat_layout().total, dev, required=args.allreduce == "xgmi", log=xgmi_log)
        tr = FusedMnistTrainer(batch_size=B, source=src, lr=0.01, momentum=0.5, device=dev,
                               seed=1, grad_sync=sync)
        tr.fuse_conv12 = bool(args.fuse_conv12)
        tr.conv_chunk = args.conv_chunk
        tr.stage_batches = bool(args.stage)
        if world > 1:  # DDP constructor semantics: start from rank 0's parameters
            dist.broadcast(tr.flat_params, 0)
        spg = args.steps_per_graph if args.steps_per_graph > 0 else pick_steps_per_graph(args.steps, args.warmup)
        done_w = 0
        tune = None
        if (xg is not None or (force and sync is not None)) and args.allreduce == "auto" and \
                args.mode != "eager":
            # measured choice between the RCCL forms and the xGMI kernel (the trials are warm-up
            # steps; forced at world 1 only the two RCCL forms race)
            from pytorch_operator_amd.parallel.autotune import choose_grad_sync
            tr.train_step()  # momentum initialisation + library load, outside any graph
            done_w = 1
            runner, ar_path, tune = choose_grad_sync(tr, sync, xg, mode=args.mode, spg=spg, trial_steps=40,
                                                     launch=args.launch)
            done_w += tune.pop("steps")
        elif xg is not None:
            tr.grad_sync, ar_path = xg, "xgmi"
            runner = GraphedStep(tr, mode="graph" if args.mode != "eager" else "eager", steps_per_graph=spg,
                                 launch=args.launch)
        else:
            runner = GraphedStep(tr, mode=args.mode, steps_per_graph=spg, launch=args.launch)
        prewarm(args.prewarm_ms, dev)
        runner.warm(max(0, args.warmup - done_w - runner.internal_steps))

        def run(n):
            runner.run(n)
        steps = args.steps - args.steps % runner.steps_per_graph
        xgmi_error = (lambda: xg.xar.error()) if xg is not None else (lambda: 0)
        mode_desc = (f"{args.mode}(launch={runner.launch},spg={runner.steps_per_graph},"
                     f"allreduce={ar_path},conv_chunk={args.conv_chunk},stage={args.stage})")
    else:
        from pytorch_operator_amd.models.mnist import Net
        import torch.nn.functional as F
        torch.manual_seed(1)
        model = Net().to(dev)
        if world > 1:
            model = torch.nn.parallel.DistributedDataParallel(model, device_ids=[dev.index])
        opt = torch.optim.SGD(model.parameters(), lr=0.01, momentum=0.5)
        xf = ds.float_images()
        lab = ds.labels.long()
        state = {"i": 0}

        def run(n):
            for _ in range(n):
                i = state["i"]
                idx = ds.perm[(i * B) % ds.n: (i * B) % ds.n + B].long()
                state["i"] = i + 1
                opt.zero_grad(set_to_none=True)
                loss = F.nll_loss(model(xf[idx]), lab[idx])
                loss.backward()
                opt.step()
        prewarm(args.prewarm_ms, dev)
        run(args.warmup)
        steps = args.steps
        mode_desc = "torch-eager"
        ar_path, tune = "ddp", None
        xgmi_error = lambda: 0  # noqa: E731

    # no garbage-collector pass inside the timed region (as timeit does): after torch's imports an
    # automatic generation-0 / -1 collection stalls the host 0.2 / 1.5 ms (measured on the CPU),
    # 10-75 us per step at the driver's K = 20 once the GPU drains the queued launches.  No explicit
    # collection here: its ~90 ms of GPU idle right before the region lets the clocks drop (K = 20
    # measured 39.5-40.0 instead of 35.9-36.1 us, profiles/r6_twostream/gc_collect_k20.txt)
    gc.disable()
    torch.cuda.synchronize(dev)
    if pg:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    run(steps)
    torch.cuda.synchronize(dev)
    if pg:  # every rank's GPU work done, then the barrier, then this rank's device once more
        dist.barrier()
        torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    gc.enable()
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    # a bounded wait that timed out inside the xGMI kernel means the replicas went rank-local:
    # the number above is then not a DDP result (reported, and the exit code is 138)
    ar_err = int(xgmi_error()) if ar_path.startswith("xgmi") else 0  # both DDP forms (xgmi, xgmi-r5)
    in_sync = None
    if world > 1:
        # DDP invariant (checked after the timed region): every replica holds rank 0's weights
        flat = tr.flat_params if args.kernels == "hip" else torch.cat(
            [q.detach().reshape(-1) for q in model.parameters()])
        ref = flat.clone()
        dist.broadcast(ref, 0)
        diff = (flat - ref).abs().max().reshape(1)
        dist.all_reduce(diff, op=dist.ReduceOp.MAX)
        in_sync = bool(float(diff.item()) == 0.0) and ar_err == 0
    nranks = rccl_nranks()

    # a forced-collectives bench forces them in the job's pods too (their race lands in job.allreduce_trial)
    lat = job_latency(world, rank, args.job_timeout, *job_plan,
                      extra_args=("--force-collectives", "1") if force else ()) if args.job_latency else {}

    samples = steps * B * world
    value = samples / dt
    result = {
        "metric": "mnist_ddp_train_samples_per_sec",
        "value": round(value, 1),
        "unit": "samples/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / steps * 1e3, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(value / (BASELINE_PER_RANK * world), 1),
        "world_size": pg_world,
        "rccl_nranks": nranks,
        "launcher": os.environ.get(SELF_LAUNCH_ENV) or ("external" if "WORLD_SIZE" in os.environ else "none"),
        "replicas_in_sync": in_sync,
        "grad_allreduce_error": ar_err,
        "device_prewarm_ms": args.prewarm_ms,
        **lat,
        "dtype": "fp32",
        "data": "synthetic (learnable MNIST-shaped uint8 images in HBM), random-init weights",
        "config": {
            "model": "mnist-cnn (reference examples/mnist/mnist.py Net: conv20-conv50-fc500-fc10)",
            "global_batch": B * world,
            "per_rank_batch": B,
            "seq_len": None,
            "parallelism": f"dp{world}",
            "optimizer": "SGD(lr=0.01, momentum=0.5)",
            "kernels": args.kernels,
            "exec": mode_desc,
            "backend": ("rccl" if env.backend == "nccl" else env.backend) if pg else "none",
            "grad_allreduce": ar_path,
            "forced_collectives": force,
            "allreduce_trial": tune,
            "xgmi_note": "; ".join(xgmi_note) or None,
        },
    }
    if rank == 0:
        line = json.dumps(result)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    if pg:
        dist.barrier()
        dist.destroy_process_group()
    return 138 if ar_err else 0


if __name__ == "__main__":
    sys.exit(main())
