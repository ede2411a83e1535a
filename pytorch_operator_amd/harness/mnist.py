"""The PyTorchJob MNIST DDP worker (the container entrypoint of the example jobs).

Behavioural parity with the reference worker examples/mnist/mnist.py:

* same CLI (``--batch-size 64 --test-batch-size 1000 --epochs 1 --lr 0.01
  --momentum 0.5 --no-cuda --seed 1 --log-interval 10 --save-model --dir logs
  --backend``), same model (``models.mnist.Net``), SGD(lr, momentum), NLL loss;
* process group from the operator's env contract (MASTER_ADDR/MASTER_PORT/WORLD_SIZE/
  RANK, mnist.py:82-116) when WORLD_SIZE > 1;
* the same stdout lines (``Train Epoch: e [n/N (p%)]\\tloss=x`` every log interval,
  ``accuracy=x`` after each epoch's test pass) and TensorBoard scalars ``loss`` /
  ``accuracy`` under ``--dir``.

MI355X-native differences:

* ``--backend rccl`` (alias of nccl: RCCL over xGMI); ``mpi`` fails clearly;
* on a GPU the step runs the fused gfx950 kernels (``--kernels hip``, default) on an
  HBM-resident uint8 dataset, replayed as hipGraphs; DDP gradients go through whichever of
  the xGMI peer-memory all-reduce fused with SGD (``parallel/xgmi.py``, after its start-up
  self-test), two stream-launched flat-bucket RCCL all-reduces, or one hipGraph per step with
  the RCCL collectives captured wins a timed start-up race (``parallel/autotune.py``, the same
  race ``bench.py`` runs).  ``--kernels torch`` is the plain PyTorch path (also used on CPU with
  gloo);
* data: real MNIST IDX files from ``--data-dir`` if present, else the synthetic set
  (no network); by default every rank iterates the full dataset like the reference
  (quirk Q8: no DistributedSampler); ``--shard`` gives each rank a disjoint slice like a
  ``DistributedSampler``;
* one machine-readable JSON line per milestone (``first_step``, ``train_done``) so the
  operator benchmarks can measure create-to-first-step latency and throughput.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time
from typing import Optional

_T_MODULE = time.time_ns()  # worker entry when run as ``python -m pytorch_operator_amd.harness.mnist``

# Kernel arguments in device memory, pinned before anything can initialise HIP (the same pin as
# bench.py; host-memory kernargs cost +8.3 us per MNIST step, profiles/r5_env/ab.txt).  The
# operator also injects it into the pod (--inject-rccl-env); a value the environment sets wins.
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")


def parse_args(argv=None):
    p = argparse.ArgumentParser(description="PyTorch MNIST Example (MI355X-native worker)")
    p.add_argument("--batch-size", type=int, default=64, metavar="N")
    p.add_argument("--test-batch-size", type=int, default=1000, metavar="N")
    p.add_argument("--epochs", type=int, default=1, metavar="N")
    p.add_argument("--lr", type=float, default=0.01, metavar="LR")
    p.add_argument("--momentum", type=float, default=0.5, metavar="M")
    p.add_argument("--no-cuda", action="store_true", default=False)
    p.add_argument("--seed", type=int, default=1, metavar="S")
    p.add_argument("--log-interval", type=int, default=10, metavar="N")
    p.add_argument("--save-model", action="store_true", default=False)
    p.add_argument("--dir", default="logs", metavar="L", help="TensorBoard summary directory")
    p.add_argument("--backend", type=str, default="gloo", choices=["gloo", "nccl", "rccl", "mpi"])
    # MI355X-native extensions
    p.add_argument("--kernels", choices=["auto", "hip", "torch"], default="auto")
    p.add_argument("--data-dir", default="../data", help="directory holding MNIST IDX files")
    p.add_argument("--synthetic", action="store_true", help="force the synthetic dataset")
    p.add_argument("--dataset-size", type=int, default=60000, help="synthetic train set size")
    p.add_argument("--test-size", type=int, default=10000, help="synthetic test set size")
    # reference semantics (quirk Q8): no DistributedSampler, every rank walks the full set
    p.add_argument("--shard", dest="shard", action="store_true", default=False,
                   help="give each rank a disjoint 1/W slice (DistributedSampler semantics)")
    p.add_argument("--no-shard", dest="shard", action="store_false")
    p.add_argument("--max-steps", type=int, default=0, help="cap steps per epoch (0 = full epoch)")
    p.add_argument("--no-graph", action="store_true", help="HIP path: eager launches, no hipGraphs")
    p.add_argument("--launch", choices=["graph", "stream"], default="stream",
                   help="HIP path: replay log-interval hipGraphs, or launch the captured one-step kernel "
                        "list from C++ onto the stream (no per-replay graph-launch gap)")
    p.add_argument("--allreduce", choices=["auto", "xgmi", "rccl"], default="auto",
                   help="HIP path, world>1: auto = time the xGMI peer-memory all-reduce fused with SGD "
                        "(self-tested) against RCCL at start-up and keep the faster (parallel/autotune.py); "
                        "xgmi / rccl force one")
    p.add_argument("--force-collectives", type=int,
                   default=int(os.environ.get("PTO_FORCE_COLLECTIVES", "0") not in ("", "0")),
                   help="HIP path, world 1: build a single-rank process group anyway and issue the "
                        "gradient all-reduces every step (--allreduce auto then races the RCCL step "
                        "forms); env PTO_FORCE_COLLECTIVES")
    p.add_argument("--race-steps", type=int, default=40,
                   help="training steps each candidate of the --allreduce auto race runs (the state is "
                        "restored afterwards: the race does not change the trajectory)")
    p.add_argument("--xgmi-timeout", type=float, default=5.0,
                   help="bounded wait (s) inside the xGMI exchange before it flags an error; an error "
                        "ends the worker with the retryable exit code 138")
    p.add_argument("--model-path", default="mnist_cnn.pt")
    p.add_argument("--checkpoint-dir", default=None,
                   help="write an end-of-epoch checkpoint (weights + optimizer state) here")
    p.add_argument("--resume", action="store_true",
                   help="continue from --checkpoint-dir if a checkpoint exists (e.g. after an ExitCode restart)")
    p.add_argument("--trace", action="store_true", help="roctx ranges around epochs, step blocks and eval")
    p.add_argument("--metrics-file", default=None, help="append the JSON milestone lines here too")
    p.add_argument("--metrics-port", type=int, default=int(os.environ.get("PTO_WORKER_METRICS_PORT", "-1")),
                   help="serve Prometheus /metrics on this port (0: any free port, -1: off; "
                        "docs/monitoring.md; env PTO_WORKER_METRICS_PORT)")
    return p.parse_args(argv)


class _Emitter:
    """JSON milestone lines (stdout + ``--metrics-file``), mirrored into the worker's Prometheus
    endpoint when ``--metrics-port`` is on (``wm``)."""

    def __init__(self, rank: int, path, wm=None):
        self.rank, self.path, self.wm = rank, path, wm
        self.info = {"rank": rank}

    def __call__(self, event: str, **kw):
        rec = {"event": event, "rank": self.rank, "unix_ns": time.time_ns(), **kw}
        line = json.dumps(rec)
        print(line, flush=True)
        if self.path:
            with open(self.path, "a") as f:
                f.write(line + "\n")
        if self.wm is not None:
            if event == "first_step":
                self.wm.set("pto_worker_first_step_unix_seconds", rec["unix_ns"] / 1e9)
            elif event == "startup":
                for k, v in kw["phases"].items():
                    self.wm.set("pto_worker_startup_phase_seconds", v, phase=k[:-2] if k.endswith("_s") else k)
            elif event == "grad_allreduce":
                self.info["grad_allreduce"] = kw.get("path", "")
                self.wm.set("pto_worker_info", 1, replace=True, **self.info)
                for k, v in (kw.get("trial") or {}).items():
                    if k.endswith("_ms_per_step") and v is not None:
                        self.wm.set("pto_worker_allreduce_trial_ms", v, candidate=k[:-len("_ms_per_step")])
            elif event == "xgmi_error":
                self.wm.set("pto_worker_grad_exchange_errors", kw.get("code", 1))
            elif event == "train_done" and kw.get("accuracy") is not None:
                self.wm.set("pto_worker_accuracy", kw["accuracy"])


def _datasets(args, rank: int, world: int, device):
    import torch
    from ..data.mnist_idx import load_mnist
    from ..data.synthetic import make_synthetic_mnist
    train = test = None
    if not args.synthetic:
        train = load_mnist(args.data_dir, "train")
        test = load_mnist(args.data_dir, "test")
    source = "mnist-idx"
    if train is None or test is None:
        source = "synthetic"
        # on a GPU the set is drawn on the device (ms, not the ~1-2 s of single-threaded CPU
        # warps: the biggest piece of a pod's start-up, profiles/r4_startup.md)
        gpu = device is not None and torch.device(device).type == "cuda"
        tr = make_synthetic_mnist(args.dataset_size, seed=args.seed, device=device if gpu else None, on_device=gpu)
        te = make_synthetic_mnist(args.test_size, seed=args.seed + 7919, device=device if gpu else None,
                                  on_device=gpu)
        train, test = (tr.images, tr.labels), (te.images, te.labels)
    xtr, ytr = train
    if args.shard and world > 1:
        xtr, ytr = xtr[rank::world].contiguous(), ytr[rank::world].contiguous()
    return (xtr.to(device), ytr.to(device)), (test[0].to(device), test[1].to(device)), source


def _epoch_perm(n: int, seed: int, epoch: int, rank: int, shard: bool, device):
    import torch
    # reference: DataLoader(shuffle=True) under torch.manual_seed(seed) -- identical order
    # on every rank.  Sharded runs shuffle their own slice.
    g = torch.Generator(device="cpu").manual_seed(seed * 1000003 + epoch * 7 + (rank if shard else 0))
    return torch.randperm(n, generator=g).to(torch.int32).to(device)


def _proc_start_ns() -> Optional[int]:
    """Wall-clock start of this process: now minus its age, the age from /proc/self/stat's
    starttime against /proc/uptime (both since boot, 10 ms ticks).  /proc/stat's integer
    ``btime`` is not used: its truncation put the start up to 1 s late."""
    try:
        now = time.time_ns()
        with open("/proc/self/stat") as f:
            ticks = int(f.read().rsplit(")", 1)[1].split()[19])
        with open("/proc/uptime") as f:
            up = float(f.read().split()[0])
        age = up - ticks / os.sysconf("SC_CLK_TCK")
        return int(now - max(age, 0.0) * 1e9)
    except (OSError, ValueError, IndexError):
        return None


class _Startup:
    """Wall-clock milestones from process start to the first optimizer step (the pieces of
    BASELINE's create-to-first-step latency that run inside the pod); emitted as one
    ``startup`` event with absolute ``unix_ns`` stamps and per-phase seconds."""

    def __init__(self, t_main_ns: Optional[int]):
        self.marks = [("process_start", _proc_start_ns()), ("worker_main", t_main_ns)]

    def mark(self, name: str) -> None:
        self.marks.append((name, time.time_ns()))

    def record(self) -> dict:
        marks = [(k, t) for k, t in self.marks if t is not None]
        phases = {f"{k}_s": round((t - marks[i - 1][1]) / 1e9, 4) for i, (k, t) in enumerate(marks) if i}
        return {"marks_unix_ns": dict(marks), "phases": phases}


def run(args, t_main_ns: Optional[int] = None) -> dict:
    startup = _Startup(t_main_ns)
    import torch
    import torch.nn.functional as F
    from ..parallel.dist import init_from_env
    startup.mark("import_torch")

    use_cuda = not args.no_cuda and torch.cuda.is_available()
    if use_cuda:
        print("Using CUDA")  # reference wording; the device is an MI355X over HIP
        torch.cuda.init()
        startup.mark("hip_init")
    torch.manual_seed(args.seed)
    kernels = args.kernels
    if kernels == "auto":
        kernels = "hip" if use_cuda else "torch"
    # forced collectives (HIP path): a single-rank group at world 1, all-reduces issued anyway
    args.force_collectives = bool(args.force_collectives) and kernels == "hip"
    env = init_from_env(args.backend, use_gpu=use_cuda, force_pg=args.force_collectives)
    rank, world, device = env.rank, env.world_size, env.device
    startup.mark("process_group")
    wm = None
    if args.metrics_port >= 0:
        from ..utils.worker_metrics import WorkerMetrics
        wm = WorkerMetrics()
        port = wm.serve(args.metrics_port)
    emit = _Emitter(rank, args.metrics_file, wm)
    if wm is not None:
        emit("metrics_endpoint", port=port)
    if world > 1:
        print(f"Using distributed PyTorch with {args.backend} backend")
    if kernels == "hip" and not use_cuda:
        raise SystemExit("--kernels hip needs a GPU (drop --no-cuda or use --kernels torch)")

    from ..utils.tb_writer import SummaryWriter
    writer = SummaryWriter(args.dir)
    if kernels == "hip":
        from ..ops import _native
        _native.load()
        startup.mark("hip_library")
    (xtr, ytr), (xte, yte), data_source = _datasets(args, rank, world, device)
    startup.mark("dataset")
    n = xtr.shape[0]
    B = args.batch_size
    steps_per_epoch = math.ceil(n / B)
    if args.max_steps:
        steps_per_epoch = min(steps_per_epoch, args.max_steps)
    emit("start", world_size=world, backend=env.backend, kernels=kernels, data=data_source,
         n_train=int(n), steps_per_epoch=steps_per_epoch)
    if wm is not None:
        emit.info.update(world_size=world, backend=env.backend, kernels=kernels)
        wm.set("pto_worker_info", 1, replace=True, **emit.info)

    if kernels == "hip":
        result = _train_hip(args, env, writer, emit, xtr, ytr, xte, yte, steps_per_epoch, startup)
    else:
        result = _train_torch(args, env, writer, emit, xtr, ytr, xte, yte, steps_per_epoch, startup)
    writer.close()
    emit("train_done", **result)
    import torch.distributed as dist
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()
    return result


class _Trace:
    """roctx ranges (torch.cuda.nvtx maps to roctx on ROCm builds) when --trace is given."""

    def __init__(self, on: bool):
        self.on = False
        if on:
            try:
                import torch.cuda.nvtx as nvtx
                nvtx.range_push("probe")
                nvtx.range_pop()
                self.nvtx, self.on = nvtx, True
            except Exception:  # noqa: BLE001 -- tracing is best effort
                self.on = False

    def __call__(self, name):
        import contextlib
        if not self.on:
            return contextlib.nullcontext()

        @contextlib.contextmanager
        def rng():
            self.nvtx.range_push(name)
            try:
                yield
            finally:
                self.nvtx.range_pop()
        return rng()


XGMI_FAILED_EXIT = 138  # SIGUSR1-class retryable code (tf-operator train_util.go:18-53)


def _xgmi_guard(sync, emit, where: str) -> None:
    """Fail fast when the fused xGMI exchange timed out: its kernel then falls back to a
    rank-local SGD and the replicas diverge silently.  Exiting with a retryable code hands
    the failure to the operator (ExitCode / OnFailure restart, ``--resume``)."""
    if not getattr(sync, "fused_sgd", False):
        return
    code = sync.xar.error()
    if code:
        emit("xgmi_error", code=int(code), where=where)
        print(f"xGMI gradient exchange failed (error {code}) at {where}; "
              f"exiting with retryable code {XGMI_FAILED_EXIT}", flush=True)
        os._exit(XGMI_FAILED_EXIT)


def _maybe_stall(rank: int, block: int) -> None:
    """Fault-injection hook: PTO_FAULT_STALL="rank:block:seconds" makes that rank sleep on
    the host before step block ``block`` (its peers' bounded xGMI waits then time out)."""
    spec = os.environ.get("PTO_FAULT_STALL")
    if spec:
        r, b, sec = spec.split(":")
        if int(r) == rank and int(b) == block:
            print(f"fault injection: rank {rank} stalls {sec}s before block {block}", flush=True)
            time.sleep(float(sec))


def _ckpt_path(args):
    return os.path.join(args.checkpoint_dir, "ckpt.pt") if args.checkpoint_dir else None


def _save_ckpt(args, rank, state: dict) -> None:
    """Rank 0 writes atomically (tmp + rename) so a crash never leaves a torn file."""
    import torch
    path = _ckpt_path(args)
    if not path or rank != 0:
        return
    os.makedirs(args.checkpoint_dir, exist_ok=True)
    tmp = path + f".tmp{os.getpid()}"
    torch.save(state, tmp)
    os.replace(tmp, path)


def _maybe_fault(epoch: int, resumed: bool) -> None:
    """Fault-injection hook for recovery tests: PTO_FAULT_EXIT_AFTER_EPOCH=N makes a
    fresh (non-resumed) run exit with PTO_FAULT_EXIT_CODE (default 137, a retryable SIGKILL
    code; 138 is what a failed xGMI exchange exits with) right after it checkpointed epoch N."""
    n = os.environ.get("PTO_FAULT_EXIT_AFTER_EPOCH")
    if n and not resumed and epoch == int(n):
        code = int(os.environ.get("PTO_FAULT_EXIT_CODE", "137"))
        print(f"fault injection: exiting with {code} after epoch {epoch}", flush=True)
        os._exit(code)


def _load_ckpt(args):
    import torch
    path = _ckpt_path(args)
    if not (args.resume and path and os.path.exists(path)):
        return None
    return torch.load(path, map_location="cpu", weights_only=True)


def _percentiles(samples_ms):
    if not samples_ms:
        return None
    xs = sorted(samples_ms)
    pick = lambda q: round(xs[min(len(xs) - 1, int(q * (len(xs) - 1) + 0.5))], 5)  # noqa: E731
    return {"p50": pick(0.5), "p90": pick(0.9), "p99": pick(0.99), "n": len(xs)}


def _log_train(epoch, batch_idx, B, n, steps_per_epoch, loss, writer, wm=None):
    print("Train Epoch: {} [{}/{} ({:.0f}%)]\tloss={:.4f}".format(
        epoch, batch_idx * B, n, 100.0 * batch_idx / steps_per_epoch, loss), flush=True)
    writer.add_scalar("loss", loss, epoch * steps_per_epoch + batch_idx)
    if wm is not None:
        wm.set("pto_worker_loss", loss)


def _log_test(acc, epoch, writer):
    print("\naccuracy={:.4f}\n".format(acc), flush=True)
    writer.add_scalar("accuracy", acc, epoch)
    writer.flush()


def _train_hip(args, env, writer, emit, xtr, ytr, xte, yte, steps_per_epoch, startup) -> dict:
    import torch
    import torch.distributed as dist
    from ..models.mnist import FusedMnistTrainer
    from ..ops import mnist as K
    from ..parallel.ddp import FlatGradAllReduce
    from ..parallel.graphed_step import GraphedStep

    dev, world, rank = env.device, env.world_size, env.rank
    B, n = args.batch_size, xtr.shape[0]
    perm = _epoch_perm(n, args.seed, 1, rank, args.shard, dev)
    cursor = torch.zeros(1, dtype=torch.int32, device=dev)
    src = K.BatchSource(xtr, ytr, perm=perm, cursor=cursor)
    sync = xg = rccl = None
    race = False
    forced = bool(getattr(args, "force_collectives", False))
    if world > 1 or forced:
        from ..models.mnist import flat_layout
        from ..parallel.xgmi import try_xgmi
        rccl = FlatGradAllReduce(force=forced)
        xg = try_xgmi(flat_layout().total, dev, required=args.allreduce == "xgmi",
                      timeout_s=args.xgmi_timeout) if args.allreduce != "rccl" and world > 1 else None
        sync = xg or rccl
        # forced at world 1 there is no xGMI candidate: the two RCCL forms race
        race = (xg is not None or forced) and args.allreduce == "auto" and not args.no_graph
        if not race:
            emit("grad_allreduce", path="xgmi" if xg is not None else "rccl")
        startup.mark("grad_sync")
    tr = FusedMnistTrainer(batch_size=B, source=src, lr=args.lr, momentum=args.momentum,
                           device=dev, seed=args.seed, grad_sync=sync)
    startup.mark("trainer")
    trace = _Trace(args.trace)
    start_epoch = 1
    ck = _load_ckpt(args) if rank == 0 else None
    if world > 1:
        flag = [ck["epoch"] if ck is not None else 0]
        dist.broadcast_object_list(flag, 0)
        resumed_epoch = flag[0]
    else:
        resumed_epoch = ck["epoch"] if ck is not None else 0
    if ck is not None:
        tr.load_state_dict({k: v.to(dev) for k, v in ck["params"].items()})
        tr.flat_momentum.copy_(ck["momentum"].to(dev))
    if resumed_epoch:
        if world > 1:
            dist.broadcast(tr.flat_momentum, 0)
        tr._first_step = False
        start_epoch = resumed_epoch + 1
        emit("resumed", epoch=resumed_epoch)
    if world > 1:
        dist.broadcast(tr.flat_params, 0)  # DDP constructor semantics
    log_iv = max(1, args.log_interval)
    runner = None
    t_train = t_capture = 0.0
    steps_done = 0
    step_ms = []
    loss = acc = float("nan")
    for epoch in range(start_epoch, args.epochs + 1):
        if epoch > 1:
            perm.copy_(_epoch_perm(n, args.seed, epoch, rank, args.shard, dev))
        cursor.zero_()
        tr.invalidate_stage()  # a batch staged from the old permutation must not be reused
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        # batch 0: eager (initialises momentum on the first epoch), logged
        tr.train_step()
        if steps_done == 0:
            torch.cuda.synchronize(dev)
            startup.mark("first_step")
            emit("startup", **startup.record())
            emit("first_step")
        _log_train(epoch, 0, B, n, steps_per_epoch, tr.loss(), writer, emit.wm)
        if emit.wm is not None:
            emit.wm.inc("pto_worker_steps_total")
        if runner is None and not args.no_graph:
            # capturing runs warm-up steps: snapshot the state, capture, restore, so the
            # trajectory is exactly the eager one (a log block = one graph replay).  The
            # capture is one-off set-up: its time is reported apart from train_seconds.
            torch.cuda.synchronize(dev)
            t_cap0 = time.perf_counter()
            saved = (tr.flat_params.clone(), tr.flat_momentum.clone())
            if race:
                # the start-up race of bench.py: every candidate runs real DDP steps, the
                # fastest (MAX over ranks) is kept; the snapshot restore below undoes the steps
                from ..parallel.autotune import choose_grad_sync
                runner, path, trial = choose_grad_sync(tr, rccl, xg, spg=log_iv, trial_steps=args.race_steps,
                                                       launch=args.launch)
                sync = runner.sync
                emit("grad_allreduce", path=path, trial=trial)
            else:
                # one graph holds whole steps unless RCCL collectives sit between the pieces
                whole = sync is None or getattr(sync, "fused_sgd", False) or not getattr(sync, "active", True)
                runner = GraphedStep(tr, mode="graph", steps_per_graph=log_iv if whole else 1, launch=args.launch)
            tr.flat_params.copy_(saved[0])
            tr.flat_momentum.copy_(saved[1])
            if xg is not None and not getattr(sync, "fused_sgd", False):
                # step 0 ran the fused xGMI exchange (each rank kept only its momentum shard);
                # the RCCL step needs every rank's whole buffer
                xg.xar.gather_sharded_(tr.flat_momentum)
            cursor.fill_(1)
            torch.cuda.synchronize(dev)
            t_capture = time.perf_counter() - t_cap0
            t0 += t_capture
        # blocks of log_iv steps ending on a logged batch (batches 1..L, L+1..2L, ...)
        b = 1
        events = []
        with trace(f"epoch{epoch}"):
            while b < steps_per_epoch:
                chunk = min(log_iv, steps_per_epoch - b)
                _maybe_stall(rank, b // log_iv)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                with trace("steps"):
                    if runner is not None and chunk % runner.steps_per_graph == 0:
                        runner.run(chunk)
                    elif runner is not None:
                        runner.warm(chunk)  # the one-step graph covers an epoch's odd tail
                    else:
                        for _ in range(chunk):
                            tr.train_step()
                e1.record()
                events.append((e0, e1, chunk))
                b += chunk
                if emit.wm is not None:
                    emit.wm.inc("pto_worker_steps_total", chunk)
                if (b - 1) % log_iv == 0:
                    _log_train(epoch, b - 1, B, n, steps_per_epoch, tr.loss(), writer, emit.wm)
                    if emit.wm is not None:  # tr.loss() synchronised: the interval's events are done
                        sec = e0.elapsed_time(e1) / 1e3 / chunk
                        emit.wm.set("pto_worker_step_seconds", sec)
                        emit.wm.set("pto_worker_samples_per_second", B * world / sec)
                    _xgmi_guard(sync, emit, f"epoch {epoch} batch {b - 1}")
        torch.cuda.synchronize(dev)
        _xgmi_guard(sync, emit, f"end of epoch {epoch}")
        t_train += time.perf_counter() - t0
        step_ms += [e0.elapsed_time(e1) / c for e0, e1, c in events]
        steps_done += steps_per_epoch
        with trace("eval"):
            loss, acc = _evaluate_hip(tr, K, xte, yte, args.test_batch_size)
        _log_test(acc, epoch, writer)
        if args.checkpoint_dir:
            if getattr(sync, "fused_sgd", False):
                sync.xar.gather_sharded_(tr.flat_momentum)  # xGMI keeps only this rank's shard
            _save_ckpt(args, rank, {"epoch": epoch, "momentum": tr.flat_momentum.detach().cpu().clone(),
                                    "params": {k: v.detach().cpu().clone() for k, v in tr.state_dict().items()}})
        _maybe_fault(epoch, resumed_epoch > 0)
    if args.save_model and rank == 0:
        torch.save({k: v.detach().cpu().clone() for k, v in tr.state_dict().items()}, args.model_path)
    return {"steps": steps_done, "train_seconds": round(t_train, 4),
            "samples_per_sec": round(steps_done * B * world / t_train, 1) if t_train else None,
            "step_ms": _percentiles(step_ms), "capture_seconds": round(t_capture, 4),
            "test_loss": round(loss, 5), "accuracy": round(acc, 5)}


def _evaluate_hip(tr, K, xte, yte, batch_size):
    src = K.BatchSource(xte, yte)
    return tr.evaluate(src, batch_size=min(batch_size, xte.shape[0]))


def _train_torch(args, env, writer, emit, xtr, ytr, xte, yte, steps_per_epoch, startup) -> dict:
    import torch
    import torch.nn.functional as F
    from ..models.mnist import Net

    dev, world, rank = env.device, env.world_size, env.rank
    B, n = args.batch_size, xtr.shape[0]
    torch.manual_seed(args.seed)
    model = Net().to(dev)
    if world > 1:
        kw = {"device_ids": [dev.index]} if dev.type == "cuda" else {}
        model = torch.nn.parallel.DistributedDataParallel(model, **kw)
    opt = torch.optim.SGD(model.parameters(), lr=args.lr, momentum=args.momentum)
    core = model.module if hasattr(model, "module") else model
    start_epoch = 1
    ck = _load_ckpt(args)
    if ck is not None:  # every rank loads (CPU jobs share the checkpoint directory)
        core.load_state_dict(ck["model"])
        opt.load_state_dict(ck["optim"])
        start_epoch = ck["epoch"] + 1
        emit("resumed", epoch=ck["epoch"])

    def norm(x):
        return ((x.float() / 255.0 - 0.1307) / 0.3081).view(-1, 1, 28, 28)

    t_train, steps_done = 0.0, 0
    test_loss = acc = float("nan")
    for epoch in range(start_epoch, args.epochs + 1):
        model.train()
        perm = _epoch_perm(n, args.seed, epoch, rank, args.shard, dev).long()
        t0 = time.perf_counter()
        for batch_idx in range(steps_per_epoch):
            idx = perm[batch_idx * B:(batch_idx + 1) * B]
            data, target = norm(xtr[idx]), ytr[idx].long()
            opt.zero_grad()
            loss = F.nll_loss(model(data), target)
            loss.backward()
            opt.step()
            if steps_done == 0 and batch_idx == 0:
                startup.mark("first_step")
                emit("startup", **startup.record())
                emit("first_step")
            if emit.wm is not None:
                emit.wm.inc("pto_worker_steps_total")
            if batch_idx % args.log_interval == 0:
                _log_train(epoch, batch_idx, B, n, steps_per_epoch, loss.item(), writer, emit.wm)
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        t_train += time.perf_counter() - t0
        steps_done += steps_per_epoch
        model.eval()
        test_loss, correct = 0.0, 0
        with torch.no_grad():
            for s in range(0, xte.shape[0], args.test_batch_size):
                data, target = norm(xte[s:s + args.test_batch_size]), yte[s:s + args.test_batch_size].long()
                out = model(data)
                test_loss += F.nll_loss(out, target, reduction="sum").item()
                correct += out.argmax(1).eq(target).sum().item()
        acc = correct / xte.shape[0]
        test_loss /= xte.shape[0]
        _log_test(acc, epoch, writer)
        _save_ckpt(args, rank, {"epoch": epoch, "model": core.state_dict(), "optim": opt.state_dict()})
        _maybe_fault(epoch, start_epoch > 1)
    if args.save_model and rank == 0:
        torch.save(core.state_dict(), args.model_path)
    return {"steps": steps_done, "train_seconds": round(t_train, 4),
            "samples_per_sec": round(steps_done * B * world / t_train, 1) if t_train else None,
            "test_loss": round(test_loss, 5), "accuracy": round(acc, 5)}


def main(argv=None, t_main_ns: Optional[int] = None) -> int:
    args = parse_args(argv)
    run(args, t_main_ns if t_main_ns is not None else _T_MODULE)
    return 0


if __name__ == "__main__":
    sys.exit(main())
