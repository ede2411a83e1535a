"""DDP training worker for the BASELINE's large-model job shapes (ResNet-50 / Llama-3 bf16).

The reference only ships the MNIST worker; BASELINE.json additionally names
"ResNet-50 DDP bf16" and "Llama-3 8B DDP bf16" (Master=1 Worker=7 on 8x MI355X).  This
entrypoint runs either shape under the same operator contract (env rendezvous, one
``amd.com/gpu`` per pod, ``--backend rccl``) with synthetic data and random-init
weights, and reports throughput as one JSON line (rank 0):

    python -m pytorch_operator_amd.harness.ddp_train --model resnet50 --batch-size 256
    python -m pytorch_operator_amd.harness.ddp_train --model llama3-8b --seq-len 2048 --batch-size 1

MI355X specifics: bf16 autocast (MFMA bf16 through hipBLASLt/MIOpen), fused RMSNorm / RoPE /
SwiGLU HIP kernels in the Llama blocks, bf16 matmul weights with fp32 masters updated by the
fused HIP AdamW (``--master-weights``, on by default on a GPU: no per-step weight/grad cast
kernels, fp32 all-reduce kept through a comm hook), DDP with flat gradient buckets sized for xGMI
(``--bucket-mb``, default 64: few, large RCCL collectives), ``gradient_as_bucket_view``
(no gradient copy), optional bf16 gradient compression (``--allreduce-dtype bf16``), and
the 288 GB HBM budget that lets Llama-3 8B train with plain DDP (whole fp32 model, grads
and AdamW state per GPU -- no sharding).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

MODELS = ("resnet50", "resnet-tiny", "llama3-8b", "llama3-1b", "llama-tiny")


def parse_args(argv=None):
    p = argparse.ArgumentParser(description="DDP training worker (ResNet-50 / Llama-3, synthetic data)")
    p.add_argument("--model", choices=MODELS, default="resnet50")
    p.add_argument("--batch-size", type=int, default=None, help="per-rank batch (default 256 / 1)")
    p.add_argument("--seq-len", type=int, default=2048)
    p.add_argument("--image-size", type=int, default=224)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--dtype", choices=["bf16", "fp32"], default="bf16")
    p.add_argument("--backend", default=None, choices=["gloo", "nccl", "rccl"])
    p.add_argument("--no-cuda", action="store_true")
    p.add_argument("--bucket-mb", type=float, default=64.0)
    p.add_argument("--allreduce-dtype", choices=["fp32", "bf16"], default="fp32")
    p.add_argument("--grad-checkpoint", action="store_true", help="Llama: recompute blocks in backward")
    p.add_argument("--master-weights", choices=["auto", "on", "off"], default="auto",
                   help="Llama: bf16 matmul weights + fp32 masters in the fused HIP AdamW (auto: on with a GPU)")
    p.add_argument("--conv-algo-search", choices=["on", "off"], default="on",
                   help="ResNet: let MIOpen benchmark conv algorithms per shape (torch.backends.cudnn.benchmark)")
    p.add_argument("--memory-format", choices=["channels_last", "contiguous"], default="channels_last",
                   help="ResNet activations/weights layout (NHWC maps to MIOpen's NHWC bf16 kernels)")
    p.add_argument("--bn", choices=["hip", "library"], default="hip",
                   help="ResNet: fused HIP batch-norm(+add)(+ReLU) kernels or PyTorch's BN/add/ReLU ops")
    p.add_argument("--bn-link", type=int, default=2, choices=[0, 1, 2],
                   help="ResNet: each bottleneck's bn3 backward also sums the next block's residual "
                        "gradient in-kernel (ops/batchnorm.py GradLink) instead of autograd's add pass (1); "
                        "2 also sums a stage's downsample-conv input gradient there (link_tap); 0: off")
    p.add_argument("--bn-mask", choices=["bits", "output"], default="bits",
                   help="ResNet: residual+ReLU BN backward masks from a 1-bit forward image, or re-read "
                        "from the BN output")
    p.add_argument("--pool", choices=["hip", "library"], default="hip",
                   help="ResNet stem max-pool: HIP kernels (1-byte taps, gather backward) or PyTorch's op")
    p.add_argument("--conv1x1", choices=["gemm", "library"], default="library",
                   help="ResNet: 1x1 convolutions as hipBLASLt GEMMs on the NHWC view, or MIOpen convs "
                        "(library: 30.5 vs 47.3 ms/step at B=256 -- hipBLASLt's picks for the K = N*H*W "
                        "weight-gradient GEMMs run at ~10%% of MIOpen's rate, profiles/r2_resnet_conv1x1_ab.md)")
    p.add_argument("--sgd", choices=["fused", "foreach"], default="fused",
                   help="ResNet SGD implementation (fused: one multi-tensor kernel per step)")
    p.add_argument("--attn", choices=["auto", "sdpa"], default="auto",
                   help="Llama attention: hand-written HIP flash attention where it applies, or SDPA")
    p.add_argument("--residual-norm", choices=["fused", "plain"], default="fused",
                   help="Llama: residual adds fused into the next RMSNorm (fwd and bwd) or plain add + norm")
    p.add_argument("--linear-bwd", choices=["tn", "autograd"], default="tn",
                   help="Llama projections: backward GEMMs with K-contiguous (transposed-copy) operands, "
                        "or autograd's dy.W / dy^T.x layouts")
    p.add_argument("--opt-overlap", choices=["on", "off"], default="off",
                   help="Llama (master weights): AdamW updates on a side stream, overlapped with the next "
                        "forward (each module waits only for its own parameters' updates); measured neutral "
                        "(358-360 ms both ways, profiles/r2_llama3_8b_opt_overlap_ab.json): the forward "
                        "GEMMs hold every CU")
    p.add_argument("--zero", choices=["auto", "0", "1"], default="auto",
                   help="Llama (master weights): ZeRO-1 -- reduce-scatter fp32 gradients, AdamW on this "
                        "rank's 1/W shard, all-gather bf16 weights (parallel/zero.py) instead of DDP's "
                        "fp32 all-reduce + a full optimizer per rank; auto = on when world > 1")
    p.add_argument("--zero-bucket-mb", type=float, default=256.0)
    p.add_argument("--zero-grad-view", type=int, default=1,
                   help="ZeRO bf16 buckets: backward GEMMs write weight gradients into the bucket (1/0)")
    p.add_argument("--gemm-tuning", choices=["off", "use", "tune"], default="use",
                   help="PyTorch TunableOp over hipBLASLt/rocBLAS for the model's GEMM shapes: 'use' "
                        "replays the measured per-shape winners in --gemm-tuning-file (shapes not in "
                        "it take the library default), 'tune' benchmarks every candidate solution "
                        "during the first (untimed) step and writes the file, 'off' = library default")
    p.add_argument("--gemm-tuning-file", default=None,
                   help="TunableOp results CSV (default: pytorch_operator_amd/tuning/gemm_mi355x.csv)")
    p.add_argument("--ckpt-dir", default=None,
                   help="checkpoint directory (utils/train_ckpt.py): resume from it if it holds one, save "
                        "there at the end (and every --ckpt-every steps); shared by all ranks")
    p.add_argument("--ckpt-every", type=int, default=0)
    p.add_argument("--lr", type=float, default=None)
    p.add_argument("--seed", type=int, default=1)
    p.add_argument("--json-out", default=None)
    return p.parse_args(argv)


def use_zero(args, device, world: int) -> bool:
    if not args.model.startswith("llama") or args.dtype != "bf16":
        return False
    if args.zero == "1":
        return True
    return args.zero == "auto" and world > 1 and use_master_weights(args, device)


def build(args, device, world: int = 1):
    import torch
    if args.model.startswith("resnet"):
        from ..models.resnet import (Bottleneck, resnet50, resnet_tiny, set_bn_impl, set_conv1x1_impl,
                                     set_pool_impl)
        model = set_bn_impl(resnet50() if args.model == "resnet50" else resnet_tiny(), args.bn)
        from ..ops import batchnorm as _bnm
        from ..ops.batchnorm import BatchNormAct2d
        _bnm.MASK_BITS = args.bn_mask == "bits"
        for m in model.modules():
            if isinstance(m, BatchNormAct2d) and m.link_output:
                m.link_output = bool(args.bn_link)
            if isinstance(m, Bottleneck):
                m.tap_downsample = args.bn_link >= 2
        set_pool_impl(model, args.pool)
        set_conv1x1_impl(model, args.conv1x1)
        fmt = torch.channels_last if args.memory_format == "channels_last" else torch.contiguous_format
        model = model.to(device=device, memory_format=fmt)
        if device.type == "cuda":
            torch.backends.cudnn.benchmark = args.conv_algo_search == "on"
        kw = {}
        if device.type == "cuda":
            kw = {"fused": True} if args.sgd == "fused" else {"foreach": True}
        opt = torch.optim.SGD(model.parameters(), lr=args.lr or 0.1, momentum=0.9, weight_decay=1e-4, **kw)
        return model, opt
    from ..models.llama import CONFIGS, Attention, Llama, RMSNorm, TNLinear
    Attention.impl = args.attn
    TNLinear.impl = args.linear_bwd
    RMSNorm.fuse_residual = args.residual_norm == "fused"
    with torch.device(device):
        model = Llama(CONFIGS[args.model], checkpoint_layers=args.grad_checkpoint)
    if use_zero(args, device, world):
        from ..ops.optim import to_bf16_matmul_weights
        from ..parallel.zero import ZeroAdamW
        to_bf16_matmul_weights(model)
        # bf16 gradient buckets with a bf16 reduce (at world 1 the buckets always take the
        # parameters' dtype): gradient-as-bucket-view then lets the backward GEMMs write dW
        # into the buckets directly
        opt = ZeroAdamW(model, lr=args.lr or 3e-4, betas=(0.9, 0.95), weight_decay=0.1,
                        bucket_mb=args.zero_bucket_mb,
                        reduce_dtype=torch.bfloat16 if args.allreduce_dtype == "bf16" else torch.float32,
                        grad_view=bool(args.zero_grad_view))
        return model, opt
    if use_master_weights(args, device):
        from ..ops.optim import MasterAdamW, install_overlap, to_bf16_matmul_weights
        to_bf16_matmul_weights(model)
        overlap = args.opt_overlap == "on" and device.type == "cuda"
        opt = MasterAdamW(model.parameters(), lr=args.lr or 3e-4, betas=(0.9, 0.95), weight_decay=0.1,
                          overlap=overlap)
        if overlap:
            install_overlap(model)
        return model, opt
    kw = {"fused": True} if device.type == "cuda" else {}
    try:
        opt = torch.optim.AdamW(model.parameters(), lr=args.lr or 3e-4, betas=(0.9, 0.95), weight_decay=0.1, **kw)
    except (RuntimeError, TypeError):
        opt = torch.optim.AdamW(model.parameters(), lr=args.lr or 3e-4, betas=(0.9, 0.95), weight_decay=0.1)
    return model, opt


def default_tuning_file() -> str:
    return os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tuning",
                        "gemm_mi355x.csv")


def setup_gemm_tuning(args, device) -> dict:
    """TunableOp: each GEMM shape the model issues is dispatched to the hipBLASLt/rocBLAS
    solution measured fastest for it on MI355X (results CSV kept in-tree, validated by the
    library against the ROCm / hipBLASLt / gfx versions it was tuned on).  'tune' runs the
    search inside the first, untimed step; the timed steps only replay the winners."""
    if device.type != "cuda" or args.gemm_tuning == "off":
        return {"mode": "off"}
    import torch.cuda.tunable as tunable
    path = args.gemm_tuning_file or default_tuning_file()
    if args.gemm_tuning == "use" and not os.path.exists(path):
        return {"mode": "off", "missing": path}
    tunable.enable(True)
    tunable.tuning_enable(args.gemm_tuning == "tune")
    if args.gemm_tuning == "tune":
        if os.path.exists(path):
            tunable.read_file(path)  # keep the shapes tuned before; search only new ones
        tunable.set_max_tuning_duration(20)
        tunable.set_max_tuning_iterations(30)
        # the library appends the rank to the file name when it writes; keep ours explicit
        tunable.set_filename(path + ".tuning", False)
    elif not tunable.read_file(path):
        # validators differ (another ROCm / hipBLASLt / torch build): library defaults
        tunable.enable(False)
        print(f"warning: TunableOp rejected {path}; GEMMs use the library default", file=sys.stderr)
        return {"mode": "off", "rejected": path}
    return {"mode": args.gemm_tuning, "file": os.path.relpath(path, os.getcwd())}


def write_tuning_file(path: str) -> int:
    """Write TunableOp's in-memory results (validators first, then one line per tuned GEMM
    shape) in the CSV format ``read_file`` accepts; returns the number of shapes."""
    import torch.cuda.tunable as tunable
    rows = tunable.get_results()
    with open(path, "w") as f:
        vals = tunable.get_validators()
        for name, value in (vals.items() if isinstance(vals, dict) else vals):
            f.write(f"Validator,{name},{value}\n")
        for op, params, sol, ms in rows:
            f.write(f"{op},{params},{sol},{float(ms):.6f}\n")
    return len(rows)


def use_master_weights(args, device) -> bool:
    if not args.model.startswith("llama") or args.dtype != "bf16":
        return False
    return args.master_weights == "on" or (args.master_weights == "auto" and device.type == "cuda")


def fp32_allreduce_hook(process_group, bucket):
    """DDP comm hook: all-reduce a bf16 gradient bucket in fp32 (``--allreduce-dtype fp32`` with
    bf16 master-weight training).  The fp32 mean is what the optimizer consumes: each
    parameter gets ``_pto_grad32``, a view into the reduced fp32 bucket, which ``MasterAdamW``
    reads instead of the bf16 ``.grad`` (also refreshed, rounded, for anything else)."""
    import torch.distributed as dist
    buf = bucket.buffer()
    group = process_group if process_group is not None else dist.group.WORLD
    t = buf.float().div_(dist.get_world_size(group))
    fut = dist.all_reduce(t, group=group, async_op=True).get_future()
    params, grads = bucket.parameters(), bucket.gradients()

    def done(f):
        red = f.value()[0]
        esz = buf.element_size()
        for p, g in zip(params, grads):
            off = (g.data_ptr() - buf.data_ptr()) // esz
            p._pto_grad32 = red[off:off + g.numel()].view(g.shape)
        buf.copy_(red)
        return buf
    return fut.then(done)


def param_digest(model, opt) -> str:
    """sha1 over every parameter and (MasterAdamW) fp32 master, in order: DDP replicas must agree."""
    import hashlib
    import torch
    h = hashlib.sha1()
    for p in model.parameters():
        h.update(p.detach().float().cpu().numpy().tobytes())
        st = opt.state.get(p) or {}
        if isinstance(st.get("master"), torch.Tensor):
            h.update(st["master"].detach().cpu().numpy().tobytes())
    return h.hexdigest()


def weights_digest(model) -> str:
    """sha1 over every parameter tensor as the model holds it (bf16 weights, fp32 norms)."""
    import hashlib
    h = hashlib.sha1()
    for p in model.parameters():
        h.update(p.detach().float().cpu().numpy().tobytes())
    return h.hexdigest()


def train_flops_per_sample(args) -> float:
    if args.model.startswith("resnet"):
        scale = (args.image_size / 224.0) ** 2
        return 3 * 4.09e9 * scale if args.model == "resnet50" else 0.0
    from ..models.llama import CONFIGS
    c = CONFIGS[args.model]
    n = c.num_params() - c.vocab_size * c.dim  # embedding lookup is not a matmul
    # causal attention per token: QK^T and PV over the (on average) S/2 visible keys = 2*S*d
    # forward FLOPs per layer, x3 for forward + backward = 6*L*d*S
    attn = 6 * c.n_layers * c.dim * args.seq_len
    return (6 * n + attn) * args.seq_len  # per sequence


def main(argv=None) -> int:
    args = parse_args(argv)
    import torch
    import torch.distributed as dist
    import torch.nn.functional as F
    from ..parallel.dist import init_from_env

    use_gpu = not args.no_cuda and torch.cuda.is_available()
    env = init_from_env(args.backend, use_gpu=use_gpu)
    dev, world, rank = env.device, env.world_size, env.rank
    torch.manual_seed(args.seed)
    is_llama = args.model.startswith("llama")
    B = args.batch_size or (1 if is_llama else (256 if use_gpu else 2))
    model, opt = build(args, dev, world)
    zero = use_zero(args, dev, world)
    tuning = setup_gemm_tuning(args, dev)
    n_params = sum(p.numel() for p in model.parameters())
    if world > 1 and not zero:
        from torch.nn.parallel import DistributedDataParallel as DDP
        model = DDP(model, device_ids=[dev.index] if use_gpu else None, bucket_cap_mb=args.bucket_mb,
                    gradient_as_bucket_view=True, static_graph=True)
        if args.allreduce_dtype == "bf16":
            from torch.distributed.algorithms.ddp_comm_hooks import default_hooks
            model.register_comm_hook(None, default_hooks.bf16_compress_hook)
        elif use_master_weights(args, dev):
            model.register_comm_hook(None, fp32_allreduce_hook)
    g = torch.Generator(device="cpu").manual_seed(args.seed + rank)
    if is_llama:
        from ..models.llama import CONFIGS
        V = CONFIGS[args.model].vocab_size
        data = torch.randint(0, V, (B, args.seq_len + 1), generator=g).to(dev)
        x, y = data[:, :-1].contiguous(), data[:, 1:].contiguous()
    else:
        H = args.image_size if args.model == "resnet50" else 32
        x = torch.randn(B, 3, H, H, generator=g).to(dev)
        if args.memory_format == "channels_last":
            x = x.to(memory_format=torch.channels_last)
        y = torch.randint(0, 1000 if args.model == "resnet50" else 10, (B,), generator=g).to(dev)
    amp = torch.autocast(device_type=dev.type, dtype=torch.bfloat16, enabled=args.dtype == "bf16")
    from ..utils import train_ckpt
    bare = model.module if hasattr(model, "module") else model
    gstep = train_ckpt.load(args.ckpt_dir, bare, opt, rank, world, dev)
    if gstep and rank == 0:
        print(json.dumps({"event": "resumed", "step": gstep, "dir": args.ckpt_dir}), flush=True)

    def step():
        nonlocal gstep
        gstep += 1
        if args.ckpt_dir and args.ckpt_every and gstep % args.ckpt_every == 0:
            pending_ckpt.append(gstep)
        opt.zero_grad(set_to_none=True)
        with amp:
            if is_llama:
                loss = model(x, y)
            else:
                loss = F.cross_entropy(model(x).float(), y)
        loss.backward()
        opt.step()
        if pending_ckpt:
            train_ckpt.save(args.ckpt_dir, pending_ckpt.pop(), bare, opt, rank, world)
        return loss

    pending_ckpt = []

    def sync():
        if use_gpu:
            torch.cuda.synchronize(dev)

    t_start = time.time_ns()
    loss = step()
    sync()
    if rank == 0:
        print(json.dumps({"event": "first_step", "rank": rank, "unix_ns": time.time_ns(),
                          "first_step_s": round((time.time_ns() - t_start) / 1e9, 3),
                          "loss": float(loss)}), flush=True)
    for _ in range(max(0, args.warmup - 1)):
        step()
    sync()
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    sync()
    if world > 1:
        dist.barrier()
    sync()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    samples = args.steps * B * world
    per_sample = train_flops_per_sample(args)
    unit_tokens = is_llama
    value = samples * (args.seq_len if unit_tokens else 1) / dt
    res = {"metric": f"{args.model.replace('-', '_')}_ddp_train_{'tokens' if unit_tokens else 'images'}_per_sec",
           "value": round(value, 1), "unit": "tokens/s" if unit_tokens else "images/s", "n_gpus": world,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3),
           "dtype": args.dtype, "data": "synthetic", "params": n_params, "per_rank_batch": B,
           "seq_len": args.seq_len if is_llama else None, "loss": float(loss),
           "tflops_per_gpu": round(per_sample * samples / dt / world / 1e12, 1) if per_sample else None,
           "max_mem_gb": round(torch.cuda.max_memory_allocated(dev) / 2 ** 30, 1) if use_gpu else None,
           "parallelism": f"dp{world}", "bucket_mb": args.bucket_mb, "allreduce_dtype": args.allreduce_dtype,
           "master_weights": use_master_weights(args, dev) or zero, "zero": 1 if zero else 0}
    if zero:
        res.update(optimizer_state_gb_per_rank=round(opt.state_bytes() / 2 ** 30, 2), zero_buckets=len(opt.buckets),
                   zero_grad_sinks=opt.sinks, zero_grad_dtypes=sorted({str(b.gdt).replace("torch.", "") for b in opt.buckets}))
    res.update(gemm_tuning=tuning.get("mode"))
    if is_llama:
        res.update(attn=args.attn, residual_norm=args.residual_norm, linear_bwd=args.linear_bwd,
                   opt_overlap=args.opt_overlap if res["master_weights"] and not zero else None)
    if tuning.get("mode") == "tune" and rank == 0:
        import torch.cuda.tunable as tunable
        out = args.gemm_tuning_file or default_tuning_file()
        os.makedirs(os.path.dirname(out), exist_ok=True)
        write_tuning_file(out)
        res.update(gemm_tuning_file=out, gemm_tuned_shapes=len(tunable.get_results()))
    if not is_llama:
        res.update(memory_format=args.memory_format, conv_algo_search=args.conv_algo_search, sgd=args.sgd, bn=args.bn, bn_link=args.bn_link,
                   bn_mask=args.bn_mask, pool=args.pool,
                   conv1x1=args.conv1x1)
    if args.ckpt_dir:
        train_ckpt.save(args.ckpt_dir, gstep, bare, opt, rank, world)
        res.update(checkpoint_step=gstep)
    if zero:
        opt.synchronize()
        digest = opt.full_masters_digest()
    else:
        digest = param_digest(model.module if hasattr(model, "module") else model, opt)
    wdig = weights_digest(model.module if hasattr(model, "module") else model)
    print(json.dumps({"event": "param_digest", "rank": rank, "digest": digest, "weights_digest": wdig}),
          flush=True)
    if rank == 0:
        print(json.dumps(res), flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(json.dumps(res) + "\n")
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
