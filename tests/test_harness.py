"""Worker entrypoints on CPU: the MNIST DDP worker and the smoke send/recv test.

The reference has no tests for examples/; these pin its observable contract (CLI,
log lines, TensorBoard scalars, DDP over the env rendezvous) for the MI355X worker.
Multi-process cases use gloo with world_size 2 on 127.0.0.1.
"""
import glob
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

from pytorch_operator_amd.data.mnist_idx import load_mnist, read_idx, write_idx
from pytorch_operator_amd.utils.tb_writer import SummaryWriter, crc32c, read_events

ROOT = Path(__file__).resolve().parent.parent


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _launch(module, args, world, cwd, timeout=240):
    port = _port()
    procs = []
    for r in range(world):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(r),
                   PYTHONPATH=str(ROOT), OMP_NUM_THREADS="1")
        procs.append(subprocess.Popen([sys.executable, "-m", module, *args], cwd=cwd, env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        out, _ = p.communicate(timeout=timeout)
        outs.append((p.returncode, out))
    return outs


def _events(out):
    return [json.loads(x) for x in out.splitlines() if x.startswith('{"event"')]


def test_crc32c_known_vector():
    assert crc32c(b"123456789") == 0xE3069283


def test_tensorboard_writer_roundtrip(tmp_path):
    with SummaryWriter(str(tmp_path)) as w:
        w.add_scalar("loss", 2.5, 0)
        w.add_scalar("loss", 1.25, 10)
        w.add_scalar("accuracy", 0.5, 1)
    ev = read_events(glob.glob(str(tmp_path / "events.out.tfevents.*"))[0])
    assert ev[1:] == [(0, {"loss": 2.5}), (10, {"loss": 1.25}), (1, {"accuracy": 0.5})]
    lines = [json.loads(x) for x in open(tmp_path / "scalars.jsonl")]
    assert [x["tag"] for x in lines] == ["loss", "loss", "accuracy"]


def test_idx_reader_roundtrip(tmp_path):
    x = np.random.default_rng(0).integers(0, 256, (7, 28, 28), dtype=np.uint8)
    y = np.arange(7, dtype=np.uint8)
    raw = tmp_path / "MNIST" / "raw"
    raw.mkdir(parents=True)
    write_idx(str(raw / "train-images-idx3-ubyte.gz"), x)
    write_idx(str(raw / "train-labels-idx1-ubyte"), y)
    assert (read_idx(str(raw / "train-images-idx3-ubyte.gz")) == x).all()
    xi, yi = load_mnist(str(tmp_path), "train")
    assert xi.shape == (7, 784) and xi.dtype == torch.uint8 and yi.dtype == torch.int32
    assert (xi.numpy().reshape(7, 28, 28) == x).all() and (yi.numpy() == y).all()
    assert load_mnist(str(tmp_path), "test") is None


def test_mnist_worker_single_process_reference_output(tmp_path):
    (rc, out), = _launch("pytorch_operator_amd.harness.mnist",
                         ["--dataset-size", "1280", "--test-size", "400", "--log-interval", "5", "--save-model",
                          "--dir", str(tmp_path / "tb")], 1, tmp_path)
    assert rc == 0, out
    assert "Train Epoch: 1 [0/1280 (0%)]\tloss=" in out
    assert "Train Epoch: 1 [320/1280 (25%)]\tloss=" in out
    assert "\naccuracy=" in out
    ev = _events(out)
    assert [e["event"] for e in ev] == ["start", "startup", "first_step", "train_done"]
    assert ev[0]["kernels"] == "torch" and ev[-1]["steps"] == 20
    # create-to-first-step breakdown: every in-pod phase, in order, summing to the wall clock
    st = ev[1]
    marks = st["marks_unix_ns"]
    assert list(marks) == ["process_start", "worker_main", "import_torch", "process_group", "dataset",
                           "first_step"], marks
    assert list(marks.values()) == sorted(marks.values())
    assert abs(sum(st["phases"].values()) - (marks["first_step"] - marks["process_start"]) / 1e9) < 1e-3
    sd = torch.load(tmp_path / "mnist_cnn.pt", weights_only=True)
    assert sd["fc1.weight"].shape == (500, 800)
    scal = [json.loads(x) for x in open(tmp_path / "tb" / "scalars.jsonl")]
    assert [s["step"] for s in scal if s["tag"] == "loss"] == [20, 25, 30, 35]  # epoch*len + batch_idx


def test_mnist_worker_learns_on_real_idx_files(tmp_path):
    """IDX files present -> used instead of synthetic data (content from the synthetic generator)."""
    from pytorch_operator_amd.data.synthetic import make_synthetic_mnist
    d = tmp_path / "data"
    d.mkdir()
    tr, te = make_synthetic_mnist(3000, seed=3), make_synthetic_mnist(500, seed=4)
    write_idx(str(d / "train-images-idx3-ubyte"), tr.images.numpy().reshape(-1, 28, 28))
    write_idx(str(d / "train-labels-idx1-ubyte"), tr.labels.numpy().astype(np.uint8))
    write_idx(str(d / "t10k-images-idx3-ubyte"), te.images.numpy().reshape(-1, 28, 28))
    write_idx(str(d / "t10k-labels-idx1-ubyte"), te.labels.numpy().astype(np.uint8))
    (rc, out), = _launch("pytorch_operator_amd.harness.mnist", ["--data-dir", str(d), "--epochs", "2",
                                                                "--dir", str(tmp_path / "tb")], 1, tmp_path)
    assert rc == 0, out
    ev = _events(out)
    assert ev[0]["data"] == "mnist-idx" and ev[0]["n_train"] == 3000
    assert out.count("accuracy=") == 2
    assert ev[-1]["accuracy"] > 0.5


def test_mnist_worker_ddp_gloo_two_ranks(tmp_path):
    outs = _launch("pytorch_operator_amd.harness.mnist",
                   ["--backend", "gloo", "--dataset-size", "1280", "--test-size", "256", "--shard", "--dir",
                    str(tmp_path / "tb")], 2, tmp_path)
    for rc, out in outs:
        assert rc == 0, out
        assert "Using distributed PyTorch with gloo backend" in out
    ev0, ev1 = _events(outs[0][1]), _events(outs[1][1])
    # sharded: 640 samples per rank -> 10 steps each; DDP keeps the replicas identical
    assert ev0[-1]["steps"] == 10 and ev1[-1]["steps"] == 10
    assert ev0[-1]["test_loss"] == ev1[-1]["test_loss"]


def test_mnist_worker_default_matches_reference_semantics(tmp_path):
    outs = _launch("pytorch_operator_amd.harness.mnist",
                   ["--backend", "gloo", "--dataset-size", "640", "--test-size", "128",
                    "--dir", str(tmp_path / "tb")], 2, tmp_path)
    for rc, out in outs:
        assert rc == 0, out
    assert _events(outs[0][1])[-1]["steps"] == 10  # every rank walks the whole set


def test_backend_aliases():
    from pytorch_operator_amd.parallel.dist import backend_for
    assert backend_for("rccl", True) == "nccl"
    assert backend_for("GLOO", False) == "gloo"
    assert backend_for(None, False) == "gloo" and backend_for(None, True) == "nccl"
    with pytest.raises(ValueError):
        backend_for("ucc", False)
    with pytest.raises(RuntimeError):
        backend_for("mpi", False)


def test_dist_sendrecv_three_ranks(tmp_path):
    outs = _launch("pytorch_operator_amd.harness.dist_sendrecv", [], 3, tmp_path, timeout=120)
    for rc, out in outs:
        assert rc == 0, out
    master = outs[0][1]
    assert "Result from worker 1" in master and "Result from worker 2" in master
    assert "all_reduce ok (6.0)" in master
    assert "MASTER_ADDR: 127.0.0.1" in master and "WORLD_SIZE: 3" in master


def test_checkpoint_resume_continues_at_next_epoch(tmp_path):
    ck = tmp_path / "ck"
    common = ["--dataset-size", "640", "--test-size", "128", "--checkpoint-dir", str(ck), "--dir", str(tmp_path / "tb")]
    (rc, out), = _launch("pytorch_operator_amd.harness.mnist", ["--epochs", "1", *common], 1, tmp_path)
    assert rc == 0, out
    assert (ck / "ckpt.pt").exists()
    (rc, out), = _launch("pytorch_operator_amd.harness.mnist", ["--epochs", "2", "--resume", *common], 1, tmp_path)
    assert rc == 0, out
    ev = _events(out)
    assert any(e["event"] == "resumed" and e["epoch"] == 1 for e in ev)
    assert "Train Epoch: 2 [0/640" in out and "Train Epoch: 1 " not in out
    assert ev[-1]["steps"] == 10  # only epoch 2 ran
    sd = torch.load(ck / "ckpt.pt", weights_only=True)
    assert sd["epoch"] == 2 and "optim" in sd


def test_fault_injection_hook_exits_137_after_checkpoint(tmp_path):
    ck = tmp_path / "ck"
    env_args = ["--dataset-size", "640", "--test-size", "128", "--epochs", "2", "--checkpoint-dir", str(ck),
                "--resume", "--dir", str(tmp_path / "tb")]
    os.environ["PTO_FAULT_EXIT_AFTER_EPOCH"] = "1"
    try:
        (rc, out), = _launch("pytorch_operator_amd.harness.mnist", env_args, 1, tmp_path)
        assert rc == 137 and (ck / "ckpt.pt").exists()
        (rc, out), = _launch("pytorch_operator_amd.harness.mnist", env_args, 1, tmp_path)
        assert rc == 0, out  # resumed runs are never faulted
        assert any(e["event"] == "resumed" for e in _events(out))
    finally:
        del os.environ["PTO_FAULT_EXIT_AFTER_EPOCH"]


def test_ddp_train_worker_llama_tiny_two_ranks(tmp_path):
    outs = _launch("pytorch_operator_amd.harness.ddp_train",
                   ["--model", "llama-tiny", "--seq-len", "32", "--batch-size", "2", "--steps", "2", "--warmup", "1",
                    "--backend", "gloo", "--allreduce-dtype", "bf16"], 2, tmp_path)
    for rc, out in outs:
        assert rc == 0, out
    res = json.loads([ln for ln in outs[0][1].splitlines() if ln.startswith('{"metric"')][-1])
    assert res["metric"] == "llama_tiny_ddp_train_tokens_per_sec" and res["n_gpus"] == 2


def test_ddp_train_worker_llama_tiny_master_weights_two_ranks(tmp_path):
    """bf16 matmul weights + fp32 masters (MasterAdamW) under DDP with the fp32 all-reduce hook."""
    outs = _launch("pytorch_operator_amd.harness.ddp_train",
                   ["--model", "llama-tiny", "--seq-len", "32", "--batch-size", "2", "--steps", "2", "--warmup", "1",
                    "--backend", "gloo", "--master-weights", "on", "--zero", "0"], 2, tmp_path)
    for rc, out in outs:
        assert rc == 0, out
    res = json.loads([ln for ln in outs[0][1].splitlines() if ln.startswith('{"metric"')][-1])
    assert res["master_weights"] is True and res["zero"] == 0 and res["loss"] == res["loss"]
    # replicas stay identical: every rank's parameters AND fp32 masters hash the same
    digests = [json.loads([ln for ln in out.splitlines() if '"param_digest"' in ln][-1])["digest"]
               for _, out in outs]
    assert len(set(digests)) == 1, digests


def _digests(outs):
    return [json.loads([ln for ln in out.splitlines() if '"param_digest"' in ln][-1]) for _, out in outs]


def test_ddp_train_llama_zero1_matches_ddp_master_adamw(tmp_path):
    """ZeRO-1 (parallel/zero.py: fp32 reduce-scatter, AdamW on a 1/W shard, bf16 all-gather)
    must produce bit-identical weights to DDP + fp32 all-reduce hook + MasterAdamW, with the
    gathered fp32 masters identical on every rank, and hold 1/W of the optimizer state."""
    base = ["--model", "llama-tiny", "--seq-len", "32", "--batch-size", "2", "--steps", "3", "--warmup", "1",
            "--backend", "gloo", "--master-weights", "on", "--zero-bucket-mb", "0.05"]
    (tmp_path / "z").mkdir()
    (tmp_path / "d").mkdir()
    outs_z = _launch("pytorch_operator_amd.harness.ddp_train", base + ["--zero", "1"], 2, tmp_path / "z")
    outs_d = _launch("pytorch_operator_amd.harness.ddp_train", base + ["--zero", "0"], 2, tmp_path / "d")
    for rc, out in outs_z + outs_d:
        assert rc == 0, out
    rz = json.loads([ln for ln in outs_z[0][1].splitlines() if ln.startswith('{"metric"')][-1])
    rd = json.loads([ln for ln in outs_d[0][1].splitlines() if ln.startswith('{"metric"')][-1])
    assert rz["zero"] == 1 and rz["zero_buckets"] > 2 and rd["zero"] == 0
    assert rz["loss"] == rd["loss"]
    dz, dd = _digests(outs_z), _digests(outs_d)
    assert len({d["weights_digest"] for d in dz + dd}) == 1, (dz, dd)
    assert len({d["digest"] for d in dz}) == 1, dz
    from pytorch_operator_amd.models.llama import CONFIGS
    n = CONFIGS["llama-tiny"].num_params()
    assert rz["optimizer_state_gb_per_rank"] * 2 ** 30 < 12 * n * 0.6  # ~1/2 of 12 B/param


@pytest.mark.parametrize("zero", ["0", "1"])
def test_ddp_train_checkpoint_resume_matches_uninterrupted(tmp_path, zero):
    """OnFailure-restart contract for the Llama worker: 2 steps + checkpoint, then a fresh process
    pair resuming for 2 more, ends bit-identical to 4 uninterrupted steps (DDP + MasterAdamW and
    ZeRO-1 sharded optimizer state)."""
    base = ["--model", "llama-tiny", "--seq-len", "32", "--batch-size", "2", "--warmup", "1",
            "--backend", "gloo", "--master-weights", "on", "--zero", zero, "--zero-bucket-mb", "0.05"]
    for d in ("a", "b"):
        (tmp_path / d).mkdir()
    ck = str(tmp_path / "b" / "ckpt")
    outs_a = _launch("pytorch_operator_amd.harness.ddp_train", base + ["--steps", "3"], 2, tmp_path / "a")
    outs_b1 = _launch("pytorch_operator_amd.harness.ddp_train", base + ["--steps", "1", "--ckpt-dir", ck], 2,
                      tmp_path / "b")
    outs_b2 = _launch("pytorch_operator_amd.harness.ddp_train", base + ["--steps", "1", "--ckpt-dir", ck], 2,
                      tmp_path / "b")
    for rc, out in outs_a + outs_b1 + outs_b2:
        assert rc == 0, out
    assert '"event": "resumed", "step": 2' in outs_b2[0][1]
    ra = json.loads([ln for ln in outs_a[0][1].splitlines() if ln.startswith('{"metric"')][-1])
    rb = json.loads([ln for ln in outs_b2[0][1].splitlines() if ln.startswith('{"metric"')][-1])
    assert rb["checkpoint_step"] == 4 and rb["loss"] == ra["loss"]
    da, db = _digests(outs_a), _digests(outs_b2)
    assert {x["weights_digest"] for x in da} == {x["weights_digest"] for x in db}
    assert {x["digest"] for x in da} == {x["digest"] for x in db}


def test_ddp_train_resnet_tiny_checkpoint_resume(tmp_path):
    """The torch-optimizer path (ResNet, SGD momentum buffers): resume equals uninterrupted."""
    base = ["--model", "resnet-tiny", "--batch-size", "4", "--warmup", "1", "--backend", "gloo", "--dtype", "fp32"]
    for d in ("a", "b"):
        (tmp_path / d).mkdir()
    ck = str(tmp_path / "b" / "ckpt")
    (ra, oa), = _launch("pytorch_operator_amd.harness.ddp_train", base + ["--steps", "3"], 1, tmp_path / "a")
    (r1, o1), = _launch("pytorch_operator_amd.harness.ddp_train", base + ["--steps", "1", "--ckpt-dir", ck], 1,
                        tmp_path / "b")
    (r2, o2), = _launch("pytorch_operator_amd.harness.ddp_train", base + ["--steps", "1", "--ckpt-dir", ck], 1,
                        tmp_path / "b")
    assert ra == r1 == r2 == 0, o1 + o2
    assert _digests([(0, oa)])[0]["weights_digest"] == _digests([(0, o2)])[0]["weights_digest"]


def test_ddp_train_llama_zero1_three_ranks_bf16_reduce(tmp_path):
    """Non-power-of-two world (copy + divide path) with the bf16 reduce-scatter: replicas agree."""
    outs = _launch("pytorch_operator_amd.harness.ddp_train",
                   ["--model", "llama-tiny", "--seq-len", "32", "--batch-size", "2", "--steps", "2", "--warmup", "1",
                    "--backend", "gloo", "--master-weights", "on", "--zero", "1", "--allreduce-dtype", "bf16"],
                   3, tmp_path)
    for rc, out in outs:
        assert rc == 0, out
    res = json.loads([ln for ln in outs[0][1].splitlines() if ln.startswith('{"metric"')][-1])
    assert res["zero"] == 1 and res["n_gpus"] == 3 and res["loss"] == res["loss"]
    d = _digests(outs)
    assert len({x["weights_digest"] for x in d}) == 1 and len({x["digest"] for x in d}) == 1, d


@pytest.mark.parametrize("reduce_dtype", ["float32", "bfloat16"])
def test_zero_adamw_single_process_matches_master_adamw(reduce_dtype):
    """World 1 (no process group): ZeroAdamW's update equals MasterAdamW's, element for element,
    whatever the reduce dtype (at world 1 every gradient bucket takes its parameters' dtype)."""
    import copy
    from pytorch_operator_amd.models.llama import CONFIGS, Llama
    from pytorch_operator_amd.ops.optim import MasterAdamW, to_bf16_matmul_weights
    from pytorch_operator_amd.parallel.zero import ZeroAdamW
    torch.manual_seed(0)
    m1 = Llama(CONFIGS["llama-tiny"])
    m2 = copy.deepcopy(m1)
    to_bf16_matmul_weights(m1)
    to_bf16_matmul_weights(m2)
    o1 = MasterAdamW(m1.parameters(), lr=1e-3, betas=(0.9, 0.95), weight_decay=0.1)
    o2 = ZeroAdamW(m2, lr=1e-3, betas=(0.9, 0.95), weight_decay=0.1, bucket_mb=0.02,
                   reduce_dtype=getattr(torch, reduce_dtype))
    x = torch.randint(0, 256, (2, 17))
    for _ in range(3):
        for m, o in ((m1, o1), (m2, o2)):
            o.zero_grad(set_to_none=True)
            with torch.autocast("cpu", dtype=torch.bfloat16):
                loss = m(x[:, :-1], x[:, 1:])
            loss.backward()
            o.step()
    for a, b in zip(m1.parameters(), m2.parameters()):
        assert torch.equal(a, b)


def test_zero_adamw_unused_parameter_matches_master_adamw():
    """A bucket with a parameter that gets no gradient: the gradients that did
    arrive are kept (not zeroed by the partial-bucket fallback) and the unused parameter is left
    untouched, as MasterAdamW skips parameters without a gradient."""
    import copy
    import torch.nn as nn
    from pytorch_operator_amd.ops.optim import MasterAdamW
    from pytorch_operator_amd.parallel.zero import ZeroAdamW

    class TwoHead(nn.Module):
        def __init__(self):
            super().__init__()
            self.a = nn.Linear(8, 8)
            self.unused = nn.Linear(8, 8)  # same bucket, never in the graph
            self.b = nn.Linear(8, 4)

        def forward(self, x):
            return self.b(torch.relu(self.a(x)))

    torch.manual_seed(1)
    m1 = TwoHead()
    m2 = copy.deepcopy(m1)
    o1 = MasterAdamW(m1.parameters(), lr=1e-2, betas=(0.9, 0.95), weight_decay=0.1)
    o2 = ZeroAdamW(m2, lr=1e-2, betas=(0.9, 0.95), weight_decay=0.1, bucket_mb=1.0)
    assert len(o2.buckets) == 1  # the unused parameter shares the bucket with the used ones
    x = torch.randn(5, 8)
    before = m2.unused.weight.detach().clone()
    for _ in range(3):
        for m, o in ((m1, o1), (m2, o2)):
            o.zero_grad(set_to_none=True)
            m(x).square().mean().backward()
            o.step()
    for (n, a), b in zip(m1.named_parameters(), m2.parameters()):
        assert torch.allclose(a, b, rtol=0, atol=1e-6), n
    assert torch.equal(m2.unused.weight, before)
    assert not torch.equal(m2.a.weight, m1.a.weight * 0)  # the used parameters did move


def test_zero_adamw_parameter_skipping_a_step_keeps_its_own_step_count():
    """a parameter that gets no gradient in one step and then trains again uses its
    own AdamW step count for the bias correction afterwards (MasterAdamW's st["step"]), not the
    optimizer's global count."""
    import copy
    import torch.nn as nn
    from pytorch_operator_amd.ops.optim import MasterAdamW
    from pytorch_operator_amd.parallel.zero import ZeroAdamW

    class Gated(nn.Module):
        def __init__(self):
            super().__init__()
            self.a = nn.Linear(8, 8)
            self.side = nn.Linear(8, 8)  # same bucket; skipped on odd steps
            self.b = nn.Linear(8, 4)

        def forward(self, x, use_side):
            h = torch.relu(self.a(x))
            if use_side:
                h = h + self.side(h)
            return self.b(h)

    torch.manual_seed(3)
    m1 = Gated()
    m2 = copy.deepcopy(m1)
    o1 = MasterAdamW(m1.parameters(), lr=1e-2, betas=(0.9, 0.95), weight_decay=0.1)
    o2 = ZeroAdamW(m2, lr=1e-2, betas=(0.9, 0.95), weight_decay=0.1, bucket_mb=1.0)
    assert len(o2.buckets) == 1
    x = torch.randn(5, 8)
    for step in range(5):
        for m, o in ((m1, o1), (m2, o2)):
            o.zero_grad(set_to_none=True)
            m(x, step % 2 == 0).square().mean().backward()
            o.step()
    assert o2.pstep[id(m2.side.weight)] == 3 and o2.pstep[id(m2.a.weight)] == 5
    for (n, a), b in zip(m1.named_parameters(), m2.parameters()):
        assert torch.allclose(a, b, rtol=0, atol=1e-6), n
    # the per-parameter counts survive a shard checkpoint round trip
    sd = o2.shard_state_dict()
    o3 = ZeroAdamW(copy.deepcopy(m2), lr=1e-2, betas=(0.9, 0.95), weight_decay=0.1, bucket_mb=1.0)
    o3.load_shard_state_dict(sd)
    assert sorted(o3.pstep.values()) == sorted(o2.pstep.values())


def test_zero_adamw_hook_without_gradient():
    """Autograd runs post-accumulate hooks even when a backward returns None for a leaf -- what
    linear_tn does for a weight whose gradient sink it wrote in place.  ZeroAdamW must treat
    that as "no gradient through the hook" (the GPU failure: a sink arrival followed by the
    hook raised "a second backward before step()").  Here the frozen-gradient weight behaves
    like an unused parameter: untouched, as MasterAdamW leaves it."""
    import copy
    import torch.nn as nn
    from pytorch_operator_amd.ops.optim import MasterAdamW
    from pytorch_operator_amd.parallel.zero import ZeroAdamW

    class NoWGrad(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x, w):
            ctx.save_for_backward(w)
            return x @ w.t()

        @staticmethod
        def backward(ctx, dy):
            (w,) = ctx.saved_tensors
            return dy @ w, None

    class M(nn.Module):
        def __init__(self):
            super().__init__()
            self.a = nn.Linear(8, 8)
            self.frozen = nn.Parameter(torch.randn(8, 8))
            self.b = nn.Linear(8, 4)

        def forward(self, x):
            return self.b(NoWGrad.apply(torch.relu(self.a(x)), self.frozen))

    torch.manual_seed(2)
    m1 = M()
    m2 = copy.deepcopy(m1)
    o1 = MasterAdamW(m1.parameters(), lr=1e-2, betas=(0.9, 0.95), weight_decay=0.1)
    o2 = ZeroAdamW(m2, lr=1e-2, betas=(0.9, 0.95), weight_decay=0.1, bucket_mb=1.0)
    x = torch.randn(5, 8)
    for _ in range(3):
        for m, o in ((m1, o1), (m2, o2)):
            o.zero_grad(set_to_none=True)
            m(x).square().mean().backward()
            o.step()
    for (n, a), b in zip(m1.named_parameters(), m2.parameters()):
        assert torch.allclose(a, b, rtol=0, atol=1e-6), n


def test_ddp_train_worker_resnet_tiny(tmp_path):
    (rc, out), = _launch("pytorch_operator_amd.harness.ddp_train",
                         ["--model", "resnet-tiny", "--batch-size", "2", "--steps", "2", "--warmup", "1"], 1, tmp_path)
    assert rc == 0, out
    assert '"resnet_tiny_ddp_train_images_per_sec"' in out


def test_example_yamls_are_valid_jobs():
    import yaml
    from opfixtures import opcore
    for path in sorted((ROOT / "examples").rglob("*.yaml")):
        job = yaml.safe_load(path.read_text())
        assert job["kind"] == "PyTorchJob", path
        err = opcore().validate_spec(json.dumps(job["spec"]))
        assert not err, (path, err)
        for spec in job["spec"]["pytorchReplicaSpecs"].values():
            for c in spec["template"]["spec"]["containers"]:
                assert "nvidia.com/gpu" not in json.dumps(c), path  # MI355X-only resources
        total = sum(int(s.get("replicas", 1)) for s in job["spec"]["pytorchReplicaSpecs"].values())
        if total == 8:  # the one-node 8 x MI355X jobs carry the xGMI pod topology (docs/xgmi_pods.md)
            for spec in job["spec"]["pytorchReplicaSpecs"].values():
                ps = spec["template"]["spec"]
                assert ps.get("hostPID") is True and ps.get("hostIPC") is True, path
                term = ps["affinity"]["podAffinity"]["requiredDuringSchedulingIgnoredDuringExecution"][0]
                assert term["topologyKey"] == "kubernetes.io/hostname", path
                assert term["labelSelector"]["matchLabels"] == {"job-name": job["metadata"]["name"]}, path
                env = {e["name"]: e for e in ps["containers"][0].get("env", [])}
                assert env["NCCL_HOSTID"]["valueFrom"]["fieldRef"]["fieldPath"] == "spec.nodeName", path


def test_util_pformat_and_rand_string():
    """pkg/util/util_test.go:5-11 (TestRandString) plus Pformat's string pass-through."""
    import json
    from pytorch_operator_amd.utils import pformat, rand_string
    assert len(rand_string(4)) == 4 and rand_string(0) == ""
    s = rand_string(64)
    assert set(s) <= set("0123456789abcdefghijklmnopqrstuvwxyz")
    assert rand_string(16) != rand_string(16)
    assert pformat("as-is") == "as-is"
    obj = {"status": {"conditions": [{"type": "Running", "status": "True"}]}}
    assert json.loads(pformat(obj)) == obj and "\n  " in pformat(obj)


def test_bench_contract_cli_and_graph_chunking():
    """bench.py (driver contract): defaults are N=1 with a K/W that finish in seconds, and the
    timed graph's size always divides K (exactly K steps are timed) -- independent of W, which
    runs on a separate one-step graph; K <= 250 is a single replay."""
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location(
        "bench_mod", os.path.join(os.path.dirname(os.path.dirname(__file__)), "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    a = bench.parse_args([])
    assert a.gpus == 1 and a.steps > 0 and a.warmup >= 0
    assert a.launch == "stream"  # measured default (profiles/r2_launch_ab.json); graph kept for A/B
    for k, w in [(2000, 50), (4000, 100), (100, 10), (7, 3), (5, 1), (30, 0), (1, 1), (1009, 5), (251, 0)]:
        spg = bench.pick_steps_per_graph(k, w)
        assert k % spg == 0 and 1 <= spg <= 250
        assert spg <= w or not any(k % d == 0 for d in range(1, min(w, 250) + 1)) or w == 0
    assert bench.pick_steps_per_graph(20, 5) == 5     # the driver's K/W: warm-up replays it once
    assert bench.pick_steps_per_graph(2000, 50) == 50
    assert bench.pick_steps_per_graph(2000, 0) == 250
    assert bench.pick_steps_per_graph(1009, 5) == 1


def test_train_ckpt_interrupted_save_keeps_previous_checkpoint(tmp_path):
    """a save that dies after writing some files of step N+k must leave the step-N
    checkpoint loadable and unmixed (files go to step_<N>/, the meta.json pointer moves last)."""
    import torch.nn as nn
    from pytorch_operator_amd.utils import train_ckpt
    torch.manual_seed(0)
    m = nn.Linear(4, 3)
    opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9)
    m(torch.randn(2, 4)).sum().backward()
    opt.step()
    d = str(tmp_path / "ck")
    train_ckpt.save(d, 5, m, opt, rank=0, world=1)
    w5 = m.weight.detach().clone()
    # a later save that crashed after model.pt: its directory exists, the pointer did not move
    with torch.no_grad():
        m.weight.add_(1.0)
    os.makedirs(os.path.join(d, "step_9"))
    torch.save({k: v.clone() for k, v in m.state_dict().items()}, os.path.join(d, "step_9", "model.pt"))
    m2 = nn.Linear(4, 3)
    opt2 = torch.optim.SGD(m2.parameters(), lr=0.1, momentum=0.9)
    assert train_ckpt.load(d, m2, opt2, rank=0, world=1, device="cpu") == 5
    assert torch.equal(m2.weight, w5)
    # the next complete save moves the pointer and prunes all but the newest `keep`
    for st in (10, 11, 12):
        train_ckpt.save(d, st, m, opt, rank=0, world=1, keep=2)
    assert sorted(os.listdir(d)) == ["meta.json", "step_11", "step_12"]
    assert train_ckpt.load(d, m2, opt2, rank=0, world=1, device="cpu") == 12
    assert torch.equal(m2.weight, m.weight)


def test_train_ckpt_resume_after_crash_keeps_the_fallback(tmp_path):
    """resume from step_5 with a dead (incomplete) step_9 left behind, then save 6:
    the complete step_5 stays as the fallback and the partial step_9 is pruned."""
    import torch.nn as nn
    from pytorch_operator_amd.utils import train_ckpt
    torch.manual_seed(0)
    m = nn.Linear(4, 3)
    opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9)
    d = str(tmp_path / "ck")
    train_ckpt.save(d, 5, m, opt, rank=0, world=1, keep=2)
    os.makedirs(os.path.join(d, "step_9"))  # crashed save: files partly written, pointer never moved
    assert train_ckpt.load(d, m, opt, rank=0, world=1, device="cpu") == 5
    train_ckpt.save(d, 6, m, opt, rank=0, world=1, keep=2)
    assert sorted(os.listdir(d)) == ["meta.json", "step_5", "step_6"]
    with open(os.path.join(d, "meta.json")) as f:
        assert json.load(f)["complete"] == ["step_5", "step_6"]


def test_flat_grad_allreduce_forced_at_world1_gloo():
    """FlatGradAllReduce at world 1: inactive by default, all-reduces issued when forced on a
    single-rank group (init_from_env(force_pg=True)); force without a group is an error."""
    import torch
    import torch.distributed as dist
    from pytorch_operator_amd.parallel.ddp import FlatGradAllReduce
    from pytorch_operator_amd.parallel.dist import init_from_env
    assert not dist.is_initialized()
    with pytest.raises(RuntimeError):
        FlatGradAllReduce(force=True)
    saved = {k: os.environ.pop(k, None) for k in ("WORLD_SIZE", "RANK", "MASTER_ADDR", "MASTER_PORT")}
    try:
        env = init_from_env("gloo", use_gpu=False, force_pg=True)
        assert dist.is_initialized() and env.world_size == 1
        off, on = FlatGradAllReduce(), FlatGradAllReduce(force=True)
        assert not off.active and on.active
        t = torch.arange(6, dtype=torch.float32)
        for s in (off, on):
            s.fc_ready(t[3:])
            s.conv_ready(t[:3])
            assert s.finish() == 1.0
        assert off.issued == 0 and on.issued == 2
        assert torch.equal(t, torch.arange(6, dtype=torch.float32))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()
        for k, v in saved.items():
            os.environ.pop(k, None)
            if v is not None:
                os.environ[k] = v


def test_worker_pins_device_kernel_arguments():
    """The operator-deployed worker pins device-memory kernel arguments before HIP can start
    (bench.py pins the same; profiles/r5_env/ab.txt), unless the pod's env chose otherwise."""
    import subprocess
    import sys
    code = ("import os, sys; import pytorch_operator_amd.harness.mnist; "
            "print(os.environ.get('HIP_FORCE_DEV_KERNARG'), 'torch.cuda' in sys.modules and "
            "__import__('torch').cuda.is_initialized())")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k != "HIP_FORCE_DEV_KERNARG"}
    env["PYTHONPATH"] = root
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0 and r.stdout.split() == ["1", "False"], r.stdout + r.stderr
    env["HIP_FORCE_DEV_KERNARG"] = "0"
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=120)
    assert r.stdout.split()[0] == "0", r.stdout + r.stderr
