"""The HIP trainer pinned to torch itself -- not to an earlier HIP variant.

* The exact bench configuration (``GraphedStep(launch="stream")``, next-batch staging,
  ``conv_chunk`` 4, the head fused into ``fc1_bwd_head``, dW_fc1 / dW_fc2 + SGD in the tail)
  against ``Net`` + ``torch.optim.SGD(lr=0.01, momentum=0.5)`` in fp32 for 24 steps on the same
  batches: parameters and momentum buffers (reference: examples/mnist/mnist.py:35-49,140).
* Two ranks (sharing GPU 0 over gloo) with both gradient paths -- the two-bucket
  ``FlatGradAllReduce`` and the xGMI ``XgmiGradSync`` -- against
  ``torch.nn.parallel.DistributedDataParallel(Net())`` + SGD on the same per-rank batches,
  including the rank-0 broadcast at start (reference: examples/mnist/mnist.py:135-140;
  ``tools/ddp_parity.py``).

Both run torch's net as ``DecisionAlignedNet``: the HIP step's pool argmaxes and ReLU masks, every
value torch's own.  Without that, a single decision within fp32 rounding (a near-tied pool window,
a ReLU input ~1e-7 from 0) that the two summation orders resolve differently sends the two
trajectories apart: unaligned, the two-rank run differed by 3e-4 in parameters and 4 % in fc1's
momentum after 12 steps, while steps 1-3 agreed to 1e-7 (tools/dbg/grad_diag.py).
"""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def test_bench_configuration_matches_torch_sgd_over_24_steps():
    """24 steps of the bench's runner, one ``run(1)`` at a time (the same recorded kernel list
    the bench launches) so that each step's discontinuous decisions -- pool argmax codes and ReLU
    masks -- can be handed to the torch side (``DecisionAlignedNet``: a pool window whose top two
    values, or a ReLU input, within fp32 rounding of each other / of 0 may otherwise go either way
    and the trajectories part); ``decision_gap`` checks every HIP decision is torch's own up to
    rounding."""
    from pytorch_operator_amd.data.synthetic import make_synthetic_mnist
    from pytorch_operator_amd.models.mnist import DecisionAlignedNet, FusedMnistTrainer, _views, reference_init
    from pytorch_operator_amd.ops import mnist as K
    from pytorch_operator_amd.parallel.graphed_step import GraphedStep
    dev = torch.device("cuda")
    B, n = 64, 4096  # 64 batches: no epoch wrap inside the steps taken
    ds = make_synthetic_mnist(n, seed=5, device=dev)
    cursor = torch.zeros(1, dtype=torch.int32, device=dev)
    src = K.BatchSource(ds.images, ds.labels, perm=ds.perm, cursor=cursor)
    tr = FusedMnistTrainer(batch_size=B, source=src, lr=0.01, momentum=0.5, device=dev, seed=1)
    # the bench's knobs, spelled out (bench.py defaults)
    tr.fuse_conv12, tr.conv_chunk, tr.stage_batches = True, 4, True
    assert tr.w1_tail and tr.fuse_head and tr.fc1_ks == 2 and tr.stage is not None
    runner = GraphedStep(tr, mode="graph", steps_per_graph=1, launch="stream")
    assert runner.launch == "stream" and runner.internal_steps == 0
    codes = []
    for _ in range(24):
        runner.run(1)
        torch.cuda.synchronize()
        codes.append((tr.idx1[:B].cpu(), tr.idx2[:B].cpu(), (tr.a1[:B] > 0).cpu(), (tr.a2[:B] > 0).cpu(),
                          (tr.h1[:B] > 0).cpu()))
    steps = int(cursor.item())
    assert steps == 24

    net = DecisionAlignedNet()
    net.load_state_dict(reference_init(1))
    opt = torch.optim.SGD(net.parameters(), lr=0.01, momentum=0.5)
    xf, lab, perm = ds.float_images().cpu(), ds.labels.long().cpu(), ds.perm.long().cpu()
    losses = []
    for t in range(steps):
        idx = perm[t * B:(t + 1) * B]
        opt.zero_grad(set_to_none=True)
        loss = F.nll_loss(net(xf[idx], *codes[t]), lab[idx])
        loss.backward()
        opt.step()
        losses.append(float(loss.detach()))
    assert losses[-1] < losses[0]  # the trajectory compared is a learning one
    assert net.decision_gap < 1e-5, net.decision_gap
    mom = _views(tr.flat_momentum, tr.layout)
    for name, prm in net.named_parameters():
        ep = _rel(tr.params[name], prm.data)
        em = _rel(mom[name], opt.state[prm]["momentum_buffer"])
        assert ep < 1e-4 and em < 1e-4, (name, ep, em)
    # the statistics slot holds the last step's loss (the tail's fused NLL)
    assert abs(tr.loss() - losses[-1]) < 1e-4 * max(1.0, abs(losses[-1])), (tr.loss(), losses[-1])


def test_gradient_contract_of_the_step_forms():
    """The default step keeps the fc gradients in registers: ``grads`` refuses to hand out the
    stale buffer; materialize_fc1_grad (or forward_backward) stores them, and they match torch."""
    from pytorch_operator_amd.models.mnist import FusedMnistTrainer, Net, reference_init
    from pytorch_operator_amd.ops import mnist as K
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(3)
    x = torch.randint(0, 256, (64, 784), generator=g, dtype=torch.uint8)
    y = torch.randint(0, 10, (64,), generator=g, dtype=torch.int32)
    src = K.BatchSource(x.to(dev), y.to(dev))
    tr = FusedMnistTrainer(batch_size=64, source=src, seed=2)
    tr.train_step(advance_cursor=False)
    with pytest.raises(RuntimeError, match="fc1.weight"):
        tr.grads
    tr2 = FusedMnistTrainer(batch_size=64, source=src, seed=2)
    tr2.materialize_fc1_grad = True
    tr2.train_step(advance_cursor=False)
    torch.cuda.synchronize()
    net = Net()
    net.load_state_dict(reference_init(2))
    F.nll_loss(net(((x.float() / 255.0 - 0.1307) / 0.3081).view(-1, 1, 28, 28)), y.long()).backward()
    for name, prm in net.named_parameters():
        assert _rel(tr2.grads[name], prm.grad) < 2e-4, name
    tr.forward_backward()
    assert set(tr.grads) == {n for n, _ in net.named_parameters()}


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.timeout(300)
def test_two_ranks_match_torch_ddp():
    env = dict(os.environ, PYTHONPATH=str(ROOT), PTO_XGMI_ANY_BACKEND="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), str(ROOT / "tools" / "ddp_parity.py"),
           "--steps", "12"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=280, cwd=ROOT, env=env)
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert lines, r.stdout[-3000:] + r.stderr[-3000:]
    res = lines[-1]
    rec = os.environ.get("PTO_TEST_RECORD_DIR")
    if rec:
        Path(rec).mkdir(parents=True, exist_ok=True)
        (Path(rec) / "ddp_parity_w2.json").write_text(json.dumps(res))
    assert r.returncode == 0 and res["all_ok"], res
    assert res["rccl"]["steps"] >= 10 and res["xgmi"]["steps"] >= 10, res
    w = res["worst_over_ranks"]
    assert w["rccl_param_rel"] < 1e-4 and w["rccl_momentum_rel"] < 1e-4 and w["xgmi_param_rel"] < 1e-4, w
    assert w["rccl_decision_gap"] < 1e-5 and w["xgmi_decision_gap"] < 1e-5, w
