"""GPU numerics of the ResNet-50 worker (BASELINE "ResNet-50 DDP bf16" job shape).

The worker runs the network through PyTorch-ROCm library kernels (MIOpen convolutions and
batch-norm, hipBLASLt GEMM) in channels-last layout under bf16 autocast, with the conv
algorithm search on.  Reference: the same weights and batch in fp64 on the CPU.  Because
random deep nets amplify rounding differently per tensor, each GPU error is judged against
what PyTorch's own CPU path at the same precision gets on the same inputs (fp32 vs fp32,
bf16 autocast vs bf16 autocast), not against a fixed number.  Plus: a few steps of the
worker's fused SGD must fit a fixed batch.  The network is models/resnet.py; its
last-BN-of-each-block zero init would leave every residual branch without gradient, so the
BN affine weights are randomised first.
"""
import copy

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _net(num_classes=10, seed=0):
    from pytorch_operator_amd.models.resnet import resnet50
    torch.manual_seed(seed)
    net = resnet50(num_classes)
    g = torch.Generator().manual_seed(seed + 1)
    with torch.no_grad():
        for m in net.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.weight.copy_(0.5 + 0.5 * torch.rand(m.weight.shape, generator=g))
                m.bias.copy_(0.1 * torch.randn(m.bias.shape, generator=g))
    return net


def _batch(B=4, H=64, classes=10, seed=3):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(B, 3, H, H, generator=g), torch.randint(0, classes, (B,), generator=g)


def _fwd_bwd(net, x, y, amp=False):
    net.zero_grad(set_to_none=True)
    with torch.autocast(device_type=x.device.type, dtype=torch.bfloat16, enabled=amp):
        out = net(x)
    loss = F.cross_entropy(out.float(), y)
    loss.backward()
    return out.float(), loss, {n: p.grad.float() for n, p in net.named_parameters()}


def _rel(a, b):
    a, b = a.detach().cpu().double(), b.detach().cpu().double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def _flat(g):
    return torch.cat([g[n].flatten().double() for n in sorted(g)])


@pytest.fixture
def algo_search():
    """The worker's setting: MIOpen times every algorithm per shape and keeps the fastest."""
    old = torch.backends.cudnn.benchmark
    torch.backends.cudnn.benchmark = True
    yield
    torch.backends.cudnn.benchmark = old


@pytest.fixture
def full_fp32_convs():
    """fp32 checks pin MIOpen to its default (non-searched) fp32 algorithms with TF32-style
    shortcuts off: the search may pick a faster algorithm whose fp32 is ~1e-3 accurate (seen
    once in layer1: 1.2e-3 vs 1e-6 on CPU), which is MIOpen's business, not this stack's."""
    old = torch.backends.cudnn.benchmark, torch.backends.cudnn.allow_tf32, torch.backends.cudnn.deterministic
    torch.backends.cudnn.benchmark, torch.backends.cudnn.allow_tf32 = False, False
    torch.backends.cudnn.deterministic = True
    yield
    torch.backends.cudnn.benchmark, torch.backends.cudnn.allow_tf32, torch.backends.cudnn.deterministic = old


def _errors(bn_train, amp, B=8, H=64):
    """Per-tensor relative gradient errors of CPU and GPU runs (same precision) against an fp64
    CPU run, plus logits / flat-gradient errors."""
    ref = _net()
    ref.train(bn_train)
    x, y = _batch(B=B, H=H)
    out64, loss64, g64 = _fwd_bwd(copy.deepcopy(ref).double(), x.double(), y)
    out_c, _, g_c = _fwd_bwd(copy.deepcopy(ref), x, y, amp=amp)
    gpu = copy.deepcopy(ref).cuda().to(memory_format=torch.channels_last)
    out_g, loss_g, g_g = _fwd_bwd(gpu, x.cuda().to(memory_format=torch.channels_last), y.cuda(), amp=amp)
    return dict(out_c=_rel(out_c, out64), out_g=_rel(out_g, out64),
                flat_c=_rel(_flat(g_c), _flat(g64)), flat_g=_rel(_flat(g_g), _flat(g64)),
                per_c={n: _rel(g_c[n], g64[n]) for n in g64}, per_g={n: _rel(g_g[n], g64[n]) for n in g64},
                loss=(float(loss_g.detach()), float(loss64.detach())), gpu=gpu, ref=ref)


def test_resnet50_fp32_matches_fp64_like_cpu_fp32(full_fp32_convs):
    """Inference-mode batch norm (well conditioned): every conv / BN / linear gradient of the
    MIOpen fp32 path is as close to fp64 as PyTorch's CPU fp32 path is (within 5x + 1e-4)."""
    e = _errors(bn_train=False, amp=False)
    assert e["out_g"] < 1e-4 and e["flat_g"] < 1e-3, (e["out_g"], e["flat_g"])
    bad = [(n, e["per_g"][n], e["per_c"][n]) for n in e["per_g"] if e["per_g"][n] > 5 * e["per_c"][n] + 1e-4]
    assert not bad, bad[:5]


def test_resnet50_bf16_autocast_error_is_bf16_sized(algo_search):
    """The worker's bf16 autocast path: logits and the whole gradient vector are as close to
    fp64 as CPU bf16 autocast gets (within 3x), i.e. bf16 rounding, nothing structurally off."""
    e = _errors(bn_train=False, amp=True)
    assert e["out_g"] < max(3 * e["out_c"], 2e-2), (e["out_g"], e["out_c"])
    assert e["flat_g"] < max(3 * e["flat_c"], 0.1), (e["flat_g"], e["flat_c"])
    assert abs(e["loss"][0] - e["loss"][1]) < 2e-2 * e["loss"][1]


def test_resnet50_train_mode_batchnorm_matches_fp64_like_cpu_fp32(full_fp32_convs):
    """Training-mode batch norm over a small batch is ill-conditioned: layer4 normalises 8 x 2 x 2
    values per channel, some channels nearly dead after the ReLU in front, so the last bits of
    the convolutions are amplified into the layer-4 gradients (CPU fp32 itself is 0.1-3 % off
    fp64 there, and on the GPU the same net moves by ~1 % between MIOpen algorithm choices).
    Per-tensor bounds would test that amplification, not this stack, so the train-mode check
    is on the logits, the loss and the whole gradient vector (within 10x of CPU fp32's error)
    plus the running statistics; the fused BN kernels themselves are pinned to fp64 per tensor
    in tests/test_batchnorm_gpu.py, and every tensor of the well-conditioned eval-mode net in
    test_resnet50_fp32_matches_fp64_like_cpu_fp32."""
    e = _errors(bn_train=True, amp=False)
    assert e["out_g"] < 1e-3, e["out_g"]
    assert abs(e["loss"][0] - e["loss"][1]) < 1e-4 * e["loss"][1]
    assert e["flat_g"] < 10 * e["flat_c"] + 1e-4, (e["flat_g"], e["flat_c"])
    ref64 = copy.deepcopy(e["ref"]).double()
    x, y = _batch(B=8, H=64)
    _fwd_bwd(ref64, x.double(), y)  # same batch: running stats of one step
    for (n, b), (_, br) in zip(e["gpu"].named_buffers(), ref64.named_buffers()):
        if b.dtype.is_floating_point:
            assert _rel(b, br) < 1e-3, n


def test_resnet50_bf16_sgd_fits_a_fixed_batch(algo_search):
    """The worker's optimizer (fused SGD, momentum 0.9, wd 1e-4) under bf16 autocast drives the
    loss of one fixed 16-image batch well below chance."""
    net = _net(seed=5).cuda().to(memory_format=torch.channels_last)
    x, y = _batch(B=16, seed=7)
    x, y = x.cuda().to(memory_format=torch.channels_last), y.cuda()
    opt = torch.optim.SGD(net.parameters(), lr=0.02, momentum=0.9, weight_decay=1e-4, fused=True)
    losses = []
    for _ in range(30):
        opt.zero_grad(set_to_none=True)
        with torch.autocast(device_type="cuda", dtype=torch.bfloat16):
            loss = F.cross_entropy(net(x).float(), y)
        loss.backward()
        opt.step()
        losses.append(float(loss))
    assert all(v == v for v in losses), losses
    assert losses[-1] < 0.5 * losses[0] and losses[-1] < 1.0, losses
