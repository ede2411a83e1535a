"""GPU: the fused batch-norm(+residual)(+ReLU) HIP kernels (csrc/kernels/batchnorm.hip) vs an
fp64 PyTorch reference of the same op on the same (dtype-rounded) inputs: output, dx,
dgamma, dbeta, the residual's gradient, running statistics and num_batches_tracked."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

SHAPES = [(2, 64, 7, 5), (8, 2048, 7, 7), (3, 8, 11, 13), (4, 256, 14, 14), (1, 512, 1, 3)]


def _case(shape, dtype, relu, res, seed=0, mean=0.0):
    from pytorch_operator_amd.ops.batchnorm import batch_norm_act
    g = torch.Generator().manual_seed(seed)
    N, C, H, W = shape
    x = (mean + torch.randn(shape, generator=g)).to(dtype)
    z = torch.randn(shape, generator=g).to(dtype) if res else None
    w = 0.5 + torch.rand(C, generator=g)
    b = 0.2 * torch.randn(C, generator=g)
    dy = torch.randn(shape, generator=g).to(dtype)
    rm, rv = 0.1 * torch.randn(C, generator=g), 1 + torch.rand(C, generator=g)

    cl = dict(memory_format=torch.channels_last)
    xg = x.cuda().contiguous(**cl).requires_grad_(True)
    zg = z.cuda().contiguous(**cl).requires_grad_(True) if res else None
    wg, bg = w.cuda().requires_grad_(True), b.cuda().requires_grad_(True)
    rmg, rvg, nbt = rm.cuda(), rv.cuda(), torch.zeros((), dtype=torch.long, device="cuda")
    y = batch_norm_act(xg, wg, bg, rmg, rvg, nbt, True, 0.1, 1e-5, relu, zg, impl="hip")
    y.backward(dy.cuda().contiguous(**cl))

    xr = x.double().requires_grad_(True)
    zr = z.double().requires_grad_(True) if res else None
    wr, br = w.double().requires_grad_(True), b.double().requires_grad_(True)
    rmr, rvr = rm.double(), rv.double()
    yr = F.batch_norm(xr, rmr, rvr, wr, br, True, 0.1, 1e-5)
    if res:
        yr = yr + zr
    if relu:
        yr = F.relu(yr)
    yr.backward(dy.double())
    return dict(y=(y, yr), dx=(xg.grad, xr.grad), dw=(wg.grad, wr.grad), db=(bg.grad, br.grad),
                dz=(zg.grad, zr.grad) if res else None, rm=(rmg, rmr), rv=(rvg, rvr), nbt=nbt, y_dtype=y.dtype)


def _close(pair, rtol, atol, what):
    a, r = pair
    torch.testing.assert_close(a.detach().cpu().double(), r.detach().double(), rtol=rtol, atol=atol, msg=what)


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["fp32", "bf16"])
@pytest.mark.parametrize("relu,res", [(False, False), (True, False), (True, True), (False, True)],
                         ids=["bn", "bn_relu", "bn_add_relu", "bn_add"])
def test_fused_batchnorm_matches_fp64(shape, dtype, relu, res):
    r = _case(shape, dtype, relu, res)
    assert r["y_dtype"] == dtype
    # outputs are rounded to the activation dtype once; reductions are fp32
    t = dict(rtol=1e-4, atol=1e-4) if dtype == torch.float32 else dict(rtol=1.6e-2, atol=1.6e-2)
    _close(r["y"], what="y", **t)
    _close(r["dx"], what="dx", **t)
    if res:
        _close(r["dz"], what="dz", **t)
    _close(r["dw"], rtol=1e-3, atol=1e-3, what="dgamma")
    _close(r["db"], rtol=1e-3, atol=1e-3, what="dbeta")
    _close(r["rm"], rtol=1e-5, atol=1e-5, what="running_mean")
    _close(r["rv"], rtol=1e-4, atol=1e-5, what="running_var")
    assert int(r["nbt"]) == 1


def test_statistics_stay_accurate_with_a_large_mean():
    """Shifted sums + Chan merges: mean 1000, unit variance -- a naive E[x^2] - E[x]^2 in fp32
    would lose the variance entirely."""
    r = _case((16, 64, 28, 28), torch.float32, False, False, seed=4, mean=1000.0)
    _close(r["rv"], rtol=2e-4, atol=1e-5, what="running_var")
    _close(r["y"], rtol=1e-3, atol=1e-3, what="y")
    _close(r["dx"], rtol=1e-3, atol=1e-3, what="dx")


def test_module_matches_library_module_and_is_deterministic():
    from pytorch_operator_amd.ops.batchnorm import BatchNormAct2d
    torch.manual_seed(0)
    m = BatchNormAct2d(256, relu=True).cuda()
    ref = torch.nn.BatchNorm2d(256).cuda()
    ref.load_state_dict(m.state_dict())
    x = torch.randn(8, 256, 14, 14, device="cuda").to(memory_format=torch.channels_last)
    outs = []
    for _ in range(2):
        xx = x.clone().requires_grad_(True)
        y = m(xx)
        y.square().sum().backward()
        outs.append((y.detach().clone(), xx.grad.clone(), m.weight.grad.clone()))
        m.weight.grad = None
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b)  # fixed-order reductions: bitwise repeatable
    xr = x.clone().requires_grad_(True)
    yr = torch.relu(ref(xr))
    yr.square().sum().backward()
    torch.testing.assert_close(outs[0][0], yr, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(outs[0][1], xr.grad, rtol=1e-3, atol=1e-4)
    torch.testing.assert_close(outs[0][2], ref.weight.grad, rtol=1e-3, atol=1e-3)
    assert int(m.num_batches_tracked) == 2 and int(ref.num_batches_tracked) == 1


def _chain(dtype, link, seed=0, C=64, shape=(4, 64, 9, 7)):
    """Two bottleneck-style BNs: y1 = relu(bn1(x1)) [producer], y2 = relu(bn2(h(y1)) + y1)
    [consumer: y1 feeds both a 1x1 mixing 'conv' h and the residual add]; loss = <y2, dy>."""
    from pytorch_operator_amd.ops.batchnorm import batch_norm_act
    g = torch.Generator().manual_seed(seed)
    x1 = torch.randn(shape, generator=g).to(dtype)
    wm = (torch.randn(C, C, generator=g) / C ** 0.5).to(dtype)
    w1, b1 = 0.5 + torch.rand(C, generator=g), 0.2 * torch.randn(C, generator=g)
    w2, b2 = 0.5 + torch.rand(C, generator=g), 0.2 * torch.randn(C, generator=g)
    dy = torch.randn(shape, generator=g).to(dtype)
    cl = dict(memory_format=torch.channels_last)

    def h(y, w):
        return torch.einsum("nchw,dc->ndhw", y, w).contiguous(**cl)

    xg = x1.cuda().contiguous(**cl).requires_grad_(True)
    p = [t.cuda().requires_grad_(True) for t in (w1, b1, w2, b2)]
    y1 = batch_norm_act(xg, p[0], p[1], relu=True, impl="hip", link_output=link)
    y2 = batch_norm_act(h(y1, wm.cuda()), p[2], p[3], relu=True, residual=y1, impl="hip")
    y2.backward(dy.cuda().contiguous(**cl))
    got = [xg.grad] + [t.grad for t in p]

    xr = x1.double().requires_grad_(True)
    pr = [t.double().requires_grad_(True) for t in (w1, b1, w2, b2)]
    y1r = F.relu(F.batch_norm(xr, None, None, pr[0], pr[1], True, 0.1, 1e-5))
    y2r = F.relu(F.batch_norm(h(y1r, wm.double()), None, None, pr[2], pr[3], True, 0.1, 1e-5) + y1r)
    y2r.backward(dy.double())
    return got, [xr.grad] + [t.grad for t in pr], y1


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["fp32", "bf16"])
def test_residual_gradient_summed_in_bn_backward_matches_fp64(dtype):
    """GradLink: the consumer BN hands the residual gradient to the producer BN, whose backward
    sums it with the conv-branch gradient in-kernel (fp32) -- dx and every dgamma/dbeta match
    an fp64 autograd reference, the link was claimed and drained, and the result agrees with
    the unfused path (autograd's own gradient sum)."""
    got, ref, y1 = _chain(dtype, link=True)
    assert y1._pto_link.claimed and y1._pto_link.dz is None
    unfused, _, y1u = _chain(dtype, link=False)
    assert getattr(y1u, "_pto_link", None) is None
    names = ["dx", "dgamma1", "dbeta1", "dgamma2", "dbeta2"]

    def rel(a, r):
        a, r = a.detach().cpu().double(), r.double()
        return float((a - r).norm() / r.norm().clamp_min(1e-30))

    for name, a, u, r in zip(names, got, unfused, ref):
        ea, eu = rel(a, r), rel(u, r)
        if dtype == torch.float32:
            assert ea < 2e-5, (name, ea, eu)
        else:
            # bf16 activations: both paths round y1, h(y1) and the gradients to bf16; the fused
            # fp32 sum must be no less accurate than autograd's bf16 sum (vs fp64)
            assert ea < 2e-2 and ea <= 1.05 * eu + 1e-4, (name, ea, eu)


def test_resnet_blocks_claim_links():
    """In the ResNet every identity bottleneck's residual comes from the previous bn3 through a
    link (12 of ResNet-50's 16 blocks), and a stage's first (downsample) block taps the previous
    bn3's link for its downsample conv's input gradient (3 more); only the last bn3 (feeding the
    pooling head) has no second consumer."""
    from pytorch_operator_amd.models.resnet import ResNet
    m = ResNet((2, 2, 1, 1), num_classes=10, width=8).cuda().to(memory_format=torch.channels_last)
    x = torch.randn(2, 3, 32, 32, device="cuda").to(memory_format=torch.channels_last)
    links = []
    hook = lambda mod, inp, out: links.append(getattr(out, "_pto_link", None))  # noqa: E731
    hs = [b.bn3.register_forward_hook(hook) for b in m.modules() if hasattr(b, "bn3")]
    out = m(x)
    out.sum().backward()
    for h in hs:
        h.remove()
    assert len(links) == 6 and all(lk is not None for lk in links)
    # blocks 2 of layer1 / layer2 take their residual from the previous block's bn3; the first
    # blocks of layer2-4 tap it for the downsample conv
    assert [lk.claimed for lk in links] == [True, True, True, True, True, False]
    assert all(lk.dz is None for lk in links)


def _tap_chain(dtype, tap, seed=1, C=64, shape=(4, 64, 9, 7)):
    """Stage-entry shape: y1 = relu(bn1(x)) [producer] feeds two 1x1 'convs' -- ha (conv1,
    through autograd) and hb (downsample, through ``link_tap`` when ``tap``); loss =
    <relu(bn2(ha(y1))), dy> + <bn3(hb(y1)), dz>."""
    from pytorch_operator_amd.ops.batchnorm import batch_norm_act, link_tap
    g = torch.Generator().manual_seed(seed)
    x1 = torch.randn(shape, generator=g).to(dtype)
    wa = (torch.randn(C, C, generator=g) / C ** 0.5).to(dtype)
    wb = (torch.randn(C, C, generator=g) / C ** 0.5).to(dtype)
    ps = [0.5 + torch.rand(C, generator=g) if i % 2 == 0 else 0.2 * torch.randn(C, generator=g) for i in range(6)]
    dy = torch.randn(shape, generator=g).to(dtype)
    dz = torch.randn(shape, generator=g).to(dtype)
    cl = dict(memory_format=torch.channels_last)

    def h(y, w):
        return torch.einsum("nchw,dc->ndhw", y, w).contiguous(**cl)

    xg = x1.cuda().contiguous(**cl).requires_grad_(True)
    p = [t.cuda().requires_grad_(True) for t in ps]
    y1 = batch_norm_act(xg, p[0], p[1], relu=True, impl="hip", link_output=True)
    ya = batch_norm_act(h(y1, wa.cuda()), p[2], p[3], relu=True, impl="hip")
    yb = batch_norm_act(h(link_tap(y1) if tap else y1, wb.cuda()), p[4], p[5], impl="hip")
    ((ya.float() * dy.cuda().float()).sum() + (yb.float() * dz.cuda().float()).sum()).backward()
    got = [xg.grad] + [t.grad for t in p]

    xr = x1.double().requires_grad_(True)
    pr = [t.double().requires_grad_(True) for t in ps]
    y1r = F.relu(F.batch_norm(xr, None, None, pr[0], pr[1], True, 0.1, 1e-5))
    yar = F.relu(F.batch_norm(h(y1r, wa.double()), None, None, pr[2], pr[3], True, 0.1, 1e-5))
    ybr = F.batch_norm(h(y1r, wb.double()), None, None, pr[4], pr[5], True, 0.1, 1e-5)
    ((yar * dy.double()).sum() + (ybr * dz.double()).sum()).backward()
    return got, [xr.grad] + [t.grad for t in pr], y1


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["fp32", "bf16"])
def test_downsample_tap_gradient_summed_in_bn_backward_matches_fp64(dtype):
    """link_tap: the second conv consumer's input gradient reaches the producer BN through its
    link and is summed in-kernel -- x / gamma / beta gradients match fp64 autograd and are no
    less accurate than autograd's own sum (the untapped run)."""
    got, ref, y1 = _tap_chain(dtype, tap=True)
    assert y1._pto_link.claimed and y1._pto_link.dz is None
    unfused, _, y1u = _tap_chain(dtype, tap=False)
    assert not y1u._pto_link.claimed

    def rel(a, r):
        a, r = a.detach().cpu().double(), r.double()
        return float((a - r).norm() / r.norm().clamp_min(1e-30))

    for name, a, u, r in zip(["dx", "dg1", "db1", "dg2", "db2", "dg3", "db3"], got, unfused, ref):
        ea, eu = rel(a, r), rel(u, r)
        if dtype == torch.float32:
            assert ea < 2e-5, (name, ea, eu)
        else:
            # bf16 rounding of y1, both conv outputs and the gradients: ~3 % vs fp64 on this
            # chain either way; the fused fp32 sum must be no less accurate than autograd's
            assert ea < 5e-2 and ea <= 1.05 * eu + 1e-4, (name, ea, eu)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["fp32", "bf16"])
def test_relu_mask_bits_match_the_output_mask_bitwise(dtype, monkeypatch):
    """Residual + ReLU: the backward's mask from the forward's 1-bit image (mask mode 3) gives
    bitwise the gradients of the mask re-read from y (mode 2), including values that round to
    zero in bf16."""
    from pytorch_operator_amd.ops import batchnorm as bnm
    g = torch.Generator().manual_seed(3)
    N, C, H, W = 4, 64, 9, 7
    x = torch.randn(N, C, H, W, generator=g).to(dtype)
    z = torch.randn(N, C, H, W, generator=g).to(dtype)
    z[:, :, 0, 0] = 0.0
    w, b = 0.5 + torch.rand(C, generator=g), 0.2 * torch.randn(C, generator=g)
    dy = torch.randn(N, C, H, W, generator=g).to(dtype)
    cl = dict(memory_format=torch.channels_last)
    outs = []
    for bits in (True, False):
        monkeypatch.setattr(bnm, "MASK_BITS", bits)
        xg = x.cuda().contiguous(**cl).requires_grad_(True)
        zg = z.cuda().contiguous(**cl).requires_grad_(True)
        p = [t.cuda().requires_grad_(True) for t in (w, b)]
        y = bnm.batch_norm_act(xg, p[0], p[1], relu=True, residual=zg, impl="hip")
        y.backward(dy.cuda().contiguous(**cl))
        outs.append([y.detach(), xg.grad, zg.grad, p[0].grad, p[1].grad])
    for a, r in zip(*outs):
        assert torch.equal(a, r)
