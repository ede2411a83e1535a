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
