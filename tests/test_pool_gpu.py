"""Stem max-pool HIP kernels (csrc/kernels/pool.hip) vs PyTorch fp32 max_pool2d(3, 2, 1)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _x(N, C, H, W, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.randn(N, C, H, W, generator=g).to(torch.bfloat16)
    return x.cuda().to(memory_format=torch.channels_last)


@pytest.mark.parametrize("shape", [(4, 64, 112, 112), (3, 8, 7, 9), (2, 16, 10, 10), (1, 24, 5, 6)])
def test_maxpool_fwd_bwd_matches_fp32_reference(shape):
    from pytorch_operator_amd.ops import _native
    from pytorch_operator_amd.ops.pool import _MaxPool, supported
    _native.load()
    x = _x(*shape)
    assert supported(x)
    xh = x.detach().clone().requires_grad_(True)
    y = _MaxPool.apply(xh)
    xr = x.float().detach().requires_grad_(True)
    yr = F.max_pool2d(xr, 3, 2, 1)
    assert y.shape == yr.shape and y.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(y.float(), yr)  # a max is exact
    dy = torch.randn(y.shape, generator=torch.Generator().manual_seed(1)).to(torch.bfloat16).cuda()
    dy = dy.to(memory_format=torch.channels_last)
    y.backward(dy)
    yr.backward(dy.float())
    # fp32 sum of <= 4 bf16 terms, rounded once: equal to the fp32 reference rounded to bf16
    assert torch.equal(xh.grad.float(), xr.grad.to(torch.bfloat16).float())


def test_maxpool_ties_and_nan_follow_pytorch():
    from pytorch_operator_amd.ops.pool import _MaxPool
    x = torch.zeros(1, 8, 6, 6, dtype=torch.bfloat16).cuda().to(memory_format=torch.channels_last)
    x[0, 1, 2, 2] = float("nan")
    x[0, 2, 0, 0] = -1.0
    xh = x.clone().requires_grad_(True)
    y = _MaxPool.apply(xh)
    ref = F.max_pool2d(x.float(), 3, 2, 1, return_indices=True)
    assert torch.equal(torch.isnan(y.float()), torch.isnan(ref[0]))
    assert torch.equal(torch.nan_to_num(y.float()), torch.nan_to_num(ref[0]))
    dy = torch.ones_like(y)
    y.backward(dy)
    xr = x.float().requires_grad_(True)
    F.max_pool2d(xr, 3, 2, 1).backward(dy.float())
    assert torch.equal(xh.grad.float(), xr.grad)  # all-zero windows: the first tap wins, as in PyTorch


def test_resnet_stem_uses_hip_pool():
    from pytorch_operator_amd.models.resnet import resnet_tiny
    from pytorch_operator_amd.ops.pool import MaxPool3x3s2
    m = resnet_tiny()
    assert isinstance(m.maxpool, MaxPool3x3s2) and m.maxpool.impl == "hip"
