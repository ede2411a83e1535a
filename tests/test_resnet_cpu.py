"""CPU: the ResNet worker's 1x1-convolution-as-GEMM path equals nn.Conv2d (fwd and bwd)."""
import pytest
import torch


@pytest.mark.parametrize("stride", [1, 2])
@pytest.mark.parametrize("hw", [7, 9])
def test_conv1x1_gemm_matches_conv2d(stride, hw):
    from pytorch_operator_amd.models.resnet import Conv1x1
    torch.manual_seed(0)
    c = Conv1x1(16, 24, stride=stride)
    x = torch.randn(3, 16, hw, hw).to(memory_format=torch.channels_last).requires_grad_(True)
    y = c(x)
    assert y.is_contiguous(memory_format=torch.channels_last)
    xr = x.detach().clone().requires_grad_(True)
    wr = c.weight.detach().clone().requires_grad_(True)
    yr = torch.nn.functional.conv2d(xr, wr, stride=stride)
    torch.testing.assert_close(y, yr, rtol=1e-5, atol=1e-5)
    g = torch.randn_like(yr)
    y.backward(g)
    yr.backward(g)
    torch.testing.assert_close(x.grad, xr.grad, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(c.weight.grad, wr.grad, rtol=1e-4, atol=1e-4)


def test_resnet_tiny_gemm_and_library_conv1x1_agree():
    from pytorch_operator_amd.models.resnet import resnet_tiny, set_bn_impl, set_conv1x1_impl
    torch.manual_seed(1)
    a = set_bn_impl(resnet_tiny(), "library")
    b = set_bn_impl(resnet_tiny(), "library")
    b.load_state_dict(a.state_dict())
    set_conv1x1_impl(a, "gemm")
    set_conv1x1_impl(b, "library")
    a, b = a.to(memory_format=torch.channels_last), b.to(memory_format=torch.channels_last)
    x = torch.randn(2, 3, 32, 32).to(memory_format=torch.channels_last)
    la, lb = a(x).square().mean(), b(x).square().mean()
    la.backward()
    lb.backward()
    torch.testing.assert_close(la, lb, rtol=1e-5, atol=1e-6)
    for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
        torch.testing.assert_close(pa.grad, pb.grad, rtol=1e-4, atol=1e-5, msg=n)


def test_link_tap_routes_the_gradient_to_the_link():
    """link_tap: with an unclaimed link the second consumer's gradient lands in link.dz (for the
    producer's backward) instead of autograd; without one it is the identity."""
    from pytorch_operator_amd.ops.batchnorm import GradLink, link_tap
    x = torch.randn(2, 3, requires_grad=True)
    y = x * 1.0
    assert link_tap(y) is y  # no link: autograd path
    y._pto_link = GradLink()
    t = link_tap(y)
    assert t is not y and y._pto_link.claimed
    assert link_tap(y) is y  # claimed once only
    g = torch.randn(2, 3)
    (t * g).sum().backward()
    torch.testing.assert_close(y._pto_link.dz, g)
    assert x.grad is None or float(x.grad.abs().sum()) == 0.0
