"""Max-pool module on CPU: PyTorch's op (the reference path of MaxPool3x3s2)."""
import torch
import torch.nn.functional as F

from pytorch_operator_amd.ops.pool import MaxPool3x3s2, supported


def test_maxpool_module_cpu_equals_torch():
    x = torch.randn(2, 8, 9, 9)
    m = MaxPool3x3s2()
    assert not supported(x)
    assert torch.equal(m(x), F.max_pool2d(x, 3, 2, 1))
