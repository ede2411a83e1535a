"""ResNet-50 for the BASELINE "ResNet-50 DDP bf16" PyTorchJob config.

Not part of the reference (its only workload is MNIST); BASELINE.json lists it as a
north-star job shape: Master=1 Worker=7, one ``amd.com/gpu`` each, bf16.  The network is
the standard torchvision-style ResNet-50 v1.5 (stride on the 3x3 conv of each
bottleneck), written out here because torchvision is not in this image.  On MI355X it
runs channels-last under bf16 autocast: convolutions go to MIOpen, the classifier GEMM to
hipBLASLt (plain library kernels), while every batch-norm with the ReLU and residual add
around it is one fused HIP op (``ops/batchnorm.py``: ``relu(bn(x) [+ identity])`` in one
statistics + one normalise pass, its backward in one reduction + one dx pass).
``set_bn_impl(model, "library")`` switches back to PyTorch's batch-norm / add / ReLU ops.
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.batchnorm import BatchNormAct2d, link_tap
from ..ops.pool import MaxPool3x3s2


class Conv1x1(nn.Conv2d):
    """1x1 convolution that, on channels-last activations, runs as ONE GEMM on hipBLASLt:
    NHWC memory viewed as [N*H*W, Cin] times W^T [Cin, Cout] gives the NHWC output with no
    layout copies (stride 2 first takes the strided subsample).  Its backward is the two
    GEMMs of ``F.linear`` (dX = dY.W, dW = dY^T.X).  Same parameter, init and state dict as
    ``nn.Conv2d``; ``impl = "library"`` (or a non-channels-last input) keeps MIOpen's conv."""

    impl = "library"  # measured: MIOpen 30.5 vs GEMM 47.3 ms/step (profiles/r2_resnet_conv1x1_ab.md)

    def __init__(self, cin: int, cout: int, stride: int = 1):
        super().__init__(cin, cout, 1, stride=stride, bias=False)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.impl != "gemm" or x.dim() != 4 or not x.is_contiguous(memory_format=torch.channels_last):
            return super().forward(x)
        if self.stride[0] != 1:
            x = x[:, :, ::self.stride[0], ::self.stride[1]].contiguous(memory_format=torch.channels_last)
        N, C, H, W = x.shape
        y = F.linear(x.permute(0, 2, 3, 1).reshape(N * H * W, C), self.weight.view(self.out_channels, C))
        return y.view(N, H, W, self.out_channels).permute(0, 3, 1, 2)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes: int, planes: int, stride: int = 1, downsample: Optional[nn.Module] = None):
        super().__init__()
        width = planes
        self.conv1 = Conv1x1(inplanes, width)
        self.bn1 = BatchNormAct2d(width, relu=True)
        self.conv2 = nn.Conv2d(width, width, 3, stride=stride, padding=1, bias=False)
        self.bn2 = BatchNormAct2d(width, relu=True)
        self.conv3 = Conv1x1(width, planes * self.expansion)
        # relu(bn3(.) + identity); its output feeds the next block's conv1 and residual add, whose
        # two gradients bn3's backward sums in-kernel (ops/batchnorm.py GradLink)
        self.bn3 = BatchNormAct2d(planes * self.expansion, relu=True, link_output=True)
        self.downsample = downsample

    tap_downsample = True  # a stage's input gradient from the downsample conv summed in bn3 (link_tap)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.downsample is None:
            idt = x
        else:
            idt = self.downsample(link_tap(x) if self.tap_downsample else x)
        out = self.bn1(self.conv1(x))
        out = self.bn2(self.conv2(out))
        return self.bn3(self.conv3(out), idt)


class ResNet(nn.Module):
    def __init__(self, layers: List[int] = (3, 4, 6, 3), num_classes: int = 1000, width: int = 64):
        super().__init__()
        self.inplanes = width
        self.conv1 = nn.Conv2d(3, width, 7, stride=2, padding=3, bias=False)
        self.bn1 = BatchNormAct2d(width, relu=True)
        self.maxpool = MaxPool3x3s2()  # nn.MaxPool2d(3, 2, 1); HIP kernels for channels-last bf16
        self.layer1 = self._make(width, layers[0])
        self.layer2 = self._make(width * 2, layers[1], stride=2)
        self.layer3 = self._make(width * 4, layers[2], stride=2)
        self.layer4 = self._make(width * 8, layers[3], stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.fc = nn.Linear(width * 8 * Bottleneck.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        for m in self.modules():  # zero-init the last BN of each block (standard trick)
            if isinstance(m, Bottleneck):
                nn.init.zeros_(m.bn3.weight)

    def _make(self, planes: int, blocks: int, stride: int = 1) -> nn.Sequential:
        down = None
        if stride != 1 or self.inplanes != planes * Bottleneck.expansion:
            down = nn.Sequential(Conv1x1(self.inplanes, planes * Bottleneck.expansion, stride=stride),
                                 BatchNormAct2d(planes * Bottleneck.expansion))
        layers = [Bottleneck(self.inplanes, planes, stride, down)]
        self.inplanes = planes * Bottleneck.expansion
        layers += [Bottleneck(self.inplanes, planes) for _ in range(1, blocks)]
        return nn.Sequential(*layers)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = self.maxpool(self.bn1(self.conv1(x)))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(torch.flatten(self.avgpool(x), 1))


def set_bn_impl(model: nn.Module, impl: str) -> nn.Module:
    """``"hip"``: fused HIP batch-norm(+add)(+ReLU) kernels; ``"library"``: PyTorch's ops."""
    if impl not in ("hip", "library"):
        raise ValueError(impl)
    for m in model.modules():
        if isinstance(m, BatchNormAct2d):
            m.impl = impl
    return model


def set_pool_impl(model: nn.Module, impl: str) -> nn.Module:
    """``"hip"``: the stem max-pool on ``csrc/kernels/pool.hip``; ``"library"``: PyTorch's op."""
    if impl not in ("hip", "library"):
        raise ValueError(impl)
    for m in model.modules():
        if isinstance(m, MaxPool3x3s2):
            m.impl = impl
    return model


def set_conv1x1_impl(model: nn.Module, impl: str) -> nn.Module:
    """``"gemm"``: 1x1 convolutions as hipBLASLt GEMMs on the NHWC view; ``"library"``: MIOpen."""
    if impl not in ("gemm", "library"):
        raise ValueError(impl)
    for m in model.modules():
        if isinstance(m, Conv1x1):
            m.impl = impl
    return model


def resnet50(num_classes: int = 1000) -> ResNet:
    return ResNet((3, 4, 6, 3), num_classes)


def resnet_tiny(num_classes: int = 10) -> ResNet:
    """Same topology family, small enough for CPU tests."""
    return ResNet((1, 1, 1, 1), num_classes, width=8)
